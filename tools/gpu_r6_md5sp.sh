#!/bin/bash
# round 6: md5 whole-line stores (policy) against its store-policy A/Bs
# (SP 1: tile stores default policy; SP 2: tail stores too), C2, same process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06h}; mkdir -p $O
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes md5 --variants 561152,569344,577536,557056 --rounds 5 --iters 10 \
    > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
for v in 569344 577536; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${v}_WRITE_SIZE -o pmc --output-format csv -- \
      python3 tools/pmc_run.py --config C2 --mode md5 --variant 0:0:$v --iters 5 > $O/pmc_${v}.log 2>&1 || { tail $O/pmc_${v}.log; exit 1; }
done
echo done
