#!/bin/bash
# round 6: the C4 shard's line kernels with the offsets' default cache policy
# (A/B against nt), md5 / crc32 / fnv1a_64, same process, plus FETCH_SIZE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06k}; mkdir -p $O
for mv in md5:13107200,13115392 crc32:15204352,15204864 fnv1a_64:15209472,15209984; do
  m=${mv%%:*}; v=${mv#*:}
  timeout -k 10 300 python3 tools/ab.py --configs C4S --modes $m --variants $v,$v --rounds 5 --iters 10 \
      > $O/ab_$m.jsonl 2> $O/ab_$m.err || { tail -20 $O/ab_$m.err; exit 1; }
  cat $O/ab_$m.jsonl
  for var in ${v//,/ }; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${m}_${var} -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config C4S --mode $m --variant 0:0:$var --iters 5 > $O/pmc_${m}_${var}.log 2>&1 \
        || { tail $O/pmc_${m}_${var}.log; exit 1; }
  done
done
echo done
