#!/bin/bash
# round 6: md5's S64 form (keys <= 64 B by the shape) — parity (md5 tests),
# then C2 against the generic whole-line form (bit 14), same process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06s}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "md5 or direct_ragged or full_size or kats" -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes md5 --variants 561152,577536,557056 --rounds 5 --iters 10 \
    > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU -d $O/pmc_valu -o pmc --output-format csv -- \
    python3 tools/pmc_run.py --config C2 --mode md5 --variant 0:0:0 --iters 5 > $O/pmc_valu.log 2>&1 || { tail $O/pmc_valu.log; exit 1; }
echo done
