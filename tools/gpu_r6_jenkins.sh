#!/bin/bash
# round 6: C3 jenkins, the register-staged policy against the short-key kernel
# at sixteen waves per CU (as crc16), with 1 / 2 / 3 tiles in flight
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06j}; mkdir -p $O
timeout -k 10 300 python3 tools/ab.py --configs C3 --modes jenkins --variants 0,530432,1579008,2627584 --rounds 5 --iters 10 \
    > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
