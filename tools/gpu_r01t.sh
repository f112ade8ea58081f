#!/bin/bash
# NT-variant screen + A/B sweep + md5/fnv1a SQ counter passes on C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_screen.sh r01t 0:0:64 0:0:96 0:1:64 || exit $?
timeout -k 10 400 python3 tools/sweep.py --modes fnv1a_64,md5 --variants 0:0:0,0:0:32,0:0:64,0:0:96 --rounds 3 \
    > gpurun_out/r01t/sweep.log 2>&1 || exit $?
CFG=C3 MODE=md5 VAR=0:0:0 OUT=gpurun_out/r01t/pmc bash tools/pmc_c3.sh || exit $?
CFG=C3 MODE=fnv1a_64 VAR=0:0:32 OUT=gpurun_out/r01t/pmc bash tools/pmc_c3.sh || exit $?
echo done
