#!/bin/bash
# nt-by-default build: parity suite + full-size screen, A/B sweep, md5 SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_screen.sh r01u 0:0:0 0:1:0 0:0:32 || exit $?
timeout -k 10 500 python3 tools/sweep.py --modes fnv1a_64,md5 --variants 0:0:0,0:0:32,0:0:64,0:1:0,0:0:8 --rounds 3 \
    > gpurun_out/r01u/sweep.log 2>&1 || exit $?
CFG=C3 MODE=md5 VAR=0:0:0 OUT=gpurun_out/r01u/pmc bash tools/pmc_c3.sh || exit $?
CFG=C2 MODE=fnv1a_64 VAR=0:0:0 OUT=gpurun_out/r01u/pmc bash tools/pmc_c3.sh || exit $?
echo done
