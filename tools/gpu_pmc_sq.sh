#!/bin/bash
# SQ counter pass per (mode, variant): where do the wave cycles go?
#   tools/gpu_pmc_sq.sh TAG CONFIG MODE "VARIANTS"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcsq}
mkdir -p "$OUT"
CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
for v in ${4:-0}; do
    timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/v$v" -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config ${2:-C2} --mode ${3:-fnv1a_64} --variant 0:0:$v --iters 5 > "$OUT/v$v.log" 2>&1 || exit $?
done
echo done
