#!/bin/bash
# One rocprofv3 counter pass per counter set, over tools/pmc_run.py.
#   tools/gpu_pmc.sh TAG CONFIG MODE VARIANT "SET1" ["SET2" ...]   (a SET is a space-separated counter list)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; CFG=$2; MODE=$3; VAR=$4; shift 4
mkdir -p "$OUT"
i=0
for set in "$@"; do
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config $CFG --mode $MODE --variant 0:0:$VAR --iters 5 --nkeys ${NKEYS:-0} > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
    i=$((i+1))
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
