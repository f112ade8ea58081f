#!/bin/bash
# All 12 modes on C3 (BASELINE.json configs[2]): in-process variant sweep,
# rocprofv3 kernel-trace stats, and one FETCH_SIZE / WRITE_SIZE pass each
# (variant 0 = the shape policy's pipeline). First failure ends the script.   usage: tools/gpu_modes.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
MODES=one_at_a_time,md5,crc16,crc32,crc32a,fnv1_64,fnv1a_64,fnv1_32,fnv1a_32,hsieh,murmur,jenkins
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || tail -n 20 "$OUT/$name.log"; return $rc
}
step sweep 500 python3 tools/sweep.py --configs C3 --modes $MODES --variants 0:0:0,0:0:65536,0:0:32,0:0:896,0:1:65536,0:0:524288,0:0:526336 --rounds 3 || exit $?
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o modes --output-format csv -- \
    python3 tools/pmc_run.py --config C3 --mode $MODES --variant 0:0:0 --iters 10 || exit $?
for ctr in FETCH_SIZE WRITE_SIZE; do
    step "pmc_$ctr" 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_$ctr" -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config C3 --mode $MODES --variant 0:0:0 --iters 3 || exit $?
done
echo done
