#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats of the SAME bench
# command, FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run,
# nothing else traced) for C2/C3 x fnv1a_64/md5, and the end-to-end host
# batch benchmark. Every GPU step has its own limit; the first failure ends
# the script.     usage: tools/gpu_profile_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"

step() {  # name limit cmd...
    local name=$1 limit=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    [ $rc -eq 0 ] || tail -n 20 "$OUT/$name.log"
    return $rc
}

step bench 600 python3 bench.py || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
step rocprof_bench 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
    python3 bench.py || exit $?
grep '^{' "$OUT/rocprof_bench.log" > "$OUT/bench_under_rocprof.json"
for cfg in C2 C3; do for mode in fnv1a_64 md5; do for ctr in FETCH_SIZE WRITE_SIZE; do
    step "pmc_${cfg}_${mode}_${ctr}" 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_${cfg}_${mode}_${ctr}" -o pmc \
        --output-format csv -- python3 tools/pmc_run.py --config $cfg --mode $mode --variant 0:0:0 --iters 5 || exit $?
done; done; done
step e2e 400 tools/nc_e2e_bench 1.5 || exit $?
grep '^{' "$OUT/e2e.log" > "$OUT/e2e.jsonl"
echo done
