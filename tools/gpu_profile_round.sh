#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats of the SAME bench
# command, FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run,
# nothing else traced) for every bench leg's hash kernel (C2 fnv1a_64 / md5 /
# server_idx, C3 fnv1a_64 / crc32 / md5, C4 shard md5 / crc32 / fnv1a_64), the
# end-to-end host batch benchmark and the C5 replay. Every GPU step has its own limit; the first failure ends
# the script.     usage: tools/gpu_profile_round.sh <tag> [bench|pmc]   (default: both;
# the parts fit one gpurun call each)
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

PART=${2:-all}
if [ "$PART" != pmc ]; then
step bench 600 python3 bench.py || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
step rocprof_bench 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
    python3 bench.py || exit $?
grep '^{' "$OUT/rocprof_bench.log" > "$OUT/bench_under_rocprof.json"
fi
[ "$PART" = bench ] && { echo done; exit 0; }
for cm in C2:fnv1a_64 C2:md5 C2:server_idx C3:fnv1a_64 C3:crc32 C3:md5 C4S:md5 C4S:crc32 C4S:fnv1a_64; do
    cfg=${cm%%:*}; mode=${cm#*:}
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step "pmc_${cfg}_${mode}_${ctr}" 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_${cfg}_${mode}_${ctr}" -o pmc \
            --output-format csv -- python3 tools/pmc_run.py --config $cfg --mode $mode --variant 0:0:0 --iters 5 \
            || exit $?
    done
done
step e2e 400 tools/nc_e2e_bench 1.5 || exit $?
grep '^{' "$OUT/e2e.log" > "$OUT/e2e.jsonl"
step c5 300 tools/nc_c5_replay 1.0 || exit $?
grep '^{' "$OUT/c5.log" > "$OUT/c5.jsonl"
echo done
