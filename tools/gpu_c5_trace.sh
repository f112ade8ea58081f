#!/bin/bash
# C5 replay under rocprofv3 kernel + HIP API trace (no counters): per-API
# host cost per batch and the kernel durations, to see what serialises the
# in-flight batches.
#   usage: tools/gpu_c5_trace.sh TAG [seconds-per-point]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 120 tools/nc_c5_replay ${2:-0.3} > $O/c5_plain.jsonl 2> $O/c5_plain.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace -o c5 --output-format csv -- \
    tools/nc_c5_replay ${3:-0.05} > $O/c5_traced.jsonl 2> $O/c5_traced.err || exit $?
find $O/trace -name "*_stats.csv" -exec cp {} $O/ \;
find $O/trace -name "*kernel_trace.csv" -size +20M -delete
find $O/trace -name "*hip_api_trace.csv" -size +40M -delete
ls -la $O
