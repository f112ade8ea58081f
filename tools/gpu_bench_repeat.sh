#!/bin/bash
# One plain bench.py run per call (a fresh box per call): box-to-box variance
# of the bench line.   usage: tools/gpu_bench_repeat.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > "gpurun_out/$1.log" 2>&1 || { tail -20 "gpurun_out/$1.log"; exit 1; }
grep '^{' "gpurun_out/$1.log" | tail -1 > "gpurun_out/$1.json"
echo done
