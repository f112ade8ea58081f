#!/bin/bash
# Same-process A/B of the wave-sorted pipeline (variant bit 24) against the
# policy on C2, plus its parity tests.   usage: tools/gpu_wsort_ab.sh <tag>
#   16777216 = wsort (4 tiles/wave), 17825792 = 2 tiles/wave, 18874368 = 8,
#   20971520 = DIAGNOSTIC no-hash build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-wsort}
mkdir -p "$O"
timeout -k 10 120 python3 tools/ws_debug.py 1048576 16777216 > "$O/debug.log" 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes fnv1a_64 --variants 0,16777216,17825792,18874368,20971520 > "$O/c2.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes one_at_a_time,fnv1_32 --variants 0,16777216,17825792 >> "$O/c2.jsonl" 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "wsort or sort_and_grid or corpus" > "$O/pytest.log" 2>&1
