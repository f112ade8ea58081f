#!/bin/bash
# C4 fnv1a_64 by placement: keys synthesised first in a fresh process, and
# after holding a 32 GiB spacer (tools/c4_placement.py), twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05_c4_place3}
mkdir -p "$O"
for i in 1 2; do
  timeout -k 10 300 python3 tools/c4_placement.py --rounds 3 > "$O/nospacer_$i.json" 2> "$O/nospacer_$i.err" || exit 1
  timeout -k 10 300 python3 tools/c4_placement.py --rounds 3 --spacer-gib 32 > "$O/spacer_$i.json" 2> "$O/spacer_$i.err" || exit 1
done
echo done
