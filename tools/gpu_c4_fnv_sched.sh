#!/bin/bash
# C4 shard fnv1a_64 on the two-lines-per-round kernel: tiles per wave (16 / 8 /
# 32 = policy / 64) and interleaving, twice in one process each, on whatever
# box this lands (the leg runs 1.41-1.44 ms on some boxes, 1.53-1.54 on
# others with the same kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05_c4_fnv_sched}
mkdir -p "$O"
for i in 1 2; do
  timeout -k 10 300 python3 tools/ab.py --configs C4S --modes fnv1a_64 --rounds 5 \
      --variants 15209472,13112320,14160896,16258048,6820864 > "$O/ab_$i.jsonl" 2> "$O/ab_$i.err" || { tail -20 "$O/ab_$i.err"; exit 1; }
done
echo done
