#!/bin/bash
# C4 fnv1a_64 / md5 / crc32: the synthesised keys against a copy in
# physically contiguous device memory (tools/c4_placement.py --contig-only),
# three processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05_c4_contig}
mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/c4_placement.py --rounds 3 --contig-only > "$O/fnv_$i.json" 2> "$O/fnv_$i.err" || { tail -5 "$O/fnv_$i.err"; exit 1; }
done
timeout -k 10 300 python3 tools/c4_placement.py --rounds 3 --contig-only --mode md5 > "$O/md5.json" 2> "$O/md5.err" || exit 1
timeout -k 10 300 python3 tools/c4_placement.py --rounds 3 --contig-only --mode crc32 > "$O/crc32.json" 2> "$O/crc32.err" || exit 1
echo done
