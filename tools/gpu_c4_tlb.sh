#!/bin/bash
# C4 fnv1a_64's two modes against translation counters: four placements of
# the same keys in one process (tools/c4_placement.py --grid --keys-only),
# timed, then one PMC pass per counter group over the same sequence
# (PMC_GROUPS: space-separated groups, counters joined by commas; START: first pass number - 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_c4tlb}; mkdir -p $O
timeout -k 10 300 python3 tools/c4_placement.py --grid --keys-only --rounds 1 --iters 5 > $O/plain.json 2> $O/plain.err || exit 1
cat $O/plain.json
i=${START:-0}
GROUPS_DEFAULT="TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_REQUEST_sum,TCP_UTCL1_STALL_MULTI_MISS_sum \
GRBM_UTCL2_BUSY,GRBM_GUI_ACTIVE,TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum,TCP_UTCL1_STALL_INFLIGHT_MAX_sum"
for grp in ${PMC_GROUPS:-$GROUPS_DEFAULT}; do
  ctrs=${grp//,/ }
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs -d $O/pmc$i -o pmc -- python3 tools/c4_placement.py --grid --keys-only --rounds 1 --iters 5 > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
done
echo done
