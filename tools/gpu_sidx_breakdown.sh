#!/bin/bash
# Where the fused ketama dispatch's time goes on C2, one box, one process:
# the plain hash of the same keys, server_idx (policy; no search; no hash_tag
# code and no search; the same without the continuum's prologue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/${1:-r05_sidx_breakdown}
mkdir -p "$D"
for i in 1 2; do
  timeout -k 10 200 python -u tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --rounds 5 --pipes plain_hash,policy,diag_nosearch,diag_bare,diag_bare_noprologue > "$D/sidx_$i.jsonl" 2>&1 || exit 1
done
echo done
