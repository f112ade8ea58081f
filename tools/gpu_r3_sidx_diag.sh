#!/bin/bash
# Round 3 DIAGNOSTIC: what the fused ketama dispatch costs on the grouped
# pipeline (packed LDS continuum) — without the hash_tag code, without the
# search, without both — beside the plain fnv1a_64 hash launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03sidxdiag
mkdir -p "$O"
timeout -k 10 400 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --tags none \
    --pipes ${PIPES:-policy,grouped_5b,diag_notag,diag_nosearch,diag_bare} --rounds 5 > "$O/ab_sidx.jsonl" 2> "$O/ab_sidx.err" \
    || { tail -20 "$O/ab_sidx.err"; exit 1; }
cat "$O/ab_sidx.jsonl"
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes fnv1a_64 --variants 0 --rounds 5 --iters 10 \
    > "$O/ab.jsonl" 2> "$O/ab.err" || { tail -20 "$O/ab.err"; exit 1; }
cat "$O/ab.jsonl"
