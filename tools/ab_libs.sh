#!/bin/bash
# Same-box A/B of library builds: tools/ab.py once per build, the builds in
# turn, twice over (so a clock or thermal drift shows up as a difference
# between the two passes, not between builds). Older builds come from
# `git worktree add /tmp/wt <commit> && make -C /tmp/wt/twemproxy_amd/csrc`
# copied into ab_libs/ (git-ignored).
#   usage: tools/ab_libs.sh <out-tag> "<ab.py args>" lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
ARGS=$2
shift 2
mkdir -p "$OUT"
for pass in 1 2; do
    for lib in "$@"; do
        # shellcheck disable=SC2086
        timeout -k 10 150 python3 -u tools/ab.py --lib "$lib" $ARGS >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
    done
done
grep '^{' "$OUT/ab.log"
