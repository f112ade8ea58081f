#!/bin/bash
# round 6: the packed ketama search by aligned pairs (A/B build) against quads,
# C2 server_idx, library A B x 3 on one box, plus the dispatch parity tests
# against the A/B build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06v}; mkdir -p $O
for i in 1 2 3; do
  for lib in twemproxy_amd/libnc_gpuhash.so abl/libnc_kpairs.so; do
    tag=$(basename $lib .so)
    timeout -k 10 300 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --pipes policy,plain_hash \
        --rounds 3 --lib $lib > $O/ab_${tag}_$i.jsonl 2> $O/ab_${tag}_$i.err || { tail -20 $O/ab_${tag}_$i.err; exit 1; }
    echo "$tag $(cat $O/ab_${tag}_$i.jsonl | cut -c1-400)"
  done
done
