#!/bin/bash
# The batch ring: device staging (HBM written through the PCIe BAR) against
# host staging, and write-through hashes against plain stores + release
# (the acquire fence against sc0 sc1 fetch loads was r06zd): the ring and
# batch-site tests (both stagings), then the C5 replay and the depth-1
# timeline under each configuration (staging:write-through[:copy[:deep]],
# copy = memcpy|avx2|avx512 for the staging copy, x = 1 for the variant under
# test (r06zo: deep byte readers; r06zq: a batch's keys spread over every
# wave); repeated configs give a paired comparison on one box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06x_bar}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 100 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ring.py tests/test_gpu_batch_site.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
for cfg in ${CONFIGS:-default:1 host:1 default:1 host:1}; do
    IFS=: read -r st wt cp dp <<< "$cfg"
    if [ $st = default ]; then unset NC_GPUHASH_RING_STAGING; else export NC_GPUHASH_RING_STAGING=$st; fi
    export NC_GPUHASH_RING_WT=$wt
    if [ -n "${cp:-}" ]; then export NC_GPUHASH_RING_COPY=$cp; else unset NC_GPUHASH_RING_COPY; fi
    # 4th field: r06zo's deep readers (removed since), now the spread key mapping
    if [ "${dp:-0}" = 1 ]; then export NC_GPUHASH_RING_SPREAD=1; else unset NC_GPUHASH_RING_SPREAD; fi
    n=$(( ${n:-0} + 1 )); tag=${st}_wt${wt}_${cp:-defcopy}_x${dp:-0}_$n
    timeout -k 10 120 tools/nc_c5_replay 1.5 timeline > $O/timeline_$tag.jsonl 2> $O/timeline_$tag.err || { cat $O/timeline_$tag.err; exit 1; }
    echo "$tag $(cat $O/timeline_$tag.jsonl)"
    timeout -k 10 120 tools/nc_c5_replay 0.4 > $O/c5_$tag.jsonl 2> $O/c5_$tag.err || { cat $O/c5_$tag.err; exit 1; }
    grep -E '"host_per_key"|"staging"' $O/c5_$tag.jsonl | sed "s/^/$tag /" | cut -c1-270
done
