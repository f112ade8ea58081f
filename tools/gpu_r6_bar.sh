#!/bin/bash
# The batch ring: device staging (HBM written through the PCIe BAR) against
# host staging, and the worker's length sort on and off: the ring and
# batch-site tests (both stagings), then the C5 replay and the depth-1
# timeline under each configuration (staging:sort:write-through).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06x_bar}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 100 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ring.py tests/test_gpu_batch_site.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
for cfg in ${CONFIGS:-default:1:0 default:0:0 host:1:0}; do
    IFS=: read -r st so wt <<< "$cfg"
    if [ $st = default ]; then unset NC_GPUHASH_RING_STAGING; else export NC_GPUHASH_RING_STAGING=$st; fi
    export NC_GPUHASH_RING_SORT=$so NC_GPUHASH_RING_WT=$wt
    tag=${st}_sort${so}_wt$wt
    timeout -k 10 120 tools/nc_c5_replay 1.5 timeline > $O/timeline_$tag.jsonl 2> $O/timeline_$tag.err || { cat $O/timeline_$tag.err; exit 1; }
    echo "$tag $(cat $O/timeline_$tag.jsonl)"
    timeout -k 10 120 tools/nc_c5_replay 0.4 > $O/c5_$tag.jsonl 2> $O/c5_$tag.err || { cat $O/c5_$tag.err; exit 1; }
    grep -E '"host_per_key"|"staging"' $O/c5_$tag.jsonl | sed "s/^/$tag /" | cut -c1-270
done
