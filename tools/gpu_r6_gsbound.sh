#!/bin/bash
# round 6: C2 fnv1a_64, the grouped tile's three bound dwords with the default
# cache policy (A/B build abl/libnc_gsbound0.so) against nt: time, then FETCH_SIZE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06m}
bash tools/gpu_ab_libs.sh ${1:-r06m} C2 fnv1a_64 0 twemproxy_amd/libnc_gpuhash.so abl/libnc_gsbound0.so 3 || exit 1
for lib in twemproxy_amd/libnc_gpuhash.so abl/libnc_gsbound0.so; do
  tag=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$tag -o pmc --output-format csv -- \
      python3 tools/pmc_run.py --config C2 --mode fnv1a_64 --variant 0:0:0 --iters 5 --lib $lib > $O/pmc_$tag.log 2>&1 \
      || { tail $O/pmc_$tag.log; exit 1; }
done
echo done
