#!/bin/bash
# Round validation on one box: smoke, every GPU test, the bench line and the
# same bench under rocprofv3 kernel-trace (tools/gpu_profile_round.sh bench),
# then PMC passes of the given workloads (tools/gpu_pmc_round.sh).
#   usage: tools/gpu_validate_round.sh TAG [CFG:MODE ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_profile_round.sh ${TAG}_prof bench || exit $?
[ $# -gt 0 ] && { bash tools/gpu_pmc_round.sh pmc_$TAG "$@" || exit $?; }
echo validate done
