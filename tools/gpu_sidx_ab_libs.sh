#!/bin/bash
# Same-box A/B of two library builds on the fused ketama dispatch (C2,
# fnv1a_64, 8 x 160 points), after the dispatch GPU tests on the in-tree build.
#   usage: tools/gpu_sidx_ab_libs.sh TAG LIB_A LIB_B [PIPES]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py tests/test_gpu_zz_robustness.py > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for i in 1 2 3; do
  for lib in "$2" "$3"; do
    tag=$(basename "$lib" .so)
    timeout -k 10 200 python -u tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --pipes "${4:-plain_hash,policy}" --rounds 5 --lib "$lib" > "$O/${tag}_$i.jsonl" 2>&1 || exit 1
  done
done
echo done
