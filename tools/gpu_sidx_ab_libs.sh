set -u
mkdir -p gpurun_out/r05_sidx_b128
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py > gpurun_out/r05_sidx_b128/tests.txt 2>&1 || exit 1
for i in 1 2 3; do
  for lib in sidx_base sidx_b128; do
    timeout -k 10 200 python -u tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --pipes policy,diag_nosearch --lib tools/ablib/$lib.so > gpurun_out/r05_sidx_b128/${lib}_$i.jsonl 2>&1 || exit 1
  done
done
echo done
