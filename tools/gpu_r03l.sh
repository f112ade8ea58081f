set -u
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_sidx.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64,murmur --dists ketama --tags none,{} > $O/ab_sidx.jsonl 2> $O/ab_sidx.err || exit $?
echo done
