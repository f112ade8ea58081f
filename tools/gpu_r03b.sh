set -u
O=gpurun_out/r03d
mkdir -p $O
export NC_GPUHASH_DEBUG=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_host_api.py tests/test_gpu_shard_dist.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
echo done
