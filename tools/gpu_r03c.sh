set -u
O=gpurun_out/r03c
mkdir -p $O
export NC_GPUHASH_DEBUG=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k pinned > $O/pytest_gpu.log 2>&1 || exit $?
echo done
