set -u
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes all --variants 0,33554432,35651584,37748736 --rounds 3 --iters 10 > $O/ab_c2_all.jsonl 2> $O/ab_c2_all.err || exit $?
export NC_GPUHASH_DEBUG=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_pipe.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "virtual_key_base" > $O/pytest_vbase.log 2>&1 || exit $?
echo done
