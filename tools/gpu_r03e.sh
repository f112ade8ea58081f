set -u
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "gsort or full_size or beyond_4gib" > $O/pytest_gsort.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes fnv1a_64,one_at_a_time,fnv1_32 --variants 0,33554432,35651584,37748736,39845888,34603008,262152 --rounds 3 --iters 10 > $O/ab_c2.jsonl 2> $O/ab_c2.err || exit $?
export NC_GPUHASH_DEBUG=2
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host_api.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "pinned_pipe_matches_oracle and tiny2" > $O/pytest_pipe.log 2>&1 || exit $?
echo done
