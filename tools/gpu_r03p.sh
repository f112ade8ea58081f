set -u
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dispatch.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gsort or full_size or virtual or golden_corpus or kats or auto_policy or ketama_lookup" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes fnv1a_64,one_at_a_time,fnv1_32 --variants 0,234881024,171966464,239075328,327680 --rounds 3 --iters 10 > $O/ab_c2.jsonl 2> $O/ab_c2.err || exit $?
echo done
