set -u
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gsort or full_size or virtual or golden_corpus" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes fnv1a_64,one_at_a_time,hsieh,jenkins --variants 0,235929600,238026752,240123904,242221056 --rounds 3 --iters 10 > $O/ab_c2.jsonl 2> $O/ab_c2.err || exit $?
echo done
