set -u
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gsort or golden_corpus or kats" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 500 python3 tools/ab.py --configs C2 --modes md5,fnv1a_64,hsieh,jenkins,murmur,crc16 --variants 0,167772160,234881024,239075328,236978176 --rounds 3 --iters 10 > $O/ab_c2.jsonl 2> $O/ab_c2.err || exit $?
echo done
