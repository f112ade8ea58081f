set -u
O=gpurun_out/rs1
mkdir -p $O
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes fnv1a_64 --variants 0,33554560,33554816,33555584,33555840,33555072,32896 > $O/c2.jsonl 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes one_at_a_time,fnv1_32 --variants 0,33554560,33554816,16777216 >> $O/c2.jsonl 2>&1 || exit $?
