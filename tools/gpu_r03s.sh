set -u
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 500 python3 tools/ab.py --configs C2 --modes all --variants 167772160,234881024,239075328,236978176 --rounds 3 --iters 10 > $O/ab_c2.jsonl 2> $O/ab_c2.err || exit $?
echo done
