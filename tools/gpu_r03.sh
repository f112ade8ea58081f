#!/bin/bash
# Round-3 validation on the GPU box: smoke, the -m gpu suite, one bench line.
# usage: tools/gpu_r03.sh <tag> [pytest -k expr]
set -u
TAG=${1:-r03}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
if [ -n "$K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1 || exit $?
else
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
echo done
