#!/bin/bash
# One GPU call, several measurements (each step time-limited; any failure ends it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_sidx_pmc.sh r03w pmc_r03 || exit $?
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 400 python3 tools/ab.py --configs C3 --modes crc16,crc32,crc32a --variants 0,8912896,9961472,12058624,524288,3670016 --rounds 3 --iters 10 > $O/ab_c3crc.jsonl 2> $O/ab_c3crc.err || { tail $O/ab_c3crc.err; exit 1; }
timeout -k 10 120 tools/probes/md5_rate > $O/md5_rate.jsonl 2>&1 || exit $?
bash tools/gpu_c5_trace.sh r03c5 0.3 0.05 || exit $?
echo batch done
