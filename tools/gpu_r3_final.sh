#!/bin/bash
# Round-3 validation + profile on one box: crc table-copies A/B (ABA across
# processes), smoke, every GPU test, the bench line and the same bench under
# rocprofv3 kernel-trace, FETCH/WRITE passes of every leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
ab() { timeout -k 10 300 python3 tools/ab.py --configs C3 --modes crc32,crc16,crc32a --variants 0 --rounds 3 --iters 10 "$@"; }
ab > $O/crc_a1.jsonl 2>$O/crc.err && ab --lib tools/ablib/libnc_gpuhash_crc16copies.so > $O/crc_b.jsonl 2>>$O/crc.err && ab > $O/crc_a2.jsonl 2>>$O/crc.err || { tail $O/crc.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes fnv1a_64,murmur --variants 0,507510784,0 --rounds 3 --iters 10 > $O/nosort.jsonl 2>$O/nosort.err || { tail $O/nosort.err; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_profile_round.sh r03f_prof bench || exit $?
echo final done
