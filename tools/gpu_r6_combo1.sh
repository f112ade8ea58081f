set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_r6_md5sp.sh r06h || exit $?
mkdir -p gpurun_out/r06i
timeout -k 10 120 python3 tools/clock_ring.py --out gpurun_out/r06i/clock_ring.json > gpurun_out/r06i/clock_ring.log 2>&1 || { tail -20 gpurun_out/r06i/clock_ring.log; exit 1; }
cat gpurun_out/r06i/clock_ring.log
