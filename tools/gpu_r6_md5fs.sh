set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes md5 --variants 557056,561152,557056,561152 --rounds 5 --iters 10 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
for v in 557056 561152; do
  for ctr in WRITE_SIZE FETCH_SIZE SQ_INSTS_VALU; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/pmc_${v}_$ctr -o pmc --output-format csv -- python3 tools/pmc_run.py --config C2 --mode md5 --variant 0:0:$v --iters 5 > $O/pmc_${v}_$ctr.log 2>&1 || { tail $O/pmc_${v}_$ctr.log; exit 1; }
  done
done
echo done
