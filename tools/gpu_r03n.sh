set -u
O=gpurun_out/r03n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o sidx --output-format csv -- python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --tags none --rounds 2 > $O/ab_sidx.jsonl 2> $O/ab_sidx.err || exit $?
echo done
