set -u
mkdir -p gpurun_out/r05_sidx_sets
for i in 1 2; do
timeout -k 10 300 python -u tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --rounds 5 --pipes plain_hash,policy,grouped1,grouped8,diag_nosearch,diag_bare,diag_bare_noprologue > gpurun_out/r05_sidx_sets/ab_$i.jsonl 2>&1 || exit 1
done
echo done
