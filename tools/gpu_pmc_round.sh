#!/bin/bash
# Counter passes for several workloads, one rocprofv3 --pmc group per run
# (nothing else traced), over tools/pmc_run.py; summary per workload.
#   tools/gpu_pmc_round.sh TAG CFG:MODE[:VARIANT] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for w in "$@"; do
  IFS=: read -r CFG MODE VAR <<< "$w"
  VAR=${VAR:-0}
  tag=${CFG}_${MODE}_${VAR}
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
    case "$MODE" in probe_*) [ $i -ge 2 ] && break;; esac
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/${tag}_p$i" -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config "$CFG" --mode "$MODE" --variant "0:0:$VAR" --iters 5 > "$OUT/${tag}_p$i.log" 2>&1
    rc=$?
    echo "$tag pass $i rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/${tag}_p$i.log"; exit $rc; }
  done
  python3 tools/pmc_summary.py "$OUT"/${tag}_p* > "$OUT/${tag}_summary.json" 2>&1
done
echo done
