#!/bin/bash
# Counter passes (one --pmc group per rocprofv3 run, nothing else traced) for
# one config/mode/variant: rocprofv3 --pmc ... -- python3 tools/pmc_run.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
CFG=${CFG:-C3}; MODE=${MODE:-fnv1a_64}; VAR=${VAR:-0:0:0}
tag=${CFG}_${MODE}_${VAR//:/-}
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/${tag}_p$i" -o pmc --output-format csv -- \
      python3 tools/pmc_run.py --config "$CFG" --mode "$MODE" --variant "$VAR" --iters 5 > "$OUT/${tag}_p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
