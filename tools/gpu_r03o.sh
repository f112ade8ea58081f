set -u
# PMC passes for the md5 legs (C2, C4 shard) and the C2 headline (grouped pipeline)
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
MEM="TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum"
bash tools/gpu_pmc.sh r03o/c2_md5 C2 md5 0 "$SQ" "$MEM" "FETCH_SIZE" "WRITE_SIZE" > /dev/null || exit 1
bash tools/gpu_pmc.sh r03o/c4_md5 C4S md5 0 "$SQ" "$MEM" "FETCH_SIZE" "WRITE_SIZE" > /dev/null || exit 1
bash tools/gpu_pmc.sh r03o/c2_fnv C2 fnv1a_64 0 "$SQ" "$MEM" "FETCH_SIZE" "WRITE_SIZE" > /dev/null || exit 1
bash tools/gpu_pmc.sh r03o/c2_fnv_nohash C2 fnv1a_64 168820736 "$SQ" "$MEM" > /dev/null || exit 1
echo done
