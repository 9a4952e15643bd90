#!/bin/bash
# End-of-round evidence for the default bench: kernel stats + the per-launch list (prof_round.sh, then
# tools/klaunch.py), the FETCH_SIZE / WRITE_SIZE passes, and two SQ counter passes over the local passes.
# Usage: tools/gpu/round_profiles.sh <tag>   (outputs under gpurun_out/<tag>)
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 300 make -s -C "$R/tools" stage_bench > "$OUT/make.log" 2>&1 || { echo "stage_bench build failed"; tail "$OUT/make.log"; exit 1; }
bash "$R/tools/gpu/prof_round.sh" "$TAG" || exit 1
python3 "$R/tools/klaunch.py" "$OUT/stats" extract_hist > "$OUT/kernel_launches.txt" 2>&1
KRE="extract_partition_fast|local_unique|local_merge|dummy_sink|msd_partition"
bash "$R/tools/gpu/run_sq.sh" "$TAG/sq1" "$KRE" SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES > "$OUT/sq1.txt" || exit 1
bash "$R/tools/gpu/run_sq.sh" "$TAG/sq2" "$KRE" SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_WAVES > "$OUT/sq2.txt" || exit 1
cat "$OUT/sq1.txt" "$OUT/sq2.txt"
