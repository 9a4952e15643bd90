#!/bin/bash
# Kernel trace + stats of the default bench, the per-launch listing of one step, then SQ PMC passes
# over the named kernels.  Usage: tools/gpu/prof_r3.sh <tag> [kernel regex for the SQ passes]
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
KRE=${2:-local_unique|local_merge|dummy_sink}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --fasta-reads 0 > "$OUT/bench_stats.log" 2>&1 || { echo "stats rc=$?"; tail -20 "$OUT/bench_stats.log"; exit 1; }
python3 "$R/tools/kstats.py" "$OUT/stats" 40 > "$OUT/kernel_stats.txt" 2>&1
python3 "$R/tools/klaunch.py" "$OUT/stats" > "$OUT/kernel_launches.txt" 2>&1
echo "stats ok"; tail -1 "$OUT/bench_stats.log" | cut -c1-300
bash "$R/tools/gpu/run_sq.sh" "$TAG/sq1" "$KRE" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU > "$OUT/sq1.txt" 2>&1 || { echo "sq1 failed"; cat "$OUT/sq1.txt"; exit 1; }
bash "$R/tools/gpu/run_sq.sh" "$TAG/sq2" "$KRE" SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU > "$OUT/sq2.txt" 2>&1 || { echo "sq2 failed"; cat "$OUT/sq2.txt"; exit 1; }
echo "sq ok"; cat "$OUT/sq1.txt" "$OUT/sq2.txt"
