#!/bin/bash
# Round 6: SQ counters of the GRU-mode convolutions (tools/gc_bench.py, presets only), two
# passes of <= 8 SQ counters, summarised per kernel by tools/sq_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gcsq_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
         "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/p$n -o run --output-format csv -- \
      python3 $R/tools/gc_bench.py --reps 3 --presets-only > $O/p$n.log 2>&1 || exit 1
done
python3 $R/tools/sq_summary.py $O/sq_summary.json $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    --kernel gconv > $O/sq_summary.txt 2>&1 || exit 1
cat $O/sq_summary.txt
