#!/bin/bash
# SQ counters of one bench config's kernels: two passes of <= 8 SQ counters (+ GRBM), counters
# and kernel trace only, summarised per kernel by tools/sq_summary.py.
# usage: scripts/gpu_sq.sh TAG CONFIG   (outputs under gpurun_out/sq_TAG_CONFIG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=${2:-nyu}
O=$R/gpurun_out/sq_${TAG}_$CFG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/p$n -o run --output-format csv -- \
      python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-backward --no-gru \
      --no-extra-configs --no-heads --kernel-reps 3 > $O/p$n.log 2>&1 || exit 1
done
python3 $R/tools/sq_summary.py $O/sq_summary.json $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    --kernel prop_ > $O/sq_summary.txt 2>&1 || exit 1
cat $O/sq_summary.txt
