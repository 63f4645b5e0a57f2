#!/bin/bash
# SQ counters of the C5 step kernel (bench --config nyu_k16), two passes of <= 8 SQ counters,
# counters + kernel trace only.  usage: scripts/gpu_c5_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5pmc_$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/p_$tag -o run --output-format csv -- \
      python3 $R/bench.py --config nyu_k16 --steps 3 --warmup 1 --no-cpu-baseline --no-backward --no-gru \
      --no-extra-configs --no-heads --kernel-reps 3 > $O/p_$tag.log 2>&1 || exit 1
done
ls $O
