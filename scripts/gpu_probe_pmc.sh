# PMC counters of the resident kernel (separate passes; counters + kernel trace only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_res
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/res_probe.py > $O/probe.log 2>&1 || exit 1
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace -d $O/p_$tag -o run --output-format csv -- \
      python3 $R/tools/res_probe.py dbgs=0 resident=1,0 > $O/p_$tag.log 2>&1 || exit 1
done
