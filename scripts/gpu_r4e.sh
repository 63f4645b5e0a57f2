#!/bin/bash
# round-4 experiment: resident interior-first / PF builds and the paired step window (C5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_step_fp16.py" CFGS="nyu" TRACE="nyu" \
  bash scripts/gpu_exp.sh r4e base=$L/libnlspn_r4base.so cur=- cur_noin=-:NLSPN_RES_INNER=0 nopair=$L/libnlspn_nopair.so ipf2=$L/libnlspn_ipf2.so || exit 1
CFGS="nyu_k16" TRACE="" bash scripts/gpu_exp.sh r4e_k16 base=$L/libnlspn_r4base.so cur=- nopair=$L/libnlspn_nopair.so || exit 1
NLSPN_RES_INNER=0 timeout -k 10 120 python tools/res_trace.py --config nyu --out gpurun_out/exp_r4e/res_trace_nyu_noin.json > /dev/null 2>&1 || exit 1
cat gpurun_out/exp_r4e/res_trace_nyu_noin.json
