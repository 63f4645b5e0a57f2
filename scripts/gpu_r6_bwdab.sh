#!/bin/bash
# Round 6: backward A/Bs in one process (experiments build, tools/ab_bwd.py): resident pass 1
# vs the step launches, pass 2's prefetching forms (NLSPN_BWD_PF=1 / 2), at T = 18 and T = 4;
# then the backward GPU tests (product build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_bwdab_${1:-a}; mkdir -p $O
cd $R
for T in 18 4; do
  NLSPN_LIB_PATH=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so timeout -k 10 300 python tools/ab_bwd.py --config ${CFG:-nyu} --T $T \
      res= pf1=NLSPN_BWD_PF=1 pf2=NLSPN_BWD_PF=2 steps=NLSPN_BWD_RESIDENT=0 steps_pf1=NLSPN_BWD_RESIDENT=0,NLSPN_BWD_PF=1 \
      > $O/ab_t$T.json 2> $O/ab_t$T.err || { tail -5 $O/ab_t$T.err; exit 1; }
  cat $O/ab_t$T.json
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_backward_golden.py tests/test_gpu_step_backward.py \
    -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
