#!/bin/bash
# Round 6: resident backward vs step launches per bench config (experiments build, same process),
# then the backward GPU tests (product build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_bwdcfg_${1:-a}; mkdir -p $O
cd $R
for CFG in ${CFGS:-nyu nyu_b1 kitti}; do
  NLSPN_LIB_PATH=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so timeout -k 10 300 python tools/ab_bwd.py --config $CFG \
      res= steps=NLSPN_BWD_RESIDENT=0 > $O/ab_$CFG.json 2> $O/ab_$CFG.err || { tail -5 $O/ab_$CFG.err; exit 1; }
  cat $O/ab_$CFG.json
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_backward_golden.py tests/test_gpu_step_backward.py \
    tests/test_gpu_torch_ops.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc
