#!/bin/bash
# Round 6: resident backward pass 1 with two 512-thread parts per CU (NLSPN_BWD_RES_NT=512) vs one
# 1024-thread part (experiments build, same process), C2 and KITTI; then the backward tests with
# the knob set (exp build) for parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_resnt_${1:-a}; mkdir -p $O
cd $R
export NLSPN_LIB_PATH=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so
for CFG in nyu kitti; do
  timeout -k 10 300 python tools/ab_bwd.py --config $CFG nt1024= nt512=NLSPN_BWD_RES_NT=512 steps=NLSPN_BWD_RESIDENT=0 \
      > $O/ab_$CFG.json 2> $O/ab_$CFG.err || { tail -5 $O/ab_$CFG.err; exit 1; }
  cat $O/ab_$CFG.json
done
NLSPN_BWD_RES_NT=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "resident or oracle or full" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc
