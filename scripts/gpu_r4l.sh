#!/bin/bash
# round-4: early staging loads (NLSPN_RES_EARLY=1: next iteration's rim quad loaded right after
# a wave's taps) and the output dict's inserted offsets written by the resident setup instead
# of step 1 (NLSPN_RES_OFFOUT=1), on top of the poisoned-plane hand-off: the resident tests
# with both on, then resident / parity tests at the defaults, and a same-box A/B vs the
# previous commit (poison), each feature, both, both with every hand-off write-through
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
O=gpurun_out/exp_r4l; mkdir -p $O
NLSPN_RES_EARLY=1 NLSPN_RES_OFFOUT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_features_on.log 2>&1 || { tail -30 $O/pytest_features_on.log; exit 1; }
tail -2 $O/pytest_features_on.log
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_offset_golden.py" \
  CFGS="nyu kitti nyu_b1" TRACE="nyu" bash scripts/gpu_exp.sh r4l poison=$L/libnlspn_r4poison.so cur=- \
  early=-:NLSPN_RES_EARLY=1 offout=-:NLSPN_RES_OFFOUT=1 both=-:NLSPN_RES_EARLY=1,NLSPN_RES_OFFOUT=1 \
  wt=-:NLSPN_RES_EARLY=1,NLSPN_RES_OFFOUT=1,NLSPN_RES_L2=0 || exit 1
