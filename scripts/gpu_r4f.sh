#!/bin/bash
# round-4: nonfinite reference tap (post-correction), classification skip, backward null grads
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_step_fp16.py tests/test_gpu_backward.py tests/test_backward_golden.py tests/test_gpu_parity.py" \
  CFGS="nyu kitti nyu_b1" TRACE="nyu kitti" bash scripts/gpu_exp.sh r4f base=$L/libnlspn_r4base.so cur=- || exit 1
