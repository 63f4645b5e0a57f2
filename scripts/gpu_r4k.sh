#!/bin/bash
# round-4: poisoned-plane hand-off (data as the flag) in the resident kernel: the resident /
# parity / model / backward GPU tests, then a same-box A/B against the round-3 base and the
# previous commit (flag hand-off), and the trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_model.py tests/test_backward_golden.py tests/test_gpu_step_fp16.py" \
  CFGS="nyu kitti nyu_b1" TRACE="nyu" bash scripts/gpu_exp.sh r4k base=$L/libnlspn_r4base.so flag=$L/libnlspn_r4pitch.so cur=- || exit 1
