#!/bin/bash
# round-4: early staging and setup-written offsets removed (measured slower, r4l); the
# remaining changes since the poison commit (setup span floored once, group loop folded, opaque
# poison constant): resident / parity tests, same-box A/B vs the poison commit, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py" \
  CFGS="nyu kitti nyu_b1" TRACE="nyu kitti" bash scripts/gpu_exp.sh r4n poison=$L/libnlspn_r4poison.so cur=- || exit 1
