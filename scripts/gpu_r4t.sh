#!/bin/bash
# round-4: gathers issued 4 slots ahead in the fp32 128-thread build only (C1's small parts):
# resident / parity tests, same-box A/B vs pf4-everywhere and the previous tree at C1, C2 check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py" CFGS="nyu_b1 nyu" TRACE="nyu_b1" \
  bash scripts/gpu_exp.sh r4t pf4all=$L/libnlspn_pf4.so cur=- || exit 1
