#!/bin/bash
# C5 step-kernel tile variants (NLSPN_STEP_VARIANT), same-box A/B, plus the C5 parity test per variant.
set -o pipefail
O=gpurun_out/c5var_$1; mkdir -p $O
AB_CONFIG=nyu_k16 bash scripts/gpu_ab.sh v0=-:NLSPN_STEP_VARIANT=0 v1=-:NLSPN_STEP_VARIANT=1 v2=-:NLSPN_STEP_VARIANT=2 \
    v3=-:NLSPN_STEP_VARIANT=3 > $O/ab_nyu_k16.txt 2>&1 || { cat $O/ab_nyu_k16.txt; exit 1; }
cat $O/ab_nyu_k16.txt
for V in 1 2 3; do
  NLSPN_STEP_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
      -k "c5 or k16 or 1x17 or 17" --timeout 120 --timeout-method thread > $O/pytest_v$V.log 2>&1 || { tail -20 $O/pytest_v$V.log; exit 1; }
  tail -1 $O/pytest_v$V.log
done
