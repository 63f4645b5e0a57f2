#!/bin/bash
# Parity of the wide-halo step variants (NLSPN_STEP_HALO=1), then a same-box A/B of the
# in-tree build with and without them on C5 / C2 / C3 / C1.
set -o pipefail
O=gpurun_out/r3e_$1; mkdir -p $O
NLSPN_STEP_HALO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_halo.log 2>&1 \
    || { tail -30 $O/pytest_halo.log; exit 1; }
tail -2 $O/pytest_halo.log
for CFG in nyu_k16 nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- wide=-:NLSPN_STEP_HALO=1 > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  cat $O/ab_$CFG.txt
done
