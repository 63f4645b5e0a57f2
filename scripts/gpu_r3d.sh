#!/bin/bash
# Tests of the current tree (default and NLSPN_STEP_HALO=1), then a same-box A/B of the
# in-tree build vs the wide-halo step variants and the previous commit's library (b7).
set -o pipefail
O=gpurun_out/r3d_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
NLSPN_STEP_HALO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_offset_golden.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_halo.log 2>&1 \
    || { tail -30 $O/pytest_halo.log; exit 1; }
tail -2 $O/pytest_halo.log
for CFG in nyu_k16 nyu kitti; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- wide=-:NLSPN_STEP_HALO=1 b7=nlspn_eccv20_amd/lib/ab/libnlspn_b7.so \
      > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  cat $O/ab_$CFG.txt
done
