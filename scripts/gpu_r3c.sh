#!/bin/bash
# Tests of the current tree, then a same-box A/B of the in-tree build vs the same sources with
# no SLP packing (noslp) and the round-2 library, on C2 / C3 / C5 / C1.
set -o pipefail
O=gpurun_out/r3c_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu_k16 nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- noslp=nlspn_eccv20_amd/lib/ab/libnlspn_noslp.so \
      r02=nlspn_eccv20_amd/lib/ab/libnlspn_r02.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  cat $O/ab_$CFG.txt
done
