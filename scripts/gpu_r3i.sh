#!/bin/bash
# Step kernel with the tile-level non-finite flag (no per-tap edge test): parity, then a
# same-box A/B vs the branch-free tap variant and the round-3 base library.
set -o pipefail
O=gpurun_out/r3i_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_fp16.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=nlspn_eccv20_amd/lib/ab
for CFG in nyu_k16 nyu; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- bfree=$L/libnlspn_bfree.so base=$L/libnlspn_r3base.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
