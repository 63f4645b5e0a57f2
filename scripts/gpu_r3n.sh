#!/bin/bash
# Step kernel: packed-f32 bilinear (product) vs the scalar form without SLP packing.
set -o pipefail
O=gpurun_out/r3n_$1; mkdir -p $O
NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/ab/libnlspn_scalar.so timeout -k 10 300 python -u -m pytest tests/test_gpu_step_fp16.py \
    tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu_k16 nyu; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- scalar=nlspn_eccv20_amd/lib/ab/libnlspn_scalar.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
