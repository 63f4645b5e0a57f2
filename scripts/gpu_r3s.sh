#!/bin/bash
# Step kernel: per-tap wave masks for pass B at small K (3x3) — parity, then same-box A/B vs HEAD.
set -o pipefail
O=gpurun_out/r3s_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_fp16.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for CFG in nyu nyu_b1 kitti; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- head=nlspn_eccv20_amd/lib/ab/libnlspn_head.so base=nlspn_eccv20_amd/lib/ab/libnlspn_r3base.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
