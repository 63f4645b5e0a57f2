#!/bin/bash
# (1) tests of the current tree, (2) inserted offsets from the resident setup vs step 1 (C2, C3),
# (3) C5 step-kernel builds: fp16 mixed-precision taps (cur) vs converted (nomix) vs no SLP packing.
set -o pipefail
O=gpurun_out/r3b_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_model.py \
    tests/test_gpu_torch_ops.py tests/test_offset_golden.py tests/test_gpu_heads_prologue.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu kitti; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh res=- step1=-:NLSPN_RES_OFFOUT=0 > $O/ab_offout_$CFG.txt 2>&1 || { cat $O/ab_offout_$CFG.txt; exit 1; }
done
AB_CONFIG=nyu_k16 bash scripts/gpu_ab.sh mix=- nomix=nlspn_eccv20_amd/lib/ab/libnlspn_nomix.so \
    noslp=nlspn_eccv20_amd/lib/ab/libnlspn_noslp.so > $O/ab_c5.txt 2>&1 || { cat $O/ab_c5.txt; exit 1; }
cat $O/ab_offout_nyu.txt $O/ab_offout_kitti.txt $O/ab_c5.txt
timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu.json 2>&1 || exit 1
tail -1 $O/trace_nyu.json
