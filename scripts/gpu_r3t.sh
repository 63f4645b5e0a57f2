#!/bin/bash
# C5 step kernel at 7 waves per SIMD (71 VGPRs) vs 6: parity on the 7-wave build, same-box A/B.
set -o pipefail
O=gpurun_out/r3t_$1; mkdir -p $O
NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/ab/libnlspn_w7.so timeout -k 10 300 python -u -m pytest tests/test_gpu_step_fp16.py \
    tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fp16 or c5 or 17" > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_CONFIG=nyu_k16 bash scripts/gpu_ab.sh cur=- w7=nlspn_eccv20_amd/lib/ab/libnlspn_w7.so > $O/ab_nyu_k16.txt 2>&1 || { cat $O/ab_nyu_k16.txt; exit 1; }
cat $O/ab_nyu_k16.txt
