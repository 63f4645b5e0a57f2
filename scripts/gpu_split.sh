#!/bin/bash
# Interior-first resident kernel (kResSplit): bit-exactness tests, same-box A/B against the
# no-split form and the round-1 / round-2 libraries, critical-path traces of both forms.
set -o pipefail
O=gpurun_out/split; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash scripts/gpu_ab.sh split=- nosplit=-:NLSPN_RES_SPLIT=0 r02=nlspn_eccv20_amd/lib/ab/libnlspn_r02.so \
    r01=nlspn_eccv20_amd/lib/ab/libnlspn_r01.so > $O/ab_nyu.txt 2>&1 || { cat $O/ab_nyu.txt; exit 1; }
AB_CONFIG=kitti bash scripts/gpu_ab.sh split=- nosplit=-:NLSPN_RES_SPLIT=0 r02=nlspn_eccv20_amd/lib/ab/libnlspn_r02.so \
    r01=nlspn_eccv20_amd/lib/ab/libnlspn_r01.so > $O/ab_kitti.txt 2>&1 || { cat $O/ab_kitti.txt; exit 1; }
cat $O/ab_nyu.txt $O/ab_kitti.txt
timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu_split.json 2>&1 || exit 1
NLSPN_RES_SPLIT=0 timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu_nosplit.json 2>&1 || exit 1
