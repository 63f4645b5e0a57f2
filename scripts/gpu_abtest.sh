#!/bin/bash
# Resident-kernel variant check: bit-exactness tests on the in-tree build, then a same-box
# A/B of library builds (C2 and C3) and a critical-path trace of the in-tree build.
# usage: scripts/gpu_abtest.sh TAG NAME=LIB ...   (outputs under gpurun_out/abtest_TAG)
set -o pipefail
TAG=$1; shift
O=gpurun_out/abtest_$TAG; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_offset_golden.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/gpu_ab.sh cur=- "$@" > $O/ab_nyu.txt 2>&1 || { cat $O/ab_nyu.txt; exit 1; }
AB_CONFIG=kitti bash scripts/gpu_ab.sh cur=- "$@" > $O/ab_kitti.txt 2>&1 || { cat $O/ab_kitti.txt; exit 1; }
AB_CONFIG=nyu_k16 bash scripts/gpu_ab.sh cur=- "$@" > $O/ab_nyu_k16.txt 2>&1 || { cat $O/ab_nyu_k16.txt; exit 1; }
cat $O/ab_nyu.txt $O/ab_kitti.txt $O/ab_nyu_k16.txt
timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu.json 2>&1 || exit 1
tail -1 $O/trace_nyu.json
