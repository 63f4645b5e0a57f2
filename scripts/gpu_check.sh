#!/bin/bash
# The whole GPU test suite, then a same-box A/B of library builds (C2, C3, C5) and a
# critical-path trace of the in-tree build.
# usage: scripts/gpu_check.sh TAG NAME=LIB ...   (outputs under gpurun_out/check_TAG)
set -o pipefail
TAG=$1; shift
O=gpurun_out/check_$TAG; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for CFG in nyu kitti nyu_k16; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- "$@" > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
done
cat $O/ab_nyu.txt $O/ab_kitti.txt $O/ab_nyu_k16.txt
timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu.json 2>&1 || exit 1
timeout -k 10 120 python tools/res_trace.py --config kitti --bg 2 > $O/trace_kitti.json 2>&1 || exit 1
tail -1 $O/trace_nyu.json
