#!/bin/bash
# C5 step kernel: branch-free taps at 6 and 7 waves per SIMD vs the product build.
set -o pipefail
O=gpurun_out/r3j_$1; mkdir -p $O
L=nlspn_eccv20_amd/lib/ab
NLSPN_LIB_PATH=$L/libnlspn_bfree7.so timeout -k 10 300 python -u -m pytest tests/test_gpu_step_fp16.py tests/test_gpu_parity.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "fp16 or c5 or 17" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu_k16; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- bfree=$L/libnlspn_bfree.so bfree7=$L/libnlspn_bfree7.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r3j_$1/avail.txt 2>&1 || true
