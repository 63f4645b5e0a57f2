#!/bin/bash
# Product step kernel (in-loop edge test, any-out gate, MIX staging): parity suites, same-box
# A/B vs the round-3 base library on every config, SQ counters of the C5 step kernel, and the
# request-size PMC pass of the resident configs.
set -o pipefail
O=gpurun_out/r3h_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_step_fp16.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_heads_prologue.py tests/test_gpu_resident.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu_k16 nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- base=nlspn_eccv20_amd/lib/ab/libnlspn_r3base.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
bash scripts/gpu_c5_pmc.sh $1 || exit 1
bash scripts/gpu_pmc_req.sh $1 nyu kitti nyu_b1 || exit 1
