#!/bin/bash
# Resident kernel with packed-f32 tap weights: parity (resident / parity / model suites),
# then a same-box A/B vs the scalar-tap library (the step-kernel product build).
set -o pipefail
O=gpurun_out/r3m_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_offset_golden.py \
    tests/test_gpu_model.py tests/test_gpu_replay.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- scalar=nlspn_eccv20_amd/lib/ab/libnlspn_stepprod.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
