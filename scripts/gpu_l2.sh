#!/bin/bash
# Same-XCD L2 hand-offs (kResL2): bit-exactness tests, then a same-box A/B against the
# write-through form (NLSPN_RES_L2=0) on C2 / C3 / C1, and traces of both forms.
set -o pipefail
O=gpurun_out/l2_$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_model.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for CFG in nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh l2=- wt=-:NLSPN_RES_L2=0 > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
done
cat $O/ab_nyu.txt $O/ab_kitti.txt $O/ab_nyu_b1.txt
timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu_l2.json 2>&1 || exit 1
NLSPN_RES_L2=0 timeout -k 10 120 python tools/res_trace.py --config nyu > $O/trace_nyu_wt.json 2>&1 || exit 1
tail -1 $O/trace_nyu_l2.json; tail -1 $O/trace_nyu_wt.json
