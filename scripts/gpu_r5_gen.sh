#!/bin/bash
# Round-5 geometry-generalisation check: the resident tests (3x3 + the 1x17 / 5x5 builds),
# the C5 resident-vs-steps same-process A/B, then the in-tree library vs a reference build
# (LIB_B, default the pre-generalisation HEAD build) on C2 / C3 / C1 (scripts/gpu_ab.sh).
set -o pipefail
O=gpurun_out/${TAG:-gen}; mkdir -p $O
if [ "${TESTS:-tests/test_gpu_resident.py}" != none ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_resident.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python tools/ab_env.py --env NLSPN_RESIDENT=0 --configs ${C5CFG:-nyu_k16} > $O/ab_c5.json 2> $O/ab_c5.err || { tail $O/ab_c5.err; exit 1; }
cat $O/ab_c5.json
for c in ${AB_CFGS:-nyu kitti nyu_b1}; do
  AB_CONFIG=$c timeout -k 10 600 scripts/gpu_ab.sh cur=- base=${LIB_B:-nlspn_eccv20_amd/lib/r4/libnlspn_hip_head.so} > $O/ab_$c.txt 2>&1 || { tail $O/ab_$c.txt; exit 1; }
  echo "== $c"; cat $O/ab_$c.txt
done
