#!/bin/bash
# round-4: s_sleep between a staging spin's re-loads: 1 (default) vs 0 vs 3 (A/B builds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/abx
O=gpurun_out/exp_r4v; mkdir -p $O
for CFG in nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- s0=$L/libnlspn_sleep0.so s3=$L/libnlspn_sleep3.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
