#!/bin/bash
# round-4: tap gathers issued 1/2/4 slots ahead (NLSPN_RES_PF builds) under the new grid:
# C1's 247 small parts (2 waves each: the taps are one wave's latency chain) and C2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
O=gpurun_out/exp_r4s; mkdir -p $O
for CFG in nyu_b1 nyu kitti; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- pf1=$L/libnlspn_pf1.so pf2=$L/libnlspn_pf2.so pf4=$L/libnlspn_pf4.so \
    > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
