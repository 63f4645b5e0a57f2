#!/bin/bash
# round-4: C1 (one NYU image) part grid under the poisoned-plane hand-off: the default
# 32 parts of 541 quads vs more, smaller parts (NLSPN_RES_GRID=gy,gx)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/exp_r4m; mkdir -p $O
AB_CONFIG=nyu_b1 bash scripts/gpu_ab.sh g8x4=- g16x4=-:NLSPN_RES_GRID=16x4 g8x8=-:NLSPN_RES_GRID=8x8 \
  g12x8=-:NLSPN_RES_GRID=12x8 g16x8=-:NLSPN_RES_GRID=16x8 g19x8=-:NLSPN_RES_GRID=19x8 g16x16=-:NLSPN_RES_GRID=16x16 \
  > $O/ab_grid_nyu_b1.txt 2>&1 || { cat $O/ab_grid_nyu_b1.txt; exit 1; }
cat $O/ab_grid_nyu_b1.txt
