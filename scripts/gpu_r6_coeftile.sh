#!/bin/bash
# Round 6: pass-2 tile shapes (experiments build, NLSPN_BWD_COEF_TILE), same process, C2 and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_coeftile_${1:-a}; mkdir -p $O
cd $R
for CFG in nyu kitti; do
  NLSPN_LIB_PATH=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so timeout -k 10 300 python tools/ab_bwd.py --config $CFG \
      t8x32= t16x32=NLSPN_BWD_COEF_TILE=16x32 t8x64=NLSPN_BWD_COEF_TILE=8x64 t4x64=NLSPN_BWD_COEF_TILE=4x64 \
      t4x32=NLSPN_BWD_COEF_TILE=4x32 t16x16=NLSPN_BWD_COEF_TILE=16x16 > $O/ab_$CFG.json 2> $O/ab_$CFG.err || { tail -5 $O/ab_$CFG.err; exit 1; }
  cat $O/ab_$CFG.json
done
