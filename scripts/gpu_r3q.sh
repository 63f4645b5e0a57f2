#!/bin/bash
# C2 / C1 / C3 step 1 (fp32 FIRST step kernel): the capi translation unit with SLP packing on vs off.
set -o pipefail
O=gpurun_out/r3q_$1; mkdir -p $O
for CFG in nyu nyu_b1 kitti nyu_k16; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- capislp=nlspn_eccv20_amd/lib/ab/libnlspn_capislp.so base=nlspn_eccv20_amd/lib/ab/libnlspn_r3base.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
