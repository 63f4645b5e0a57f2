#!/bin/bash
# Step-kernel ablation (edge fix-up placement, pass-B flags, MIX staging) vs the round-3 base.
set -o pipefail
O=gpurun_out/r3g_$1; mkdir -p $O
L=nlspn_eccv20_amd/lib/ab
for CFG in nyu_k16 nyu; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- base=$L/libnlspn_r3base.so edgein=$L/libnlspn_edgein.so flags=$L/libnlspn_flags.so \
      flagsedge=$L/libnlspn_flagsedge.so fen=$L/libnlspn_flagsedgenomixs.so > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
