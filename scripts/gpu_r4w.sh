#!/bin/bash
# round-4: C5 step 1 (fp16 K=16 fused prologue) with a waves-per-SIMD floor of 6 / 8 (A/B builds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/abx
O=gpurun_out/exp_r4w; mkdir -p $O
AB_CONFIG=nyu_k16 bash scripts/gpu_ab.sh cur=- w6=$L/libnlspn_f1w6.so w8=$L/libnlspn_f1w8.so > $O/ab_nyu_k16.txt 2>&1 || { cat $O/ab_nyu_k16.txt; exit 1; }
cat $O/ab_nyu_k16.txt
for n in cur w6 w8; do for r in 1 2 3; do python -c "import json;d=json.load(open('gpurun_out/ab/$n$r.json'));print('$n', d['roofline']['step1_kernel_ms'])"; done; done
