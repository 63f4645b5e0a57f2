#!/bin/bash
# round-4: contracted (FMA) bilinear in the resident taps, timing only (not oracle-exact)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
CFGS="nyu kitti nyu_b1" TRACE="nyu" bash scripts/gpu_exp.sh r4i cur=- fma=$L/libnlspn_fma.so || exit 1
O=gpurun_out/exp_r4i
export NLSPN_LIB_PATH=$L/libnlspn_fma.so
timeout -k 10 120 python tools/res_trace.py --config nyu --out $O/res_trace_nyu_fma.json > $O/res_trace_nyu_fma.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/res_trace_nyu_fma.json'));g=d['group0'];print('fma', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items() if k!='setup'})"
