#!/bin/bash
# round-4: per-wave trace stamps of the resident taps phase (which waves finish last, on
# which SIMD), in-tree build and the timing-experiment builds (fma, exp1: no gathers,
# exp2: no tap arithmetic)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
O=gpurun_out/exp_r4j; mkdir -p $O
for v in wt_cur wt_fma wt_exp1 wt_exp2; do
  export NLSPN_LIB_PATH=$L/libnlspn_$v.so
  timeout -k 10 120 python tools/res_trace.py --config nyu --out $O/res_trace_nyu_$v.json > $O/res_trace_nyu_$v.log 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/res_trace_nyu_$v.json'));g=d['group0'];print('$v', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items() if k!='setup'})"
done
