#!/bin/bash
# round-4: what bounds the resident taps phase: traces of timing-experiment builds
# (exp1: no LDS gathers; exp2: gathers without the tap arithmetic; pf2: gathers issued 2 slots ahead)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
O=gpurun_out/exp_r4g; mkdir -p $O
for v in cur exp1 exp2 pf2; do
  if [ $v = cur ]; then unset NLSPN_LIB_PATH; else export NLSPN_LIB_PATH=$L/libnlspn_$v.so; fi
  timeout -k 10 120 python tools/res_trace.py --config nyu --out $O/res_trace_nyu_$v.json > $O/res_trace_nyu_$v.log 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/res_trace_nyu_$v.json'));g=d['group0'];print('$v', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items() if k!='setup'})"
done
