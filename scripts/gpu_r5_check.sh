#!/bin/bash
# Round-5 check call: GPU tests (TESTS, default the resident + parity suites), an interleaved
# same-process env A/B (tools/ab_env.py; AB_ENV, default NLSPN_RES_FIRST=0), the default bench
# line (no CPU / backward / GRU legs) and the C2 resident trace.
# usage: TAG=x [TESTS=...] [AB_ENV=NAME=VAL] [AB_CFGS=nyu,kitti,nyu_b1] [NOBENCH=1] [TRACE="nyu kitti"] scripts/gpu_r5_check.sh
set -o pipefail
O=gpurun_out/${TAG:-r5}; mkdir -p $O
TESTS=${TESTS:-tests/test_gpu_resident.py tests/test_gpu_parity.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
if [ "${AB_ENV:-NLSPN_RES_FIRST=0}" != "none" ]; then
  timeout -k 10 300 python tools/ab_env.py --env ${AB_ENV:-NLSPN_RES_FIRST=0} --configs ${AB_CFGS:-nyu,kitti,nyu_b1} > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  cat $O/ab.json
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru --no-heads > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench.json'));print('C2',d['value'],d['roofline']['kernel_ms_mean'],{k:(v['value'],v['roofline']['kernel_ms_mean']) for k,v in d['configs'].items()})"
fi
for CFG in ${TRACE:-nyu}; do
  [ "$CFG" = none ] && continue
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/res_trace_$CFG.json > $O/res_trace_$CFG.log 2>&1 || { tail $O/res_trace_$CFG.log; exit 1; }
  python -c "import json;d=json.load(open('$O/res_trace_$CFG.json'));g=d['group0'];print('$CFG', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items()})"
done
