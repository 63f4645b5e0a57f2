#!/bin/bash
# One experiment call: selected GPU tests, a same-box A/B of library builds over bench configs,
# and the resident trace of the in-tree build.
# usage: TESTS="tests/test_gpu_resident.py ..." CFGS="nyu kitti" scripts/gpu_exp.sh TAG SPEC [SPEC ...]
#        (SPEC as scripts/gpu_ab.sh: NAME=LIBPATH_OR_-[:ENV=VAL]; outputs under gpurun_out/exp_TAG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/exp_$TAG
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for CFG in ${CFGS:-nyu}; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh "$@" > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
for CFG in ${TRACE:-nyu}; do
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/res_trace_$CFG.json > $O/res_trace_$CFG.log 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/res_trace_$CFG.json'));g=d['group0'];print('$CFG', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items() if k!='setup'})"
done
