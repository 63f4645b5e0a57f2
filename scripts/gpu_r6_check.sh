#!/bin/bash
# Round 6: selected GPU tests (TESTS, default the parity file), then optionally the
# driver-shaped bench line (BENCH=1) and the smoke (SMOKE=1).
# usage: TESTS="tests/test_gpu_parity.py" BENCH=1 scripts/gpu_r6_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6}
O=$R/gpurun_out/r6_$TAG
mkdir -p $O
cd $R
TESTS=${TESTS:-tests/test_gpu_parity.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
      > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], {k: v['value'] for k, v in d.get('configs', {}).items()})"
fi
