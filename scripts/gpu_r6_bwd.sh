#!/bin/bash
# Round 6: the resident backward pass 1 — backward GPU tests, the pass-1 A/B harness
# (tools/bwd_bench: split-step variants), the bench's backward leg, and a rocprofv3 kernel
# summary of the backward leg (BWDPROF=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_bwd_${1:-a}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_backward.py tests/test_backward_golden.py tests/test_gpu_step_backward.py} \
    -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -x tools/bwd_bench ] && [ "${BWDBENCH:-1}" = 1 ]; then
  timeout -k 10 180 tools/bwd_bench 8 228 304 30 3 > $O/bwd_bench.txt 2>&1 || { cat $O/bwd_bench.txt; exit 1; }
  cat $O/bwd_bench.txt
fi
if [ "${ABBWD:-1}" = 1 ]; then
  NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so timeout -k 10 300 python tools/ab_bwd.py --config nyu \
      res= steps=NLSPN_BWD_RESIDENT=0 res_nocw=NLSPN_BWD_CW=0 r5form=NLSPN_BWD_RESIDENT=0,NLSPN_BWD_CW=0 \
      > $O/ab_bwd_nyu.json 2> $O/ab_bwd_nyu.err || { tail -5 $O/ab_bwd_nyu.err; exit 1; }
  cat $O/ab_bwd_nyu.json
fi
if [ "${ABSTEP1:-0}" = 1 ]; then
  NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so timeout -k 10 300 python tools/ab_env.py --env NLSPN_STEP1_PX=2 \
      --configs nyu_k16 > $O/ab_step1_px2.json 2> $O/ab_step1_px2.err || { tail -5 $O/ab_step1_px2.err; exit 1; }
  cat $O/ab_step1_px2.json
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-extra-configs --no-cpu-baseline --no-heads --no-gru \
    > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d['backward']))"
if [ "${BWDPROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bwd --output-format csv -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-extra-configs --no-cpu-baseline --no-heads --no-gru > $O/prof.log 2>&1 || exit 1
fi
