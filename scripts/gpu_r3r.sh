#!/bin/bash
# Two-pass backward: coefficient kernel at 6 waves per SIMD (80 VGPRs, some spills) vs 5 (92 VGPRs).
set -o pipefail
O=gpurun_out/r3r_$1; mkdir -p $O
NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/ab/libnlspn_coef6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for m in cur coef6; do
    unset NLSPN_LIB_PATH
    [ $m = coef6 ] && export NLSPN_LIB_PATH=nlspn_eccv20_amd/lib/ab/libnlspn_coef6.so
    timeout -k 10 300 python bench.py --no-gru --no-extra-configs --no-cpu-baseline --no-heads --steps 20 --warmup 5 \
        > $O/bench_$m$r.json 2> $O/bench_$m$r.err || { tail -5 $O/bench_$m$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_$m$r.json'))['backward'];print('$m', d['ms_bwd_per_iter'], d.get('ms_bwd_per_iter_graph'), d.get('ms_fwd_bwd_per_step_graph'))"
  done
done
