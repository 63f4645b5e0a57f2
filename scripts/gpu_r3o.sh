#!/bin/bash
# Two-pass propagation backward: GPU backward / training suites, then a same-box A/B of the
# bench's backward timing (graph-replayed fwd+bwd) against the one-pass form.
set -o pipefail
O=gpurun_out/r3o_$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_step_backward.py tests/test_gpu_torch_ops.py \
    tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for m in two one; do
    if [ $m = one ]; then export NLSPN_BWD_ONEPASS=1; else unset NLSPN_BWD_ONEPASS; fi
    timeout -k 10 300 python bench.py --no-gru --no-extra-configs --no-cpu-baseline --no-heads --steps 20 --warmup 5 \
        > $O/bench_$m$r.json 2> $O/bench_$m$r.err || { tail -5 $O/bench_$m$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_$m$r.json'))['backward'];print('$m', d['ms_bwd_per_iter'], d.get('ms_bwd_per_iter_graph'), d.get('ms_fwd_bwd_per_step_graph'))"
  done
done
unset NLSPN_BWD_ONEPASS
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/stats -o bwd --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-gru --no-extra-configs --no-cpu-baseline --no-heads --steps 10 --warmup 3 \
    > $GRAFT_REPO_ROOT/$O/stats.log 2>&1 || exit 1
