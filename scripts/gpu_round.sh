#!/bin/bash
# Round evidence on the GPU box: full GPU test suite, bench lines (C2 resident and
# per-iteration A/B, C3, C5), rocprofv3 kernel stats, PMC HBM-traffic passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_nyu.json 2> $O/bench_nyu.err &&
NLSPN_RESIDENT=0 timeout -k 10 300 python bench.py --no-backward --cpu-reps 1 > $O/bench_nyu_steps.json 2> $O/bench_nyu_steps.err &&
timeout -k 10 400 python bench.py --config kitti --no-backward --cpu-reps 1 > $O/bench_kitti.json 2> $O/bench_kitti.err &&
timeout -k 10 400 python bench.py --config nyu_k16 --cpu-reps 1 > $O/bench_nyu_k16.json 2> $O/bench_nyu_k16.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_nyu -o nyu --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-backward > $O/stats_nyu.log 2>&1 &&
for C in FETCH_SIZE WRITE_SIZE; do
  NLSPN_PLAN_GRAPH=1 timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_$C -o run --output-format csv -- \
      python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru --kernel-reps 5 > $O/pmc_$C.log 2>&1 || exit 1
done
