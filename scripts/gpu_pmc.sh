#!/bin/bash
# PMC passes (counters only with --kernel-trace, one counter group per pass) over
# the A/B harness (calibration kernel with known bytes) and the product bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace -d $O/sb_$tag -o run --output-format csv -- \
      $R/tools/step_bench k8f32 8 228 304 10 1 2.0 > $O/sb_$tag.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $O/bench_$tag -o run --output-format csv -- \
      python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-reps 20 > $O/bench_$tag.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_nyu -o nyu --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/stats_nyu.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_kitti -o kitti --output-format csv -- \
    python3 $R/bench.py --config kitti --steps 20 --warmup 5 --no-cpu-baseline > $O/stats_kitti.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_k16 -o k16 --output-format csv -- \
    python3 $R/bench.py --config nyu_k16 --steps 10 --warmup 3 --no-cpu-baseline > $O/stats_k16.log 2>&1
