#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench lines, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; steps are chained with && so the first
# failure (fault, abort, timeout) ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== host: $(nproc) cpus; $(lscpu | grep 'Model name' | head -1)" > $O/host.txt
rocminfo 2>/dev/null | grep -E "Marketing Name|Compute Unit|gfx950" | head -6 >> $O/host.txt
STAGE=${1:-all}
run_tests() { timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; }
run_bench() {
  timeout -k 10 400 python bench.py > $O/bench_nyu.json 2> $O/bench_nyu.err &&
  timeout -k 10 300 python bench.py --config kitti --no-cpu-baseline > $O/bench_kitti.json 2> $O/bench_kitti.err &&
  timeout -k 10 300 python bench.py --config nyu_k16 --no-cpu-baseline > $O/bench_nyu_k16.json 2> $O/bench_nyu_k16.err
}
run_prof() {
  cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o nyu --output-format csv -- \
      python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_nyu.log 2>&1 &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kitti --output-format csv -- \
      python3 $R/bench.py --config kitti --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_kitti.log 2>&1
}
case $STAGE in
  all) run_tests && run_smoke && run_bench && run_prof ;;
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  benchprof) run_bench && run_prof ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc" >> $O/host.txt
exit $rc
