#!/bin/bash
# Round 6: HBM traffic per config of the final forward kernels (rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE, one counter per pass, each config alone) -> gpurun_out/r6_pmc_TAG/pmc_CFG.json (the
# files bench.py reads from profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-a}
O=$R/gpurun_out/r6_pmc_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in nyu kitti nyu_k16 nyu_b1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_${CFG}_$C -o run --output-format csv -- \
        python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
        --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_${CFG}_$C.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py --bench $CFG "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config $CFG (scripts/gpu_r6_pmc.sh $TAG)" \
      $O/pmc_$CFG.json $O/pmc_${CFG}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${CFG}_WRITE_SIZE/run_counter_collection.csv \
      > $O/pmc_$CFG.txt 2>&1 || exit 1
  cat $O/pmc_$CFG.txt | head -5
done
