#!/bin/bash
# Round-5 counters of chosen configs: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes,
# tools/pmc_summary.py) and the SQ counters of the resident kernel (scripts/gpu_sq.sh).
# usage: scripts/gpu_r5_pmc.sh TAG "CFG ..." "SQCFG ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; O=$R/gpurun_out/round_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in $2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_${CFG}_$C -o run --output-format csv -- \
        python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
        --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_${CFG}_$C.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py --bench $CFG "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config $CFG (scripts/gpu_r5_pmc.sh $TAG)" \
      $O/pmc_$CFG.json $O/pmc_${CFG}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${CFG}_WRITE_SIZE/run_counter_collection.csv \
      > $O/pmc_$CFG.txt 2>&1 || exit 1
  cat $O/pmc_$CFG.txt
done
cd $R
for CFG in $3; do
  bash scripts/gpu_sq.sh $TAG $CFG > $O/sq_$CFG.log 2>&1 || { tail $O/sq_$CFG.log; exit 1; }
  cp gpurun_out/sq_${TAG}_$CFG/sq_summary.json $O/sq_resident_$CFG.json || exit 1
  cat gpurun_out/sq_${TAG}_$CFG/sq_summary.txt
done
