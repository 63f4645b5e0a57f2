#!/bin/bash
# round-4 final evidence, part b: PMC HBM traffic per config (FETCH_SIZE / WRITE_SIZE passes),
# SQ counters of the resident kernel (C2), resident traces (C2, C3, C1), same-box A/B vs the
# round-3 library, then the C1 part-grid sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=r04
O=$R/gpurun_out/round_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in nyu kitti nyu_b1 nyu_k16; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_${CFG}_$C -o run --output-format csv -- \
        python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
        --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_${CFG}_$C.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py --bench $CFG "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config $CFG (scripts/gpu_r4p.sh)" \
      $O/pmc_$CFG.json $O/pmc_${CFG}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${CFG}_WRITE_SIZE/run_counter_collection.csv \
      > $O/pmc_$CFG.txt 2>&1 || exit 1
  cat $O/pmc_$CFG.txt | tail -3
done
bash $R/scripts/gpu_sq.sh $TAG nyu > $O/sq_nyu.log 2>&1 || exit 1
cp $R/gpurun_out/sq_${TAG}_nyu/sq_summary.json $O/sq_resident_nyu.json || exit 1
tail -3 $O/sq_nyu.log
cd $R
for CFG in nyu kitti nyu_b1; do
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/res_trace_$CFG.json > $O/res_trace_$CFG.log 2>&1 || exit 1
done
for CFG in nyu kitti nyu_b1 nyu_k16; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- base=nlspn_eccv20_amd/lib/ab/libnlspn_r4base.so > $O/ab_$CFG.txt 2>&1 || exit 1
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
bash scripts/gpu_r4m.sh || exit 1
