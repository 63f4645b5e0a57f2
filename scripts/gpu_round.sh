#!/bin/bash
# Round evidence on the GPU box: full GPU test suite, the default bench line (C2 headline
# + C3 / C5 / C1 under "configs" + cpu_baseline), rocprofv3 kernel stats of the default
# bench, and PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, one counter per pass).
# usage: [PART=a|b] scripts/gpu_round.sh [TAG]   (outputs under gpurun_out/round_TAG; PART a =
#        tests, bench lines and kernel stats, b = counters, traces and A/B; default both)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
O=$R/gpurun_out/round_$TAG
mkdir -p $O
cd $R
PART=${PART:-ab}
if [[ $PART == *a* ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
NLSPN_RESIDENT=0 timeout -k 10 300 python bench.py --no-backward --no-gru --no-extra-configs --no-cpu-baseline \
    > $O/bench_nyu_steps.json 2> $O/bench_nyu_steps.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-backward --no-gru > $O/stats.log 2>&1 || exit 1
# kernel stats per config (kernels are shared between configs, so the default run's
# averages mix them): each bench config alone, for the roofline cross-check
for CFG in nyu kitti nyu_k16 nyu_b1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$CFG -o bench --output-format csv -- \
      python3 $R/bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-backward --no-gru --no-heads \
      --no-extra-configs > $O/stats_$CFG.log 2>&1 || exit 1
done
fi
[[ $PART == *b* ]] || exit 0
cd /tmp && export TMPDIR=/tmp
# PMC HBM traffic, one config per pass pair (kernels are shared between configs)
for CFG in nyu kitti nyu_k16 nyu_b1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_${CFG}_$C -o run --output-format csv -- \
        python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
        --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_${CFG}_$C.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py --bench $CFG "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config $CFG (scripts/gpu_round.sh $TAG)" \
      $O/pmc_$CFG.json $O/pmc_${CFG}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${CFG}_WRITE_SIZE/run_counter_collection.csv \
      > $O/pmc_$CFG.txt 2>&1 || exit 1
done
# the reference's last head layers on MIOpen (input to the head-epilogue fusion work)
cd $R && timeout -k 10 180 python tools/head_prof.py > $O/head_prof.json 2> $O/head_prof.err || exit 1
# request-size PMC passes (read / write bytes by request width: checks the x2 FETCH_SIZE
# correction on this code) and the C5 step kernel's SQ counters
bash $R/scripts/gpu_pmc_req.sh $TAG nyu kitti nyu_b1 nyu_k16 || exit 1
bash $R/scripts/gpu_c5_pmc.sh $TAG || exit 1
# SQ counters of the resident kernel (C2) and its trace
bash $R/scripts/gpu_sq.sh $TAG nyu > $O/sq_nyu.log 2>&1 || exit 1
cp $R/gpurun_out/sq_${TAG}_nyu/sq_summary.json $O/sq_resident_nyu.json || exit 1
cd $R
for CFG in nyu kitti nyu_b1; do
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/res_trace_$CFG.json > $O/res_trace_$CFG.log 2>&1 || exit 1
done
# same-box A/B against the round's base library (the previous round's HEAD), when present
BASE=${AB_BASE:-nlspn_eccv20_amd/lib/ab/libnlspn_r4base.so}
if [ -f $BASE ]; then
  for CFG in nyu kitti nyu_k16 nyu_b1; do
    AB_CONFIG=$CFG bash scripts/gpu_ab.sh cur=- base=$BASE > $O/ab_$CFG.txt 2>&1 || exit 1
  done
fi
