#!/bin/bash
# round-4: C1 (247 parts) trace, PMC traffic and kernel stats for the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/exp_r4r; mkdir -p $O
timeout -k 10 120 python tools/res_trace.py --config nyu_b1 --out $O/res_trace_nyu_b1.json > $O/res_trace_nyu_b1.log 2>&1 || { cat $O/res_trace_nyu_b1.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_nyu_b1_$C -o run --output-format csv -- \
      python3 $R/bench.py --config nyu_b1 --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
      --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_nyu_b1_$C.log 2>&1 || exit 1
done
python3 $R/tools/pmc_summary.py --bench nyu_b1 "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config nyu_b1 (scripts/gpu_r4r.sh)" \
    $O/pmc_nyu_b1.json $O/pmc_nyu_b1_FETCH_SIZE/run_counter_collection.csv $O/pmc_nyu_b1_WRITE_SIZE/run_counter_collection.csv \
    > $O/pmc_nyu_b1.txt 2>&1 || exit 1
cat $O/pmc_nyu_b1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_nyu_b1 -o bench --output-format csv -- \
    python3 $R/bench.py --config nyu_b1 --steps 20 --warmup 5 --no-cpu-baseline --no-backward --no-gru --no-heads \
    --no-extra-configs > $O/stats_nyu_b1.log 2>&1 || exit 1
