#!/bin/bash
# round-4: no per-image part cap (B=1 NYU: 247 parts of 72 quads instead of 32 of 551):
# resident / parity tests, same-box A/B vs the capped build at nyu_b1 and nyu (unchanged
# shape), the C1 trace, and C1's PMC traffic + kernel stats for the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_model.py" \
  CFGS="nyu_b1 nyu" TRACE="nyu_b1" bash scripts/gpu_exp.sh r4q capped=$L/libnlspn_r4capped.so cur=- || exit 1
O=$R/gpurun_out/exp_r4q
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_nyu_b1_$C -o run --output-format csv -- \
      python3 $R/bench.py --config nyu_b1 --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
      --no-extra-configs --no-heads --kernel-reps 5 > $O/pmc_nyu_b1_$C.log 2>&1 || exit 1
done
python3 $R/tools/pmc_summary.py --bench nyu_b1 "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py --config nyu_b1 (scripts/gpu_r4q.sh)" \
    $O/pmc_nyu_b1.json $O/pmc_nyu_b1_FETCH_SIZE/run_counter_collection.csv $O/pmc_nyu_b1_WRITE_SIZE/run_counter_collection.csv \
    > $O/pmc_nyu_b1.txt 2>&1 || exit 1
cat $O/pmc_nyu_b1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_nyu_b1 -o bench --output-format csv -- \
    python3 $R/bench.py --config nyu_b1 --steps 20 --warmup 5 --no-cpu-baseline --no-backward --no-gru --no-heads \
    --no-extra-configs > $O/stats_nyu_b1.log 2>&1 || exit 1
