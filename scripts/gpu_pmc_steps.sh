#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the step-kernel
# configs C3 (kitti) and C5 (nyu_k16), for the bench's roofline.traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcsteps
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in kitti nyu_k16; do
  for C in FETCH_SIZE WRITE_SIZE; do
    NLSPN_PLAN_GRAPH=1 timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $O/${cfg}_$C -o run --output-format csv -- \
        python3 $R/bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-backward --no-gru --kernel-reps 3 \
        > $O/${cfg}_$C.log 2>&1 || exit 1
  done
done
