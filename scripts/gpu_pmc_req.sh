#!/bin/bash
# HBM read bytes by request size (gfx950: FETCH_SIZE tallies 128-B requests at 64 B, so the
# blanket x2 correction over-counts narrow reads): TCC_EA0_RDREQ (all), _32B and TCC_BUBBLE
# (128-B requests) in one pass per config.  bytes = 32*R32 + 64*(R - R32 - BUB) + 128*BUB.
# usage: scripts/gpu_pmc_req.sh TAG CFG...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcreq_$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --kernel-trace -d $O/$CFG -o run \
      --output-format csv -- python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
      --no-extra-configs --no-heads --kernel-reps 5 > $O/$CFG.log 2>&1 || { tail -20 $O/$CFG.log; exit 1; }
done
