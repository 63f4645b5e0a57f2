#!/bin/bash
# HBM-side bytes by request size (gfx950): FETCH_SIZE tallies every read request at 64 B,
# so a blanket x2 for 128-B streaming requests over-counts narrow (64-B) reads.  Two passes
# per config: TCC_EA0_RDREQ {all, 32B, 64B, 128B} and TCC_EA0_WRREQ {all, 64B};
# read bytes = 32 R32 + 64 R64 + 128 R128, write bytes = 64 W64 + 32 (W - W64); a third pass
# splits the requests that reach DRAM (TCC_EA0_*REQ_DRAM) from those the MALL serves.
# usage: scripts/gpu_pmc_req.sh TAG CFG...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcreq_$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in "$@"; do
  for P in "rd:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "wr:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "dram:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"; do
    tag=${P%%:*}; C=${P#*:}
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/${CFG}_$tag -o run --output-format csv -- \
        python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-backward --no-gru \
        --no-extra-configs --no-heads --kernel-reps 5 > $O/${CFG}_$tag.log 2>&1 || { tail -20 $O/${CFG}_$tag.log; exit 1; }
  done
done
