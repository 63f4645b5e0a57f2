#!/bin/bash
# Request-size PMC passes (read/write bytes by request width) for every config, and the C5
# step kernel's time against the batch size (grid-tail check).
set -o pipefail
O=gpurun_out/r3k_$1; mkdir -p $O
timeout -k 10 300 python tools/step_batch_scan.py > $O/batch_scan_f16_1x17.json 2> $O/batch_scan.err || { cat $O/batch_scan.err; exit 1; }
cat $O/batch_scan_f16_1x17.json
bash scripts/gpu_pmc_req.sh $1 nyu kitti nyu_b1 nyu_k16 || exit 1
