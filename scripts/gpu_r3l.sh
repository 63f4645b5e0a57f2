#!/bin/bash
set -o pipefail
bash scripts/gpu_pmc_req.sh $1 nyu kitti nyu_b1 nyu_k16 || exit 1
