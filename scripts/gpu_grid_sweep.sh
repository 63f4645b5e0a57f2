#!/bin/bash
# Same-box sweep of the resident kernel's part grid (NLSPN_RES_GRID="gy,gx"), C2 and C3.
# usage: scripts/gpu_grid_sweep.sh   (outputs under gpurun_out/grid)
set -o pipefail
O=gpurun_out/grid; mkdir -p $O
run() {  # config grid
  ( [ "$2" != "-" ] && export NLSPN_RES_GRID=$2
    timeout -k 10 120 python bench.py --config $1 --no-cpu-baseline --no-backward --no-gru --no-extra-configs \
        --steps 200 --warmup 20 > $O/$1_$2.json 2> $O/$1_$2.err ) || exit 1
  python -c "import json;d=json.load(open('$O/$1_$2.json'));print('$1', '$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
}
for r in 1 2; do
  for g in - 4,8 8,4 2,16 16,2 32,1; do run nyu $g || exit 1; done
  for g in - 8,16 4,32 16,8 2,64 32,4; do run kitti $g || exit 1; done
done
timeout -k 10 120 python tools/res_trace.py > $O/trace_c2.json 2>&1 && cat $O/trace_c2.json
