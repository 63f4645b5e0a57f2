#!/bin/bash
set -o pipefail
O=gpurun_out/grid2; mkdir -p $O
run() {
  ( [ "$2" != "-" ] && export NLSPN_RES_GRID=$2
    timeout -k 10 120 python bench.py --config $1 --no-cpu-baseline --no-backward --no-gru --no-heads --no-extra-configs \
        --steps 200 --warmup 20 > $O/$1_$2_$3.json 2> $O/$1_$2_$3.err ) || exit 1
  python -c "import json;d=json.load(open('$O/$1_$2_$3.json'));print('$1', '$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])" >> $O/summary.txt
}
for r in 1 2; do
  for g in - 16,8 32,4 8,16 64,2; do run kitti $g $r || exit 1; done
done
