#!/bin/bash
# round-4: compile-time window pitch (576-thread builds), 16x64 backward pass-1 tiles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
TESTS="tests/test_gpu_resident.py tests/test_gpu_backward.py tests/test_backward_golden.py tests/test_gpu_parity.py tests/test_gpu_model.py" \
  CFGS="nyu kitti nyu_b1" TRACE="nyu" bash scripts/gpu_exp.sh r4h base=$L/libnlspn_r4base.so r4f=$L/libnlspn_r4f.so cur=- read2=$L/libnlspn_read2.so || exit 1
O=gpurun_out/exp_r4h
for v in small large small large; do
  E=""; [ $v = small ] && E="NLSPN_BWD_TILE=small"
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-gru --no-extra-configs --no-heads --steps 20 --backward-steps 20 \
      > $O/bwd_$v.json 2> $O/bwd_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/bwd_$v.json'));b=d['backward'];print('$v', {k:v for k,v in b.items() if k.startswith('ms')})"
done
