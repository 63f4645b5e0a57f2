# Resident-kernel check on the GPU box: parity tests, then an A/B bench (resident vs per-iteration launches).
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu_resident.py -x -q -p no:cacheprovider > $O/pytest_resident.log 2>&1 &&
NLSPN_RESIDENT=1 timeout -k 10 300 python bench.py --no-backward --steps 50 --warmup 10 --cpu-reps 1 > $O/bench_res.json 2> $O/bench_res.err &&
NLSPN_RESIDENT=0 timeout -k 10 300 python bench.py --no-backward --steps 50 --warmup 10 --cpu-reps 1 > $O/bench_step.json 2> $O/bench_step.err
