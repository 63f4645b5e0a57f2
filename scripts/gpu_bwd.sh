set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_backward.py tests/test_gpu_model.py -x -q -p no:cacheprovider > $O/pytest_bwd.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nyu.json 2> $O/bench_nyu.err &&
timeout -k 10 300 python bench.py --config kitti --no-cpu-baseline > $O/bench_kitti.json 2> $O/bench_kitti.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o nyu --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_nyu.log 2>&1
