set -o pipefail
O=gpurun_out/q2; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_resident.py -x -q -p no:cacheprovider > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --config kitti --no-backward --no-cpu-baseline > $O/bench_kitti.json 2> $O/bench_kitti.err &&
timeout -k 10 300 python bench.py --config nyu_k16 --no-backward --no-cpu-baseline > $O/bench_k16.json 2> $O/bench_k16.err &&
timeout -k 10 300 python bench.py --no-backward --no-cpu-baseline > $O/bench_nyu.json 2> $O/bench_nyu.err
