set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_step_backward.py tests/test_gpu_model.py -x -q -p no:cacheprovider > $O/pytest_step_bwd.log 2>&1
