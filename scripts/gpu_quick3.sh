set -o pipefail
O=gpurun_out/q3; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider > $O/pytest.log 2>&1
