set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_resident.py -x -q -p no:cacheprovider > $O/pytest_resident.log 2>&1 &&
timeout -k 10 300 python tools/res_probe.py > $O/probe.log 2>&1
