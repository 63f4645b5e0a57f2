set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu_dcn.py tests/test_gpu_resident.py -q -p no:cacheprovider > $O/pytest_dcn_res.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_probe_pmc.sh
