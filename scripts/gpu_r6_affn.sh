set -o pipefail
mkdir -p gpurun_out/affn
timeout -k 10 600 python -u -m pytest tests/test_gpu_gru.py tests/test_backward_golden.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/affn/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/affn/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/affn/bench.json 2> gpurun_out/affn/bench.err || { tail -5 gpurun_out/affn/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/affn/bench.json'));print(d['value'], {k: v['value'] for k, v in d['configs'].items()}, d.get('gru_section'))"
