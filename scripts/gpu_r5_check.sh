set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/ab_env.py --env NLSPN_RES_TAIL=1 --configs nyu,kitti,nyu_b1 > $O/ab_tail.json 2> $O/ab_tail.err || { tail $O/ab_tail.err; exit 1; }
cat $O/ab_tail.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 120 python tools/res_trace.py --config nyu --out $O/res_trace_nyu.json > $O/res_trace_nyu.log 2>&1 || exit 1
python -c "import json;d=json.load(open('$O/res_trace_nyu.json'));g=d['group0'];print({k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items() if k!='setup'})"
