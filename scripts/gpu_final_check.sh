#!/bin/bash
# Driver-shaped final check: smoke() and the default bench command.
set -o pipefail
O=gpurun_out/final_$1; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], {k: v['value'] for k, v in d['configs'].items()})"
