set -o pipefail
O=gpurun_out/q4; mkdir -p $O
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
