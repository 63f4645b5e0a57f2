set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/res_probe.py resident=1 > $O/probe.log 2>&1
