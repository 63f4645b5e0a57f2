#!/bin/bash
# LDS / issue counters over tools/step_bench (K=16 fp16 and K=8 fp32 variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sbpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for m in k16f16 k8f32; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/$m -o run --output-format csv -- \
      $R/tools/step_bench $m 16 228 304 3 1 2.0 > $O/$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/sbpmc"
for m in ("k16f16", "k8f32"):
    fs = glob.glob(f"{O}/{m}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in fs:
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "prop_step_kernel" not in k and "stream" not in k:
            continue
        print(m, k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
