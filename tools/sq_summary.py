"""Summarise rocprofv3 --pmc counter CSVs (one or more passes) per kernel: the mean of each
counter per dispatch, plus the derived ratios the verdicts ask for (LDS bank-conflict share,
VALU / LDS instructions per wave, wait shares).
usage: python tools/sq_summary.py OUT.json PASS_CSV [PASS_CSV ...] [--kernel SUBSTR ...]"""
import collections
import csv
import json
import sys


def load(paths, kernels):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        # one dispatch reports one row per counter (summed over dimensions already, or
        # per-dimension rows: those are summed per (dispatch, counter) first)
        acc = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if kernels and not any(s in k for s in kernels):
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            names[key] = k
        for (d, c), v in acc.items():
            per[names[(d, c)]][c].append(v)
    return per


def derive(m):
    g = m.get
    out = {}
    if g("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_share"] = g("SQ_LDS_BANK_CONFLICT", 0) / g("SQ_LDS_IDX_ACTIVE")
    if g("SQ_WAVES"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES"):
            if c in m:
                out[c.lower().replace("sq_", "") + "_per_wave"] = m[c] / m["SQ_WAVES"]
    if g("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                out[c.lower().replace("sq_", "") + "_share"] = m[c] / m["SQ_WAVE_CYCLES"]
    return out


def main(argv):
    out, rest = argv[0], argv[1:]
    kernels = []
    if "--kernel" in rest:
        i = rest.index("--kernel")
        kernels = rest[i + 1:]
        rest = rest[:i]
    per = load(rest, kernels)
    res = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k[:160]] = {"dispatches": {c: len(v) for c, v in cs.items()}, "mean_per_dispatch": m, "derived": derive(m)}
    json.dump({"source": rest, "kernels": res}, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k[:100], json.dumps({a: round(b, 4) for a, b in r["derived"].items()}))


if __name__ == "__main__":
    main(sys.argv[1:])
