#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (diagnostic tool).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM), so
the HBM-side bytes are estimated as 2*FETCH_SIZE + WRITE_SIZE, and the factor is
checked against a kernel with a known byte count (tools/step_bench's
stream_ceiling: exactly 27 planes read + 1 written per pixel).

usage: pmc_summary.py OUT.json FETCH_counter.csv WRITE_counter.csv [OTHER_counter.csv...]
       pmc_summary.py --bench CONFIG SOURCE OUT.json FETCH_counter.csv WRITE_counter.csv
         writes profiles/pmc_<config>.json in the form bench.py reads (per kernel:
         fetch_kib, write_kib, hbm_bytes_per_launch, launches) from passes over ONE config
"""
import csv
import json
import re
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
            cname = row.get("Counter_Name") or row.get("Counter-Name")
            val = row.get("Counter_Value") or row.get("Counter-Value")
            if not cname or val is None:
                continue
            acc[cname][name].append(float(val))
    return acc


def short(name):
    for pat in (r"prop_step_kernel<[^>]*>", r"prologue_kernel<[^>]*>", r"stream_ceiling<[^>]*>", r"affnorm_kernel<[^>]*>",
                r"mdcn_forward_kernel<[^>]*>"):
        m = re.search(pat, name)
        if m:
            return m.group(0)
    return name[:80]


def bench_format(config, source, out, paths):
    merged = defaultdict(dict)
    for p in paths:
        for cname, per in load(p).items():
            for k, vals in per.items():
                merged[k][cname] = (sum(vals) / len(vals), len(vals))
    kernels = {}
    for k, cs in merged.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs or "copyBuffer" in k or "fillBuffer" in k:
            continue
        f, n = cs["FETCH_SIZE"]
        w, _ = cs["WRITE_SIZE"]
        kernels[k] = {"fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": round((2 * f + w) * 1024),
                      "launches": n, "source": source}
    with open(out, "w") as fh:
        json.dump({"config": config, "kernels": kernels,
                   "note": "HBM-side bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE counts "
                           "half of wide streaming reads, MI355X_MICROARCH.md; factor confirmed on a 27-plane "
                           "calibration kernel in round 1). Counts L2->fabric requests, Infinity-Cache hits "
                           "included."}, fh, indent=1, sort_keys=True)
    for k, r in kernels.items():
        print(k[:90], r["hbm_bytes_per_launch"])


def main():
    if sys.argv[1] == "--bench":
        return bench_format(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])
    out = sys.argv[1]
    merged = defaultdict(dict)
    for p in sys.argv[2:]:
        for cname, per in load(p).items():
            for k, vals in per.items():
                merged[short(k)][cname] = {"mean": sum(vals) / len(vals), "n": len(vals)}
    res = {}
    for k, cs in merged.items():
        r = {c: v["mean"] for c, v in cs.items()}
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["hbm_bytes_est"] = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024
        res[k] = r
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, r in sorted(res.items()):
        print(k, {c: round(v, 1) for c, v in r.items()})


if __name__ == "__main__":
    main()
