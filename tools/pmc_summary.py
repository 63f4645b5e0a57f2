#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (diagnostic tool).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM), so
the HBM-side bytes are estimated as 2*FETCH_SIZE + WRITE_SIZE, and the factor is
checked against a kernel with a known byte count (tools/step_bench's
stream_ceiling: exactly 27 planes read + 1 written per pixel).

usage: pmc_summary.py OUT.json FETCH_counter.csv WRITE_counter.csv [OTHER_counter.csv...]
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


def main():
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
