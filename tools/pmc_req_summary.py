"""Per-kernel HBM / fabric bytes from the request-size PMC passes of scripts/gpu_pmc_req.sh.

gfx950 counts L2 -> fabric (EA) read requests by width (TCC_EA0_RDREQ_32B/_64B/_128B) and
the subset that reaches DRAM (TCC_EA0_RDREQ_DRAM; the rest is served by the MALL /
Infinity Cache), likewise for writes.  Per launch:
  fabric read  = 32 R32 + 64 R64 + 128 R128          (all L2 misses, MALL hits included)
  fabric write = 64 W64 + 32 (W - W64)
  DRAM read    = fabric read  x RDREQ_DRAM / RDREQ   (same request mix assumed)
  DRAM write   = fabric write x WRREQ_DRAM / WRREQ
usage: python tools/pmc_req_summary.py DIR CFG [--json OUT]"""
import argparse
import collections
import csv
import json
import os


def passes(d, cfg):
    out = collections.defaultdict(dict)
    for tag in ("rd", "wr", "dram"):
        f = os.path.join(d, f"{cfg}_{tag}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"] + ("@" + tag if tag == "dram" else "")].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            for c, x in v.items():
                out[k][c] = sum(x) / len(x)
    return out


def summarize(d, cfg):
    res = {}
    for k, v in passes(d, cfg).items():
        if "prop_" not in k:
            continue
        R32, R64, R128 = (v.get(f"TCC_EA0_RDREQ_{w}B_sum", 0.0) for w in (32, 64, 128))
        W, W64 = v.get("TCC_EA0_WRREQ_sum", 0.0), v.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        rd = 32 * R32 + 64 * R64 + 128 * R128
        wr = 64 * W64 + 32 * (W - W64)
        Rd, RdD = v.get("TCC_EA0_RDREQ_sum@dram", 0.0), v.get("TCC_EA0_RDREQ_DRAM_sum@dram", 0.0)
        Wd, WdD = v.get("TCC_EA0_WRREQ_sum@dram", 0.0), v.get("TCC_EA0_WRREQ_DRAM_sum@dram", 0.0)
        fr = RdD / Rd if Rd else None
        fw = WdD / Wd if Wd else None
        res[k] = {"fabric_read_bytes": round(rd), "fabric_write_bytes": round(wr),
                  "fabric_bytes": round(rd + wr),
                  "dram_read_fraction": None if fr is None else round(fr, 4),
                  "dram_write_fraction": None if fw is None else round(fw, 4),
                  "dram_bytes": None if fr is None or fw is None else round(rd * fr + wr * fw),
                  "req_128b_share": round(R128 / max(1.0, R32 + R64 + R128), 4)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("cfg")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = summarize(a.dir, a.cfg)
    for k, v in res.items():
        print(a.cfg, k[:72], json.dumps(v))
    if a.json:
        json.dump({"config": a.cfg, "kernels": res}, open(a.json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
