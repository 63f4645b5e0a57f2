"""Bank-conflict model of the resident kernel's tap gathers (nlspn_resident.h): for a
bench workload's synthetic offsets, the LDS cycles of every ds_read_b64 footprint read of
one iteration (two 32-lane groups per wave-instruction, bank = dword mod 64, one extra
cycle per extra distinct dword on a bank within a group: MI355X_MICROARCH.md, LDS table)
under a given window row pitch and thread->quad mapping.  Offline design tool only.

usage: python tools/lds_bank_sim.py [--config nyu|kitti] [--pitch 128 136 ...]"""
import argparse
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402

K, REF, KW, CTL, PADX, RY, RXQ = 8, 4, 3, 8, 4, 8, 2
LDS = 160 * 1024


def win_cells(nt):
    return min((LDS - 4 * CTL - 16 * 11 * nt) // 8 // 4 * 4, 32764)


def res_shape(B, H, W, cus=256):
    """nlspn_capi.hip res_shape (the part grid the kernel runs)."""
    W4 = W // 4
    Q = H * W4
    for Bg in range(min(B, cus), 0, -1):
        gmax = min(cus // Bg, max(1, Q // 64))
        best, res = 1e300, None
        for g in range(gmax, max(1, gmax * 3 // 4) - 1, -1):
            for gy in range(1, g + 1):
                if g % gy:
                    continue
                gx = g // gy
                if gy > H or gx > W4:
                    continue
                ph, pq = -(-H // gy), -(-W4 // gx)
                nq = ph * pq
                nt = -(-nq // 64) * 64
                if nt > 768:
                    continue
                fb = (ph + 2 * RY) * (4 * (pq + 2 * RXQ) + 2 * PADX)
                if win_cells(nt) < fb:
                    continue
                rim = ((ph + 18) * (4.0 * pq + 18) - 4.0 * nq) / 4.0
                cost = nq + 0.2 * rim
                if cost < best:
                    best, res = cost, (Bg, gy, gx, nt)
        if res:
            return res
    raise ValueError("no shape")


def part_addresses(offy, offx, H, W, gy, gx, py, px, nt, pitch, order="row"):
    """Per thread (nt) and tap-pixel slot (32): the dword address of the footprint's upper
    pair (fwin / fwinB copy) and the pitch; None where the thread holds no quad."""
    W4 = W // 4
    r0, r1 = py * H // gy, (py + 1) * H // gy
    c0, c1 = px * W4 // gx, (px + 1) * W4 // gx
    nqw = c1 - c0
    nown = (r1 - r0) * nqw
    tid = np.arange(nt)
    if order == "row":
        rr, cc = tid // nqw, tid % nqw
    else:  # "col2": waves cover 32-lane groups of two rows of 16 quads each (experiment)
        raise NotImplementedError(order)
    act = tid < nown
    rr, cc = np.where(act, rr, 0), np.where(act, cc, 0)
    y = r0 + rr
    x0 = 4 * (c0 + cc)
    hs, ws = [], []
    for k in range(K):
        t = k if k < REF else k + 1
        i, jj = t // KW, t % KW
        for e in range(4):
            h = (y - 1 + i).astype(np.float32) + offy[k, y, x0 + e]
            w = (x0 + e - 1 + jj).astype(np.float32) + offx[k, y, x0 + e]
            hs.append(h)
            ws.append(w)
    h = np.stack(hs, 1)
    w = np.stack(ws, 1)
    valid = (h > -1) & (w > -1) & (h < H) & (w < W) & act[:, None]
    hl, wl = np.floor(h).astype(np.int64), np.floor(w).astype(np.int64)
    mn = min(r0, hl[valid].min()); mx = max(r1, (hl[valid] + 1).max())
    cmn = min(4 * c0, wl[valid].min()); cmx = max(4 * c1, (wl[valid] + 1).max())
    rlo, rhi, wq0, wq1 = mn, mx, cmn >> 2, cmx >> 2
    WWp = 4 * (wq1 - wq0 + 1)
    WW = pitch if pitch else WWp + 2 * PADX
    assert WWp + 2 * PADX <= WW, (WWp, WW)
    WC = win_cells(nt)
    assert (rhi - rlo + 1) * WW <= WC, ((rhi - rlo + 1) * WW, WC)
    hl = np.where(valid, hl, rlo)
    wl = np.where(valid, wl, 4 * wq0 - PADX)
    li = (hl - rlo) * WW + wl - 4 * wq0 + PADX
    idx = np.where(li & 1, li + WC - 1, li)
    return CTL + idx, WW, act


def cycles(addr, act):
    """LDS cycles of one ds_read_b64 over a wave (64 lanes): per 32-lane group, the most
    distinct dwords on one bank."""
    tot = 0
    for g in (slice(0, 32), slice(32, 64)):
        a = addr[g][act[g]]
        if a.size == 0:
            continue
        d = np.unique(np.concatenate([a, a + 1]))
        tot += np.bincount(d % 64, minlength=64).max()
    return tot


def simulate(cfg, pitch, parts=8, seed=7240):
    B, H, W = {"nyu": (8, 228, 304), "kitti": (4, 240, 1216)}[cfg]
    Bg, gy, gx, nt = res_shape(B, H, W)
    d = synth(1, H, W, K, seed=seed)
    off = d["off_aff"][0, :2 * K]
    offy, offx = off[0::2], off[1::2]
    tot = ideal = 0
    rng = np.random.default_rng(1)
    for j in rng.choice(gy * gx, size=min(parts, gy * gx), replace=False):
        py, px = divmod(int(j), gx)
        addr, WW, act = part_addresses(offy, offx, H, W, gy, gx, py, px, nt, pitch)
        for wv in range(nt // 64):
            sl = slice(64 * wv, 64 * wv + 64)
            if not act[sl].any():
                continue
            for s in range(32):
                for row in (0, 1):
                    a = addr[sl, s] + row * WW
                    tot += cycles(a, act[sl])
                    ideal += (1 if act[sl][:32].any() else 0) + (1 if act[sl][32:].any() else 0)
    return tot / ideal, (gy, gx, nt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="nyu")
    ap.add_argument("--pitch", type=int, nargs="*", default=[0, 128, 130, 132, 136, 144, 152, 160, 104, 112, 120])
    ap.add_argument("--parts", type=int, default=8)
    a = ap.parse_args()
    for p in a.pitch:
        try:
            f, shp = simulate(a.config, p, a.parts)
            print(f"pitch {p or 'dyn':>4}: {f:.3f} x conflict-free cycles  (grid {shp})")
        except AssertionError as e:
            print(f"pitch {p}: does not fit {e}")


if __name__ == "__main__":
    main()
