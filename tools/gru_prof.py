"""GRU-mode section timing (the reference's forced default, src/config.py:225-228) at
NYU B=8: NLSPNModel.propagate_heads with use_GRU on synthetic head outputs, eager, with
MIOpen's default algorithm choice vs torch.backends.cudnn.benchmark (MIOpen find mode).
usage: python tools/gru_prof.py [--bench 0|1] [--steps N]"""
import argparse
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import NLSPNModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--cl", type=int, default=0, help="GRU / encode / decode convs in channels_last")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.bench)
    dev = "cuda:0"
    B, H, W, K = a.B, 228, 304, 8
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=18,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True,
                                 network="resnet34", from_scratch=True, zero_init_aff=False, use_GRU=True,
                                 use_S2D=False, GRU_hidden_dim=128, GRU_input_dim=128, lr=1e-3, max_depth=10.0,
                                 patch_height=H, patch_width=W, model_name="NLSPN")
    torch.manual_seed(0)
    m = NLSPNModel(args).to(dev).eval()
    if a.cl:
        for sub in (m.GRU, m.encode_aff, m.encode_dep, m.decode_aff):
            sub.to(memory_format=torch.channels_last)
    g = torch.Generator(device=dev).manual_seed(1)
    pred_init = torch.rand((B, 1, H, W), device=dev, generator=g) * 10
    dep = pred_init * (torch.rand((B, 1, H, W), device=dev, generator=g) < 0.01)
    off_aff = torch.randn((B, 3 * K, H, W), device=dev, generator=g)
    conf = torch.rand((B, 1, H, W), device=dev, generator=g)
    with torch.no_grad():
        for _ in range(3):
            m.propagate_heads(pred_init, off_aff, conf, dep)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            m.propagate_heads(pred_init, off_aff, conf, dep)
        e1.record()
        torch.cuda.synchronize()
    print(json.dumps({"cudnn_benchmark": bool(a.bench), "channels_last": bool(a.cl), "B": B, "ms_per_section": e0.elapsed_time(e1) / a.steps}),
          flush=True)


if __name__ == "__main__":
    main()
