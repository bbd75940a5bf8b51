"""A/B of the small-image chain kernel's plane layouts (PO2Q_CHAIN_VARIANT): the ResNet56 @32
stage-2 / stage-3 stride-1 runs (bs = 256, BasicBlock form) timed per launch with HIP events,
variants interleaved over rounds.  GPU only.

    python tools/chain_ab.py [--variants 0,4] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    shapes = [(256, 16, 32, 32, 17), (256, 32, 16, 16, 17), (256, 64, 8, 8, 17)]
    cases = []
    for N, C, H, W, n in shapes:
        x = torch.relu(torch.randn(N, C, H, W, generator=g)).to(dev)
        ws = [(torch.randn(C, C, 3, 3, generator=g) * (1.0 / (9 * C) ** 0.5)).to(dev) for _ in range(n)]
        ps = [(torch.rand(C, generator=g) + 0.5).to(dev) for _ in range(n)]
        pb = [(torch.randn(C, generator=g) * 0.1).to(dev) for _ in range(n)]
        res = [-1 if l % 2 == 0 else l - 1 for l in range(n)]
        cases.append(((N, C, H, W, n), x, ws, ps, pb, res))
    variants = [v.strip() for v in args.variants.split(",")]
    times = {(c[0], v): [] for c in cases for v in variants}
    for r in range(args.rounds):
        for case in cases:
            shape, x, ws, ps, pb, res = case
            for v in variants:
                os.environ["PO2Q_CHAIN_VARIANT"] = v
                f = lambda: _lib.qconv2d_chain(x, ws, 4, "po2", post_scales=ps, post_shifts=pb,
                                               acts=["relu"] * len(ws), res_from=res)
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[(shape, v)].append(e0.elapsed_time(e1) / args.iters)
    for (shape, v), ts in times.items():
        print(json.dumps({"shape": shape, "variant": v, "ms": [round(t, 4) for t in ts],
                          "best_ms": round(min(ts), 4)}), flush=True)


if __name__ == "__main__":
    main()
