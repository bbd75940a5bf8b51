"""lin / lin+ quantizer timing: the native per-channel kernel
(po2q_quantize_lin_f32) against the reference's algorithm as plain torch ops on
the same GPU (utils/quantizers.py:59-136, restated here only as the comparison
leg), per distinct ResNet56 / MobileNetV2 weight shape.  GPU only; one JSON line
per shape.  Bytes = 8 per weight (one read, one write): the kernel is launch- and
reduction-latency bound at these sizes, not HBM bound."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402

SHAPES = [(16, 16, 3, 3), (32, 16, 3, 3), (32, 32, 3, 3), (64, 32, 3, 3), (64, 64, 3, 3), (32, 16, 1, 1),
          (64, 32, 1, 1), (144, 24, 1, 1), (960, 160, 1, 1), (960, 1, 3, 3)]


def torch_lin(w, bits, plus, iters=10):
    def qpf(x, d):
        lim = 2 ** (bits - 1) - 1
        return d.view(-1, 1, 1) * torch.clamp(torch.round(x / d.view(-1, 1, 1)), min=-lim, max=lim)
    mx = w.amax(dim=(0, 2, 3))
    mn = w.amin(dim=(0, 2, 3))
    delta = (mx - mn) / (2 ** bits - 1)
    q = qpf(w, delta) / delta.view(-1, 1, 1)
    s = torch.sqrt(torch.tensor(8.0 / 9.0, device=w.device))
    for _ in range(iters):
        delta = torch.sum(q * w, dim=[0, 2, 3]) / torch.sum(q * q, dim=[0, 2, 3])
        delta = 2 ** torch.round(torch.log2(s * delta if plus else delta))
        q = qpf(w, delta) / delta.view(-1, 1, 1)
    return q * delta.view(-1, 1, 1)


def main():
    g = torch.Generator().manual_seed(0)
    for shp in SHAPES:
        w = (torch.randn(shp, generator=g) * 0.05).cuda()
        res = {"shape": list(shp)}
        for qn in ("lin", "lin+"):
            plus = qn == "lin+"
            t_nat = timeit(lambda: _lib.quantize_lin(w, 4, plus), 21)
            t_ref = timeit(lambda: torch_lin(w, 4, plus), 21)
            same = torch.equal(_lib.quantize_lin(w, 4, plus), torch_lin(w, 4, plus))
            res[qn] = {"native_us": round(t_nat * 1e3, 2), "torch_ops_us": round(t_ref * 1e3, 2),
                       "speedup": round(t_ref / t_nat, 1), "GBs": round(8 * w.numel() / t_nat / 1e6, 2),
                       "equal_to_torch_ops": bool(same)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
