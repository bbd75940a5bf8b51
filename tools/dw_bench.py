"""Depthwise 3x3 layer timing (MobileNetV2 @32x32, bs=256 -- config 3): the LDS-halo kernel
(plan 0) and the one-output-per-lane kernel (plan 1) against torch's depthwise conv of Q(w)
(MIOpen), fused quantize + conv per call, HIP events, median of --iters.  HBM fraction from
the algorithmic bytes (x in + y out + weight twice).  GPU only; one JSON line per shape."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402

# (C, H, stride): the depthwise layers of MobileNetV2 at 32x32 (reference mobilenet.py cfg)
SHAPES = [(96, 32, 1), (144, 32, 1), (144, 32, 2), (192, 16, 1), (192, 16, 2), (384, 8, 1), (576, 8, 1),
          (576, 8, 2), (960, 4, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=21)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    N = args.batch
    for C, H, st in SHAPES:
        x = torch.randn(N, C, H, H, device=dev)
        w = torch.randn(C, 1, 3, 3, device=dev) * 0.3
        P = (H + 2 - 3) // st + 1
        nbytes = 4.0 * (N * C * H * H + N * C * P * P + 2 * C * 9)
        row = {"C": C, "H": H, "stride": st, "batch": N, "algorithmic_bytes": int(nbytes)}
        for i in range(len(_lib.plans(N, C, H, H, C, 3, 3, st, 1, 1, C, 4, "po2+"))):
            ms = timeit(lambda: _lib.qconv2d(x, w, None, st, 1, 1, C, 4, "po2+", plan=i), args.iters)
            row["plan%d_ms" % i] = round(ms, 4)
            row["plan%d_hbm_frac" % i] = round(nbytes / (ms * 1e-3) / 8e12, 3)
        qw = _lib.quantize(w, 4, "po2+")
        row["torch_ms"] = round(timeit(lambda: torch.nn.functional.conv2d(x, qw, None, st, 1, 1, C), args.iters), 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
