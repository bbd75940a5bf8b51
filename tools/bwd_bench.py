"""Backward-layer timing (QAT): native input gradient (the fused
quantize + conv of dy with the transposed / flipped weight) and native weight gradient
(po2q_qconv2d_wgrad_f32) against torch's convolution_backward (MIOpen) on the same
tensors.  HIP events, median of --iters.  GPU only; one JSON line per shape."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--iters", type=int, default=9)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    _lib.benchmark = True
    dev = torch.device("cuda:0")
    s = args.image // 224 if args.image >= 224 else 1
    for (C, H, K, R, st, pad) in [(16, args.image, 16, 3, 1, 1), (32, args.image // 2, 32, 3, 1, 1),
                                  (64, args.image // 4, 64, 3, 1, 1), (16, args.image, 32, 3, 2, 1),
                                  (32, args.image // 2, 64, 1, 2, 0)]:
        N = args.batch
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        w = torch.randn(K, C, R, R, device=dev) * 0.1
        P = (H + 2 * pad - R) // st + 1
        gy = torch.randn(N, K, P, P, device=dev)
        qw = _lib.quantize(w, 4, "po2")
        row = {"C": C, "H": H, "K": K, "R": R, "stride": st, "batch": N}
        row["wgrad_native_ms"] = round(timeit(lambda: _lib.conv_wgrad(x, gy, w.shape, st, pad), args.iters), 4)
        row["wgrad_miopen_ms"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, qw, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False]), args.iters), 4)
        if st == 1:
            wt = w.flip(2, 3).transpose(0, 1).contiguous()
            row["dgrad_native_ms"] = round(timeit(lambda: _lib.qconv2d(gy, wt, None, 1, R - 1 - pad, 1, 1, 4, "po2"),
                                                  args.iters), 4)
        row["dgrad_miopen_ms"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, qw, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False]), args.iters), 4)
        print(json.dumps(row), flush=True)
        del x, w, gy, qw


if __name__ == "__main__":
    main()
