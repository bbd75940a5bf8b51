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


def tick(row, key, fn, iters):
    row[key] = round(timeit(fn, iters), 4)
    print("  ", key, row[key], file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--miopen-find", action="store_true")
    args = ap.parse_args()
    # MIOpen immediate mode (an exhaustive find at these sizes runs for minutes on a fresh box)
    torch.backends.cudnn.benchmark = args.miopen_find
    _lib.benchmark = True
    dev = torch.device("cuda:0")
    for (C, H, K, R, st, pad) in [(16, args.image, 16, 3, 1, 1), (32, args.image // 2, 32, 3, 1, 1),
                                  (64, args.image // 4, 64, 3, 1, 1), (16, args.image, 32, 3, 2, 1),
                                  (32, args.image // 2, 64, 1, 2, 0)]:
        N = args.batch
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        w = torch.randn(K, C, R, R, device=dev) * 0.1
        P = (H + 2 * pad - R) // st + 1
        gy = torch.randn(N, K, P, P, device=dev)
        qw = _lib.quantize(w, 4, "po2")
        print("shape", C, H, K, R, st, file=sys.stderr, flush=True)
        row = {"C": C, "H": H, "K": K, "R": R, "stride": st, "batch": N}
        tick(row, "wgrad_native_ms", lambda: _lib.conv_wgrad(x, gy, w.shape, st, pad), args.iters)
        tick(row, "wgrad_miopen_ms", lambda: torch.ops.aten.convolution_backward(
            gy, x, qw, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False]), args.iters)
        if st == 1:
            wt = w.flip(2, 3).transpose(0, 1).contiguous()
            tick(row, "dgrad_native_ms", lambda: _lib.qconv2d(gy, wt, None, 1, R - 1 - pad, 1, 1, 4, "po2"), args.iters)
        tick(row, "dgrad_miopen_ms", lambda: torch.ops.aten.convolution_backward(
            gy, x, qw, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False]), args.iters)
        print(json.dumps(row), flush=True)
        del x, w, gy, qw


if __name__ == "__main__":
    main()
