"""Per-layer timing of the fused quantize+conv op for every distinct conv shape
of a model at a given batch/resolution (HIP events, median of --iters).

    python tools/layer_bench.py --model resnet56 --image 224 --batch 256
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import conv_work, resnet_qconv_layers  # noqa: E402
from po2_quantization_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet56")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--mode", default="po2")
    ap.add_argument("--torch", action="store_true", help="also time torch F.conv2d (MIOpen) on the same shapes")
    ap.add_argument("--tune", action="store_true", help="autotune each shape first (cudnn.benchmark counterpart)")
    args = ap.parse_args()
    if args.tune:
        _lib.benchmark = True
    nb = {"resnet20": 3, "resnet32": 5, "resnet44": 7, "resnet56": 9}[args.model]
    dev = torch.device("cuda:0")
    seen, shapes, H = {}, [], args.image
    blk_in = blk_out = H
    for name, C, K, R, st, pad, role in resnet_qconv_layers(nb):
        if role == "conv1":
            blk_in, blk_out = H, (H + 2 * pad - R) // st + 1
            H = blk_out
        key = (C, K, R, st, pad, blk_out if role == "conv2" else blk_in)
        if key not in seen:
            seen[key] = 0
            shapes.append(key)
        seen[key] += 1
    total_ms = 0.0
    res = []
    for (C, K, R, st, pad, Hin) in shapes:
        x = torch.randn(args.batch, C, Hin, Hin, device=dev)
        w = torch.randn(K, C, R, R, device=dev) * 0.1
        for _ in range(3):
            _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, args.mode, 1, args.precision)
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, args.mode, 1, args.precision)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]
        flops, nbytes = conv_work(args.batch, C, Hin, K, R, st, pad)
        cnt = seen[(C, K, R, st, pad, Hin)]
        total_ms += ms * cnt
        row = dict(C=C, K=K, R=R, stride=st, H=Hin, count=cnt, ms=round(ms, 4),
                   tflops=round(flops / ms / 1e9, 2), gbs=round(nbytes / ms / 1e6, 1))
        if args.torch:
            qw = _lib.quantize(w, 4, args.mode)
            for _ in range(3):
                torch.nn.functional.conv2d(x, qw, None, st, pad)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                torch.nn.functional.conv2d(x, qw, None, st, pad)
            e1.record()
            torch.cuda.synchronize()
            row["torch_ms"] = round(e0.elapsed_time(e1) / args.iters, 4)
        res.append(row)
        print(json.dumps(row), flush=True)
        del x, w
    print(json.dumps({"total_qconv_ms": round(total_ms, 3), "images_per_s": round(args.batch / total_ms * 1e3, 1)}))


if __name__ == "__main__":
    main()
