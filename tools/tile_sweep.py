"""Time every candidate plan (po2q_qconv2d_plans: both bf16x3 kernels, ranked tile
shapes) for each distinct ResNet56 qconv shape at the bench configuration, and
what the autotuner picks.  Tuning aid, GPU only; one JSON line per shape."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402

SHAPES = [(16, 224, 16, 3, 1, 1), (16, 224, 32, 3, 2, 1), (16, 224, 32, 1, 2, 0), (32, 112, 32, 3, 1, 1),
          (32, 112, 64, 3, 2, 1), (32, 112, 64, 1, 2, 0), (64, 56, 64, 3, 1, 1),
          # ResNet56 @32 (config 2) stride-1 shapes: indices 7, 8, 9
          (16, 32, 16, 3, 1, 1), (32, 16, 32, 3, 1, 1), (64, 8, 64, 3, 1, 1)]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    ev = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    return sorted(x.elapsed_time(y) for x, y in ev)[iters // 2]


def short(desc):
    f = dict(kv.split("=") for kv in desc.split())
    k = ("dma%s%s%s" % (f["waves"], "ov" if f.get("ov") == "1" else "", "" if f.get("wstream") != "0" else "wr")
         if f["kind"] == "bf16x3_dma" else ("reg" if f["kind"] == "bf16x3" else f["kind"]))
    return "%s NJ=%s vr=%s pd=%s nts=%s var=%s fp=%s %s" % (k, f["NJ"], f["vr"], f.get("pd", "0"), f.get("nts", "0"),
                                                            f.get("var", "0"), f.get("fp", "0"), f["tile"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--rounds", type=int, default=3, help="interleaved passes over the plans (median reported)")
    ap.add_argument("--warm-ms", type=float, default=1500.0, help="GPU warm-up before timing (clock ramp)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    shapes = SHAPES if args.shapes == "all" else [SHAPES[int(i)] for i in args.shapes.split(",")]
    for (C, H, K, R, st, pad) in shapes:
        x = torch.randn(args.batch, C, H, H, device=dev)
        w = torch.randn(K, C, R, R, device=dev) * 0.1
        P = (H + 2 * pad - R) // st + 1
        plans = _lib.plans(args.batch, C, H, H, K, R, R, st, pad)
        # warm the GPU up first: the first plans of a cold GPU run at ramping clocks
        import time
        t_end = time.time() + args.warm_ms / 1e3
        while time.time() < t_end:
            for _ in range(10):
                _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", plan=0)
            torch.cuda.synchronize()
        ts = [[] for _ in plans]
        for _ in range(args.rounds):  # interleaved, so drift hits every plan alike
            for i in range(len(plans)):
                ts[i].append(timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", plan=i), args.iters))
        res = [(sorted(t)[len(t) // 2], i, short(d)) for i, (t, d) in enumerate(zip(ts, plans))]
        _lib.benchmark = True
        _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2")  # autotune
        _lib.benchmark = False
        tuned = _lib.describe(args.batch, C, H, H, K, R, R, st, pad)
        t_tuned = timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2"), args.iters)
        flops = 2.0 * args.batch * K * P * P * C * R * R
        nbytes = 4.0 * (args.batch * C * H * H + args.batch * K * P * P + K * C * R * R)
        print(json.dumps({"shape": [C, H, K, R, st], "default": short(plans[0]), "default_ms": round(res[0][0], 4),
                          "tuned": short(tuned), "tuned_ms": round(t_tuned, 4),
                          "tuned_GBs": round(nbytes / t_tuned / 1e6, 1),
                          "tuned_TFs": round(flops / t_tuned / 1e9, 1),
                          "plans": [(round(r[0], 4), r[1], r[2]) for r in sorted(res)]}), flush=True)
        del x, w


if __name__ == "__main__":
    main()
