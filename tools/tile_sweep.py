"""Sweep bf16x3 conv tile shapes (PO2Q_X3_TILE="NJ,TP,TQ") for each distinct
ResNet56 qconv shape at the bench configuration; prints the planner's choice
and every candidate's median time (HIP events).  Tuning aid, GPU only."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402

SHAPES = [(16, 224, 16, 3, 1, 1), (16, 224, 32, 3, 2, 1), (16, 224, 32, 1, 2, 0), (32, 112, 32, 3, 1, 1),
          (32, 112, 64, 3, 2, 1), (32, 112, 64, 1, 2, 0), (64, 56, 64, 3, 1, 1)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--shapes", default="all")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    shapes = SHAPES if args.shapes == "all" else [SHAPES[int(i)] for i in args.shapes.split(",")]
    for (C, H, K, R, st, pad) in shapes:
        x = torch.randn(args.batch, C, H, H, device=dev)
        w = torch.randn(K, C, R, R, device=dev) * 0.1
        P = (H + 2 * pad - R) // st + 1
        os.environ.pop("PO2Q_X3_TILE", None)
        plan = _lib.describe(args.batch, C, H, H, K, R, R, st, pad)
        t_auto = timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2"), args.iters)
        res = []
        # LDS-DMA kernel (po2q_conv_x3p.hip): 4 or 8 waves, tile = 16 * waves * NJ pixels
        for waves in (4, 8):
            os.environ["PO2Q_X3P_WAVES"] = str(waves)
            for nj in (1, 2, 4):
                px = 16 * waves * nj
                cands = [(px // tq, tq, 0) for tq in (4, 8, 16, 32, 64, 128) if px % tq == 0]
                cands += [(nj * (waves // vrx), 16 * vrx, vrx) for vrx in (1, 2, 4, 8) if vrx <= waves]
                for tp, tq, vrx in cands:
                    os.environ["PO2Q_X3P_TILE"] = "%d,%d,%d,%d" % (nj, tp, tq, vrx)
                    d = _lib.describe(args.batch, C, H, H, K, R, R, st, pad)
                    if "bf16x3_dma" not in d or "tile=%dx%d" % (tp, tq) not in d or ("vr=%d" % vrx) not in d:
                        continue
                    t = timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2"), args.iters)
                    res.append((t, "dma%d%s" % (waves, "vr%d" % vrx if vrx else ""), nj, tp, tq))
        os.environ.pop("PO2Q_X3P_TILE", None)
        os.environ.pop("PO2Q_X3P_WAVES", None)
        os.environ["PO2Q_NO_DMA"] = "1"
        for nj in (1, 2, 4, 7):
            px = 64 * nj
            for tq in sorted({8, 16, 32, 56, 64, 112, P, 4}):
                if tq > P or px % tq or px // tq > 2 * P:
                    continue
                os.environ["PO2Q_X3_TILE"] = "%d,%d,%d" % (nj, px // tq, tq)
                try:
                    d = _lib.describe(args.batch, C, H, H, K, R, R, st, pad)
                    if "tile=%dx%d" % (px // tq, tq) not in d:
                        continue
                    t = timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2"), args.iters)
                except RuntimeError as e:
                    continue
                res.append((t, "reg", nj, px // tq, tq))
        os.environ.pop("PO2Q_X3_TILE", None)
        os.environ.pop("PO2Q_NO_DMA", None)
        res.sort(key=lambda r: r[0])
        flops = 2.0 * args.batch * K * P * P * C * R * R
        nbytes = 4.0 * (args.batch * C * H * H + args.batch * K * P * P + K * C * R * R)
        print(json.dumps({"shape": [C, H, K, R, st], "auto_plan": plan, "auto_ms": round(t_auto, 4),
                          "auto_GBs": round(nbytes / t_auto / 1e6, 1),
                          "auto_TFs": round(flops / t_auto / 1e9, 1),
                          "best": [(round(r[0], 4),) + tuple(r[1:]) for r in res[:8]]}), flush=True)
        del x, w


if __name__ == "__main__":
    main()
