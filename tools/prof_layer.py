"""Run ONE fused quantize+conv layer a few times (for rocprofv3 kernel traces /
PMC counters).  Shape defaults to ResNet56 stage 1 @224, bs=256.

    python tools/prof_layer.py --shape 16,224,16,3,1,1 --iters 5 [--plan I | --tile NJ,TP,TQ]

Without --plan / --tile the layer is autotuned first (as bench.py does), so the
profiled kernel is the plan the bench runs.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16,224,16,3,1,1", help="C,H,K,R,stride,pad")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tile", default=None)
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--plan", type=int, default=None, help="candidate plan index (po2q_qconv2d_plans)")
    ap.add_argument("--pair", action="store_true", help="the conv pair kernel (conv_pair<C>: stage 1 or 2) instead")
    args = ap.parse_args()
    if args.tile:
        os.environ["PO2Q_X3_TILE"] = args.tile
    from po2_quantization_amd import _lib

    C, H, K, R, st, pad = (int(v) for v in args.shape.split(","))
    dev = torch.device("cuda:0")
    if args.pair:  # PLAN key = the bench's roofline traffic key for the pair (C = 16 or 32 from --shape)
        x = torch.randn(args.batch, C, H, H, device=dev)
        w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        print("PLAN pair%d %dx%d bs=%d" % (C, H, H, args.batch), flush=True)
        for _ in range(args.iters):
            _lib.qconv2d_pair(x, w1, w2, 4, "po2")
        torch.cuda.synchronize()
        return
    x = torch.randn(args.batch, C, H, H, device=dev)
    w = torch.randn(K, C, R, R, device=dev) * 0.1
    key = (args.batch, C, H, H, K, R, R, st, st, pad, pad, 1, 1, 1, 4, 1, 1, _lib.PRECISIONS[args.precision])
    if args.plan is None and not args.tile and _lib._saved_plan(key) is not None:
        args.plan = _lib._saved_plan(key)  # the plan bench.py tuned (PO2Q_TUNE_FILE)
    if args.plan is None and not args.tile:
        _lib.benchmark = True
        _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", 1, args.precision)  # autotune
        _lib.benchmark = False
    desc = _lib.describe(args.batch, C, H, H, K, R, R, st, pad, precision=args.precision)
    if args.plan is not None:
        desc = _lib.plans(args.batch, C, H, H, K, R, R, st, pad, precision=args.precision)[args.plan]
    print("PLAN " + desc, flush=True)
    for _ in range(args.iters):
        _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", 1, args.precision, plan=args.plan)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
