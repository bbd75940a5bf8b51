"""Timing ablation of the bf16x3 conv kernel (PO2Q_X3_DEBUG bits: 1 no MFMA,
2 no split, 4 no x loads, 8 no stores) for one layer shape / tile.  Outputs of
the ablated runs are meaningless; only their time is.  GPU only."""
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
    ap.add_argument("--shape", default="16,224,16,3,1,1")
    ap.add_argument("--tile", default=None)
    ap.add_argument("--plans", default=None, help="comma-separated candidate plan indices (default: heuristic plan)")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--var", default="PO2Q_X3_DEBUG", help="ablation switch (PO2Q_ROWS_DEBUG for the row kernel)")
    ap.add_argument("--values", default="0,1,2,3,4,8,12,5,7,9,11,13,14,15")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved repetitions (median reported)")
    args = ap.parse_args()
    C, H, K, R, st, pad = (int(v) for v in args.shape.split(","))
    if args.tile:
        os.environ["PO2Q_X3_TILE"] = args.tile
    dev = torch.device("cuda:0")
    x = torch.randn(args.batch, C, H, H, device=dev)
    w = torch.randn(K, C, R, R, device=dev) * 0.1
    plans = [None] if args.plans is None else [int(p) for p in args.plans.split(",")]
    descs = _lib.plans(args.batch, C, H, H, K, R, R, st, pad)
    for pl in plans:
        res = {"plan": _lib.describe(args.batch, C, H, H, K, R, R, st, pad) if pl is None else descs[pl]}
        ts = {}
        for _ in range(args.rounds):  # interleaved, so drift between rounds hits every value alike
            for dbg in (int(v) for v in args.values.split(",")):
                os.environ[args.var] = str(dbg)
                t = timeit(lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", plan=pl), 7)
                ts.setdefault(str(dbg), []).append(t)
        for k, v in ts.items():
            res[k] = round(sorted(v)[len(v) // 2], 4)
        os.environ.pop(args.var)
        print(json.dumps(res), flush=True)
    res = {}
    # reference points: torch copy of the same bytes
    y = torch.empty_like(x)
    res["copy_in_bytes_ms"] = round(timeit(lambda: y.copy_(x), 7), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
