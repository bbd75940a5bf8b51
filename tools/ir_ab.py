"""Per-shape A/B of the fused inverted-residual block (torch.ops.po2q.qconv2d_ir) against its three
layer kernels run one by one from the same packs (qconv2d_packed x 3): every MobileNetV2 block shape
at 32x32 input, bs = 256 (BASELINE config 3), HIP-event time per call, medians over interleaved
rounds.  The packs are made once (both sides read the same workspaces).  GPU only.

    python tools/ir_ab.py [--batch 256] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402

# (Cin, Ch, Cout, H, stride, expand): MobileNetV2 @32 (stem stride 2 -> 16x16)
BLOCKS = [(32, 32, 16, 16, 1, False), (16, 96, 24, 16, 2, True), (24, 144, 24, 8, 1, True),
          (24, 144, 32, 8, 2, True), (32, 192, 32, 4, 1, True), (32, 192, 64, 4, 2, True),
          (64, 384, 64, 2, 1, True), (64, 384, 96, 2, 1, True), (96, 576, 96, 2, 1, True),
          (96, 576, 160, 2, 2, True), (160, 960, 160, 1, 1, True), (160, 960, 320, 1, 1, True)]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    N = args.batch
    for Cin, Ch, Cout, H, s, expand in BLOCKS:
        x = torch.randn(N, Cin, H, H, generator=g).to(dev)
        we = (torch.randn(Ch, Cin, 1, 1, generator=g) / Cin ** 0.5).to(dev) if expand else None
        wd = (torch.randn(Ch, 1, 3, 3, generator=g) * 0.3).to(dev)
        wp = (torch.randn(Cout, Ch, 1, 1, generator=g) / Ch ** 0.5).to(dev)
        bn = [((torch.rand(c, generator=g) + 0.5).to(dev), (torch.randn(c, generator=g) * 0.1).to(dev))
              for c in (Ch, Ch, Cout)]
        Ho = (H - 1) // s + 1
        layers = ([(we, x.shape, 1, 0, 1, 1)] if expand else []) + [(wd, (N, Ch, H, H), s, 1, 1, Ch),
                                                                     (wp, (N, Ch, Ho, Ho), 1, 0, 1, 1)]
        ws = _lib.pack_batch(layers, 4, "po2", plans=[0] * len(layers))
        ws_e, ws_d, ws_p = (ws[0] if expand else None), ws[-2], ws[-1]
        res = x if (s == 1 and Cin == Cout) else None

        def ir():
            return _lib.qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, s, 4, "po2", ps1=bn[0][0], pb1=bn[0][1],
                                   act1="relu6", ps2=bn[1][0], pb2=bn[1][1], act2="relu6", ps3=bn[2][0],
                                   pb3=bn[2][1], residual=res)

        def chain():
            h = x
            if expand:
                h = _lib.qconv2d_packed(x, we, ws_e, None, 1, 0, 1, 1, 4, "po2", post_scale=bn[0][0],
                                        post_shift=bn[0][1], act="relu6", plan=0)
            d = _lib.qconv2d_packed(h, wd, ws_d, None, s, 1, 1, Ch, 4, "po2", post_scale=bn[1][0],
                                    post_shift=bn[1][1], act="relu6", plan=0)
            return _lib.qconv2d_packed(d, wp, ws_p, None, 1, 0, 1, 1, 4, "po2", post_scale=bn[2][0],
                                       post_shift=bn[2][1], residual=res, plan=0)

        a, b = ir(), chain()
        err = float((a - b).abs().max() / b.abs().max())
        graphs = {}
        for name, fn in (("ir", ir), ("layers", chain)):  # replayed from HIP graphs: no host gaps
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                fn()
            torch.cuda.current_stream().wait_stream(st)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                fn()
            graphs[name] = gr
        t = {"ir": [], "layers": []}
        for _ in range(args.rounds):
            t["ir"].append(timed(graphs["ir"].replay, args.iters))
            t["layers"].append(timed(graphs["layers"].replay, args.iters))
        med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in t.items()}
        print(json.dumps({"block": [Cin, Ch, Cout, H, s], "N": N, "ir_us": med["ir"], "layers_us": med["layers"],
                          "normwise": err}), flush=True)


if __name__ == "__main__":
    main()
