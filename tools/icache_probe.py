"""Cold-code probe: is a small kernel's time in its instruction fetch?  Times one conv launch
(a) back to back from a HIP graph (its code stays in the caches) and (b) with a 1 GiB buffer
written between launches (the L2s and most of the Infinity Cache turned over, as a model forward
does between two launches of the same kernel), minus the flush alone.  Plans are every candidate of
the shape (plans()); GPU only, tuning aid.

    python tools/icache_probe.py [case-substring]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from po2_quantization_amd import _lib  # noqa: E402


def graph_ms(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(rounds):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * rounds)


def main():
    dev = torch.device("cuda:0")
    big = torch.empty(256 * 1024 * 1024, device=dev)  # 1 GiB
    flush = lambda: big.fill_(1.0)  # noqa: E731
    t_flush = graph_ms(flush, reps=5)
    cases = [  # (label, x shape, w shape, stride, pad, mode)
        ("mobilenet32 stem 3->32 s2 fp32", (256, 3, 32, 32), (32, 3, 3, 3), 2, 1, "none"),
        ("mobilenet32 last 1x1 320->1280 fp32", (256, 320, 4, 4), (1280, 320, 1, 1), 1, 0, "none"),
        ("mobilenet32 1x1 96->576 @2x2 po2+", (256, 96, 2, 2), (576, 96, 1, 1), 1, 0, "po2+"),
        ("resnet20 3x3 16->16 @32 po2", (256, 16, 32, 32), (16, 16, 3, 3), 1, 1, "po2"),
    ]
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for label, xs, ws, st, pad, mode in cases:
        if only and only not in label:
            continue
        x = torch.randn(*xs, device=dev)
        w = torch.randn(*ws, device=dev) * 0.1
        N, C, H, W = xs
        K, _, R, S = ws
        pl = _lib.plans(N, C, H, W, K, R, S, st, pad, 1, 1, 4, mode)
        for i in range(min(len(pl), 6)):
            run = lambda: _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, mode, plan=i)  # noqa: E731,B023
            warm = graph_ms(run)
            cold = graph_ms(lambda: (flush(), run()), reps=5) - t_flush  # noqa: B023
            print(json.dumps({"case": label, "plan": i, "kind": str(pl[i])[:90], "warm_us": round(warm * 1e3, 2),
                              "cold_us": round(cold * 1e3, 2), "flush_us": round(t_flush * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
