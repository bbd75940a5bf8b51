"""Probe: bench.py's ResNet56 @224 chain with the batch split into S micro-batches on S HIP streams
(each micro-batch walks every layer on its own stream; the weight packs of each chain object run
on its stream).  The stages differ in what bounds them (stage 1 HBM, stages 2 / 3 the matrix
cores), so micro-batches in different stages at the same time can overlap the two.  Prints the
interleaved median ms per full-batch step for each split count and whether the logits match the
single-stream run bit for bit.

    python tools/split_stream_probe.py [splits=1,2,4] [rounds=3] [steps=20]
    SPLIT_SEQ=1: the micro-batches one after another on one stream (chunk-major: a stage-3 or
    stage-2 activation of a micro-batch fits the 256 MB MALL between consecutive layers)
"""
import json
import os
import sys

import torch

SEQ = False

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from po2_quantization_amd import _lib  # noqa: E402


def main():
    global SEQ
    SEQ = os.environ.get("SPLIT_SEQ", "0") == "1"
    splits = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda:0")
    _lib.benchmark = True
    B, H = 256, 224
    x = torch.relu(torch.randn(B, 16, H, H, generator=torch.Generator().manual_seed(100))).to(dev)
    runs = {}
    for S in splits:
        parts = list(x.chunk(S))
        chains = []
        for p in parts:
            c = bench.QConvChain(9, 1000, "po2", 4, "auto", dev, seed=0)
            c.timed_layer = -1
            with torch.no_grad():
                c.forward(p)
                torch.cuda.synchronize()
            c.enable_packed()
            chains.append(c)
        streams = [torch.cuda.Stream() for _ in parts]

        def step(chains=chains, parts=parts, streams=streams):
            if SEQ:  # chunk-major on one stream: each micro-batch walks every layer before the next starts
                return torch.cat([c.forward(p) for c, p in zip(chains, parts)])
            cur = torch.cuda.current_stream()
            outs = []
            for c, p, s in zip(chains, parts, streams):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    outs.append(c.forward(p))
            for s in streams:
                cur.wait_stream(s)
            return torch.cat(outs)

        runs[S] = step
    res = {S: [] for S in splits}
    with torch.no_grad():
        ref = runs[splits[0]]()
        same = {S: bool(torch.equal(runs[S](), ref)) for S in splits}
        for _ in range(rounds):
            for S in splits:
                for _ in range(3):
                    runs[S]()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(steps):
                    runs[S]()
                e1.record()
                torch.cuda.synchronize()
                res[S].append(e0.elapsed_time(e1) / steps)
                print(json.dumps({"splits": S, "ms_per_step": round(res[S][-1], 3)}), flush=True)
    for S in splits:
        ts = sorted(res[S])
        ms = ts[len(ts) // 2]
        print(json.dumps({"splits": S, "median_ms": round(ms, 3), "img_s": round(B / ms * 1e3, 1),
                          "bitwise_equal_1": same[S]}), flush=True)


if __name__ == "__main__":
    main()
