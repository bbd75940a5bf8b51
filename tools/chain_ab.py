"""A/B of the chain kernel's variants (PO2Q_CHAIN_VARIANT) on config 2's three stage runs, one
process, interleaved rounds, HIP-event medians of graph-captured back-to-back launches."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from po2_quantization_amd import _lib

    dev = torch.device("cuda:0")
    variants = [int(v) for v in os.environ.get("CHAIN_VARIANTS", "0,1,2,3").split(",")]
    out = {}
    for stage, (C, H, n) in {1: (16, 32, 18), 2: (32, 16, 17), 3: (64, 8, 17)}.items():
        torch.manual_seed(stage)
        x = torch.relu(torch.randn(256, C, H, H, device=dev))
        ws = [torch.randn(C, C, 3, 3, device=dev) * 0.1 for _ in range(n)]
        res = {v: [] for v in variants}
        for _ in range(5):
            for v in variants:
                os.environ["PO2Q_CHAIN_VARIANT"] = str(v)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                _lib.qconv2d_chain(x, ws, 4, "po2")
                e0.record()
                for _ in range(10):
                    _lib.qconv2d_chain(x, ws, 4, "po2")
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / 10)
        out["stage%d" % stage] = {v: round(sorted(t)[len(t) // 2], 4) for v, t in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
