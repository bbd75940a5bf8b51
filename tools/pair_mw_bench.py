"""A/B of the conv pair's memory-wave kernel (PO2Q_PAIR_MW = x-ring slots; 0 = the default kernel):
stage-1 pair 16 -> 16 -> 16 @224 and stage-2 pair 32 -> 32 -> 32 @112, bs = 256, the plain chain
form (the bench's); interleaved rounds, median launch times (ms).  GPU only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for C, H, vals in ((16, 224, "0,3,4,5,6"), (32, 112, "0,3,4,5")):
        N = 256
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        ts = {}
        for _ in range(int(os.environ.get("ROUNDS", "4"))):
            for v in os.environ.get("PAIR_MW", vals).split(","):
                if v == "0":
                    os.environ.pop("PO2Q_PAIR_MW", None)
                else:
                    os.environ["PO2Q_PAIR_MW"] = v
                ts.setdefault(v, []).append(timeit(lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2"), 20))
        os.environ.pop("PO2Q_PAIR_MW", None)
        med = {k: round(sorted(t)[len(t) // 2], 4) for k, t in ts.items()}
        print(json.dumps({"pair%d_%d_bs256_ms_by_PO2Q_PAIR_MW" % (C, H): med, "all": ts}), flush=True)
        del x


if __name__ == "__main__":
    main()
