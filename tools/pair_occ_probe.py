"""Occupancy probe for the conv pair (C = 16, po2 4-bit): the same pixel count as images of
width 224 (7 waves per block, 1 block per CU), 112 (4 waves, 2 blocks per CU) and 56 (2 waves,
4 blocks per CU).  If the full-width kernel is bound by its per-step barrier locking the waves of
the only block on a CU into one phase, the narrow images run faster per byte.  HIP events,
interleaved rounds, medians; bytes = x in + y out."""
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
    C, H = 16, 224
    w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    cases = []
    for W, N in ((224, 256), (112, 512), (56, 1024)):
        x = torch.relu(torch.randn(N, C, H, W, device=dev))
        cases.append((W, N, x))
    res = {}
    for rnd in range(5):
        for W, N, x in cases:
            res.setdefault((W, N), []).append(timeit(lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2"), 11))
    for (W, N), v in res.items():
        ms = sorted(v)[len(v) // 2]
        nbytes = 4.0 * 2 * N * C * H * W
        print(json.dumps({"W": W, "N": N, "ms": round(ms, 4), "rounds": [round(t, 4) for t in v],
                          "hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
