"""Conv pair timing (bs=256; ResNet56 @224 stage 1: 16 -> 16 -> 16 @224, stage 2: 32 -> 32 -> 32
@112; po2 4-bit): the one-launch pair kernel
(po2q_qconv2d_pair_f32, every PO2Q_PAIR_VARIANT) against the same two convs as two fused
single-conv launches (the tuned row kernel).  HIP events, interleaved rounds, medians.
Algorithmic bytes of the pair: x in + y out + both weights read twice."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402


def main():
    N = int(os.environ.get("PAIR_N", "256"))
    dev = torch.device("cuda:0")
    _lib.benchmark = True
    variants = os.environ.get("PAIR_VARIANTS", "23,123,20,120").split(",")
    shapes = ((16, 224), (32, 112)) if os.environ.get("PAIR_C32", "1") == "1" else ((16, 224),)
    for C, H in shapes:  # ResNet56 @224 stage 1 and stage 2
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        _lib.qconv2d(x, w1, None, 1, 1, 1, 1, 4, "po2")  # autotune the single-conv plan
        nbytes = 4.0 * (2 * N * C * H * H + 4 * C * C * 9)
        res = {}
        for rnd in range(3):
            for v in variants:
                os.environ["PO2Q_PAIR_VARIANT"] = v
                res.setdefault("pair_" + v, []).append(timeit(lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2"), 11))
            res.setdefault("two_convs", []).append(
                timeit(lambda: _lib.qconv2d(_lib.qconv2d(x, w1, None, 1, 1, 1, 1, 4, "po2"), w2, None, 1, 1, 1, 1, 4,
                                            "po2"), 11))
        os.environ.pop("PO2Q_PAIR_VARIANT", None)
        for k, v in res.items():
            ms = sorted(v)[len(v) // 2]
            print(json.dumps({"kernel": k, "C": C, "H": H, "batch": N, "ms": round(ms, 4),
                              "pair_bytes_hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 3)}), flush=True)
        del x


if __name__ == "__main__":
    main()
