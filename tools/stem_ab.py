"""Same-process timing of the unquantized 3-channel stems (ResNet @224 3 -> 16 s1, MobileNetV2 @32
3 -> 32 s2, MobileViT @256 3 -> 16 s2) over every fp32 candidate plan, HIP events, medians of 5 x 11
launches; also the bits of each plan against plan 0.  PO2Q_LIB / ab_old select the build."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("STEM_ROOT", ROOT))
from po2_quantization_amd import _lib  # noqa: E402


def timeit(fn, n=11):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda:0")
    for N, H, K, st in ((256, 224, 16, 1), (256, 32, 32, 2), (64, 256, 16, 2)):
        x = torch.randn(N, 3, H, H, device=dev)
        w = torch.randn(K, 3, 3, 3, device=dev) * 0.2
        plans = _lib.plans(N, 3, H, H, K, 3, 3, st, 1, mode="none")
        ref = _lib.qconv2d(x, w, None, st, 1, 1, 1, 4, "none", plan=0)
        for i, d in enumerate(plans):
            ms = timeit(lambda: _lib.qconv2d(x, w, None, st, 1, 1, 1, 4, "none", plan=i))
            y = _lib.qconv2d(x, w, None, st, 1, 1, 1, 4, "none", plan=i)
            print(json.dumps({"root": os.environ.get("STEM_ROOT", "new"), "shape": [N, H, K, st], "plan": i,
                              "desc": d.split(" tile")[0][-60:], "ms": round(ms, 4),
                              "equal_plan0": bool(torch.equal(y, ref))}), flush=True)


if __name__ == "__main__":
    main()
