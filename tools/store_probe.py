"""Store-pattern probe driver (tuning aid, GPU only): times tools/store_probe.hip's
row-marching store patterns against a contiguous fill of the same bytes.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/store_probe.hip -o tools/libstore_probe.so"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.tile_sweep import timeit  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "tools", "libstore_probe.so"))
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 9


def run(y, mode, N, C, H, W, SW=32, RB=112, bar=1, nt=0, x=None):
    def f():
        assert L.probe_launch(y.data_ptr(), 0 if x is None else x.data_ptr(), mode, N, C, H, W, SW, RB, bar, nt) == 0
    return timeit(f, 7)


def main():
    N = 256
    for (C, H) in ((32, 112), (16, 224), (64, 56)):
        y = torch.empty(N, C, H, H, device="cuda")
        x = torch.randn(N, C, H, H, device="cuda")
        res = {"C": C, "H": H, "copy": timeit(lambda: y.copy_(x), 7)}
        for SW in (16, 32, 64, 128, 256):
            if SW // 4 > 64 or (C // 4) % max(1, 64 // (SW // 4)) != 0:
                continue
            for RB in (16, H):
                res["ld_SW%d_RB%d" % (SW, RB)] = run(y, 2, N, C, H, H, SW, RB, 1, 0, x)
                res["dma_SW%d_RB%d" % (SW, RB)] = run(y, 2, N, C, H, H, SW, RB, 1, 2, x)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        del y, x


if __name__ == "__main__":
    main()
