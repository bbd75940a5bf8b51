"""Timing ablation of the stage-2 pair kernel (po2q_conv_pairw.hip, 32 -> 32 -> 32 @112, bs 256, plain form)
on the diagnostic build (make -C po2_quantization_amd/csrc pairwdiag): PO2Q_PAIR_W32_DBG bits 1 no MFMAs,
2 no x DMAs, 4 no stores, 8 no epilogue / split vector work, 16 no per-step barrier.  Calls
po2q_qconv2d_pair_f32 of lib_pairwdiag/libpo2q.so through ctypes on torch's stream; the ablated outputs are
meaningless, only their times are.  Interleaved rounds, medians; PO2Q_PAIR_W32=0 times conv_pair<32>."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.tile_sweep import timeit  # noqa: E402


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "po2_quantization_amd", "lib_pairwdiag", "libpo2q.so"))
    i64, i32, p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
    L.po2q_qconv2d_pair_f32.argtypes = [p, p, p, p, i64, i64, i64, i64, i32, i32, i32, p, p, p, p, i32, p, p, p, i32, p]
    L.po2q_qconv2d_pair_f32.restype = i32
    N, C, H = 256, 32, 112
    dev = torch.device("cuda:0")
    x = torch.relu(torch.randn(N, C, H, H, device=dev))
    w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    y = torch.empty_like(x)

    def call():
        st = L.po2q_qconv2d_pair_f32(x.data_ptr(), w1.data_ptr(), w2.data_ptr(), y.data_ptr(), N, C, H, H, 4, 1, 1,
                                     None, None, None, None, 0, None, None, None, 0,
                                     torch.cuda.current_stream().cuda_stream)
        assert st == 0, st

    arms = os.environ.get("PAIRW_DBG", "old,0,1,2,4,6,8,9,16,15,14,7,24").split(",")
    ts = {}
    for _ in range(3):
        for v in arms:
            os.environ.pop("PO2Q_PAIR_W32_DBG", None)
            os.environ["PO2Q_PAIR_W32"] = "0" if v == "old" else "2"
            if v not in ("old", "0"):
                os.environ["PO2Q_PAIR_W32_DBG"] = v
            ts.setdefault(v, []).append(timeit(call, 7))
    out = {k: round(sorted(t)[len(t) // 2], 4) for k, t in ts.items()}
    out["copy_in_bytes_ms"] = round(timeit(lambda: y.copy_(x), 7), 4)
    print(json.dumps({"pairw_ablation_ms": out, "bits": "1 no MFMA, 2 no x DMA, 4 no stores, 8 no epilogue/split "
                      "VALU, 16 no barrier; old = conv_pair<32>"}), flush=True)


if __name__ == "__main__":
    main()
