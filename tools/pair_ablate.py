"""Timing ablation of the conv pair (stage-1 16 -> 16 -> 16 @224, bs = 256) on the diagnostic
build (make -C po2_quantization_amd/csrc pairdiag): PO2Q_PAIR_DEBUG bits 1 no conv-2 MFMAs,
2 no conv-1 MFMAs, 4 no x DMAs, 8 no output stores, 16 no split / epilogue-1 plane writes.
Calls po2q_qconv2d_pair_f32 of lib_pairdiag/libpo2q.so through ctypes on torch's stream;
outputs of the ablated runs are meaningless, only their times are.  Interleaved rounds, medians."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.tile_sweep import timeit  # noqa: E402


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "po2_quantization_amd", "lib_pairdiag", "libpo2q.so"))
    i64, i32, p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
    L.po2q_qconv2d_pair_f32.argtypes = [p, p, p, p, i64, i64, i64, i64, i32, i32, i32, p, p, p, p, i32, p, p, p, i32, p]
    L.po2q_qconv2d_pair_f32.restype = i32
    N = 256
    C = int(os.environ.get("PAIR_C", "16"))
    H = 224 if C == 16 else 112
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

    if C == 16:
        os.environ["PO2Q_PAIR_VARIANT"] = "23"
    vals = [v for v in os.environ.get("PAIR_DBG", "0,3,4,8,12,16,19,15,31").split(",")]
    ts = {}
    for _ in range(3):
        for v in vals:
            os.environ["PO2Q_PAIR_DEBUG"] = v
            ts.setdefault(v, []).append(timeit(call, 7))
    out = {k: round(sorted(t)[len(t) // 2], 4) for k, t in ts.items()}
    out["copy_in_bytes_ms"] = round(timeit(lambda: y.copy_(x), 7), 4)
    print(json.dumps({"C": C, "pair_ablation_ms": out, "bits": "1 no conv2 MFMA, 2 no conv1 MFMA, 4 no x DMA, "
                      "8 no stores, 16 no split/epi1 writes"}), flush=True)


if __name__ == "__main__":
    main()
