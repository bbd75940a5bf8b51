"""Phase-stamp report of the conv pair (stage-1 16 -> 16 -> 16 @224 and stage-2 32 -> 32 -> 32 @112,
bs = 256, the bench chain's plain form) on the diagnostic build (make -C po2_quantization_amd/csrc
pairstamps): s_memtime stamps around each phase of a step, the cycle sums per wave printed by the
library.  The sched_barriers around each stamp serialize the phases, so read the shares, not the
total.  Calls po2q_qconv2d_pair_f32 of lib_pairstamps/libpo2q.so through ctypes."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "po2_quantization_amd", "lib_pairstamps", "libpo2q.so"))
    i64, i32, p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
    L.po2q_qconv2d_pair_f32.argtypes = [p, p, p, p, i64, i64, i64, i64, i32, i32, i32, p, p, p, p, i32, p, p, p, i32, p]
    L.po2q_qconv2d_pair_f32.restype = i32
    dev = torch.device("cuda:0")
    os.environ["PO2Q_STAMPS"] = "1"
    for C, H in ((16, 224), (32, 112)):
        N = 256
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
        y = torch.empty_like(x)
        for _ in range(2):  # the second run is the warm one
            st = L.po2q_qconv2d_pair_f32(x.data_ptr(), w1.data_ptr(), w2.data_ptr(), y.data_ptr(), N, C, H, H, 4, 1, 1,
                                         None, None, None, None, 0, None, None, None, 0,
                                         torch.cuda.current_stream().cuda_stream)
            assert st == 0, st
        torch.cuda.synchronize()
        sys.stderr.flush()


if __name__ == "__main__":
    main()
