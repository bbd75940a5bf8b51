"""Phase stamps of the fused inverted-residual kernel (diagnostic build lib_irstamps, `make -C
po2_quantization_amd/csrc irstamps`): s_memtime cycle sums per phase and wave, averaged over the
blocks, printed by the library to stderr.  Calls the C ABI of lib_irstamps/libpo2q.so through
ctypes (plans, batched pack, po2q_qconv2d_ir_f32); torch only for device buffers.  GPU only.

    python tools/ir_stamps.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = [(256, 32, 32, 16, 16, 1, False), (256, 24, 144, 24, 8, 1, True), (256, 32, 192, 32, 4, 1, True),
          (256, 96, 576, 96, 2, 1, True), (256, 160, 960, 320, 1, 1, True)]


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "po2_quantization_amd", "lib_irstamps", "libpo2q.so"))
    P, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
    L.po2q_last_error.restype = ctypes.c_char_p
    L.po2q_qconv2d_plan_create.argtypes = [ctypes.POINTER(P), i32] + [i64] * 14 + [i32] * 4
    L.po2q_qconv2d_plan_workspace_bytes.restype = sz
    L.po2q_qconv2d_plan_workspace_bytes.argtypes = [P]
    L.po2q_qconv2d_plan_pack_batch.argtypes = [i32, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P),
                                               ctypes.POINTER(sz), P]
    L.po2q_qconv2d_ir_f32.argtypes = [P, P, P, P, sz, P, P, sz, P, P, sz, P, P, i32, P, P, i32, P, P, P, i32, P]
    os.environ["PO2Q_STAMPS"] = "1"
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for N, Cin, Ch, Cout, H, s, expand in SHAPES:
        Ho = (H - 1) // s + 1
        geo = ([(N, Cin, H, H, Ch, 1, 1, 1, 1, 0, 0, 1, 1, 1)] if expand else []) + \
              [(N, Ch, H, H, Ch, 3, 3, s, s, 1, 1, 1, 1, Ch), (N, Ch, Ho, Ho, Cout, 1, 1, 1, 1, 0, 0, 1, 1, 1)]
        ws_shapes = ([(Ch, Cin, 1, 1)] if expand else []) + [(Ch, 1, 3, 3), (Cout, Ch, 1, 1)]
        hs, wts, wss, nb = [], [], [], []
        for g, wsh in zip(geo, ws_shapes):
            h = P()
            assert L.po2q_qconv2d_plan_create(ctypes.byref(h), 0, *g, 4, 1, 1, 0) == 0, L.po2q_last_error()
            hs.append(h)
            wts.append(torch.randn(*wsh, device=dev) * 0.2)
            nb.append(L.po2q_qconv2d_plan_workspace_bytes(h))
            wss.append(torch.empty(max(nb[-1], 256), dtype=torch.uint8, device=dev))
        n = len(hs)
        assert L.po2q_qconv2d_plan_pack_batch(n, (P * n)(*[h.value for h in hs]), (P * n)(*[w.data_ptr() for w in wts]),
                                              (P * n)(*[w.data_ptr() for w in wss]), (sz * n)(*nb), stream) == 0
        x = torch.randn(N, Cin, H, H, device=dev)
        y = torch.empty(N, Cout, Ho, Ho, device=dev)
        he = hs[0] if expand else None
        e_ws = wss[0].data_ptr() if expand else None
        e_nb = nb[0] if expand else 0
        for _ in range(3):  # the last call's stamps are the steady state
            st = L.po2q_qconv2d_ir_f32(x.data_ptr(), y.data_ptr(), he, e_ws, e_nb, hs[-2], wss[-2].data_ptr(), nb[-2],
                                       hs[-1], wss[-1].data_ptr(), nb[-1], None, None, 2, None, None, 2, None, None,
                                       None, 0, stream)
            assert st == 0, L.po2q_last_error()
        torch.cuda.synchronize()
        sys.stderr.flush()


if __name__ == "__main__":
    main()
