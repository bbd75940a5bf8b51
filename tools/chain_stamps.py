"""Phase stamps of the small-image chain kernel (diagnostic build lib_chainstamps, `make -C
po2_quantization_amd/csrc chainstamps`): s_memtime cycle sums per phase (prologue, MFMA, barrier,
epilogue, barrier) averaged per layer and wave, printed by the library to stderr, for config 2's
three stage runs (bs 256, BasicBlock form, then the plain form: no residual held).  ctypes on the C ABI of lib_chainstamps; torch only for
device buffers.  GPU only."""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "po2_quantization_amd", "lib_chainstamps", "libpo2q.so"))
    P, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
    L.po2q_last_error.restype = ctypes.c_char_p
    L.po2q_qconv2d_chain_workspace_bytes.restype = sz
    L.po2q_qconv2d_chain_workspace_bytes.argtypes = [i64] * 4 + [i32]
    L.po2q_qconv2d_chain_f32.argtypes = [P] * 7 + [i32] + [i64] * 4 + [i32] * 3 + [P, P, sz, P]
    os.environ["PO2Q_STAMPS"] = "1"
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    import sys
    for form, C, H, n in [(f, C, H, n) for f in ("basic", "plain") for C, H, n in ((16, 32, 17), (32, 16, 17), (64, 8, 17))]:
        print("[chain_stamps] form %s C=%d" % (form, C), file=sys.stderr, flush=True)
        N = 256
        x = torch.relu(torch.randn(N, C, H, H, device=dev))
        ws = [torch.randn(C, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5) for _ in range(n)]
        ps = [torch.rand(C, device=dev) + 0.5 for _ in range(n)]
        pb = [torch.randn(C, device=dev) * 0.1 for _ in range(n)]
        arr = lambda ts: (P * n)(*[t.data_ptr() for t in ts])
        acts = (i32 * n)(*([1] * n))
        res = (i32 * n)(*[-1 if l % 2 == 0 or form == "plain" else l - 1 for l in range(n)])
        y = torch.empty_like(x)
        nb = L.po2q_qconv2d_chain_workspace_bytes(N, C, H, H, n)
        wsp = torch.empty(max(nb, 256), dtype=torch.uint8, device=dev)
        for _ in range(2):
            st = L.po2q_qconv2d_chain_f32(x.data_ptr(), arr(ws), None, arr(ps), arr(pb), acts, res, n, N, C, H, H, 4,
                                          1, 1, y.data_ptr(), wsp.data_ptr(), max(nb, 256), stream)
            assert st == 0, L.po2q_last_error()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
