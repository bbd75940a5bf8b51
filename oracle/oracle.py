"""ORACLE — test infrastructure only (see po2_oracle.c header).

ctypes/numpy front-end of the C restatement of the reference hot path.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it,
and only as the checker / the timed CPU baseline — never as product code.

  quantize(w, bits, mode, fsr=1)        utils/quantizers.py:19-56
  quantize_lin(w, bits, plus, iters)    utils/quantizers.py:59-136 (lin / lin+)
  sq_error(w, q)                        models/quantized_conv.py:40-45
  conv2d(x, w, b, stride, padding, ...) F.conv2d as called at quantized_conv.py:36,38
  qconv2d(x, w, b, ..., bits, mode)     models/quantized_conv.py:32-38
  cpu_reference_qconv2d(...)            the reference's own CPU path: restated
                                        quantizer + torch CPU F.conv2d (oneDNN), the
                                        same third-party conv the reference calls;
                                        used as bench.py's cpu_baseline
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libpo2oracle.so")
MODES = {"none": 0, "po2": 1, "po2+": 2}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, p = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        L.po2o_quantize.argtypes = [p, p, i64, i32, i32, i32]
        L.po2o_quantize.restype = None
        L.po2o_sq_error.argtypes = [p, p, i64]
        L.po2o_sq_error.restype = ctypes.c_double
        L.po2o_conv2d.argtypes = [p, p, p, p] + [i64] * 14
        L.po2o_conv2d.restype = None
        L.po2o_quantize_lin.argtypes = [p, p, i64, i64, i64, i64, i32, i32, i32]
        L.po2o_quantize_lin.restype = None
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def quantize(w, bits, mode, fsr=1):
    """PO2 ("po2") / PO2+ ("po2+") quantizer, bit-exact with the reference."""
    w = _f32(w)
    out = np.empty_like(w)
    lib().po2o_quantize(_ptr(w), _ptr(out), w.size, int(bits), int(fsr), MODES[mode] - 1)
    return out


def quantize_lin(w, bits, plus, num_iters=10):
    """LinearPowerOfTwo(Plus)Quantizer.forward(None, w, bits, num_iters) for a 4-D fp32
    weight (utils/quantizers.py:59-136)."""
    w = _f32(w)
    assert w.ndim == 4
    out = np.empty_like(w)
    lib().po2o_quantize_lin(_ptr(w), _ptr(out), *w.shape, int(bits), int(num_iters), int(bool(plus)))
    return out


def sq_error(w, q):
    w, q = _f32(w), _f32(q)
    return lib().po2o_sq_error(_ptr(w), _ptr(q), w.size)


def conv2d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    """Direct NCHW convolution with fp64 accumulation; returns float64."""
    x, w = _f32(x), _f32(w)
    b = _f32(b) if b is not None else None
    N, C, H, W = x.shape
    K, Cg, R, S = w.shape
    assert Cg * groups == C and K % groups == 0
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
    Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
    y = np.empty((N, K, P, Q), dtype=np.float64)
    lib().po2o_conv2d(_ptr(x), _ptr(w), _ptr(b), _ptr(y), N, C, H, W, K, R, S,
                      sh, sw, ph, pw, dh, dw, groups)
    return y


def qconv2d(x, w, b=None, stride=1, padding=1, dilation=1, groups=1, bits=4, mode="po2", fsr=1):
    """QuantizedConv2d.forward restated: returns (y float64, quantized weight)."""
    qw = _f32(w) if mode == "none" else quantize(w, bits, mode, fsr)
    return conv2d(x, qw, b, stride, padding, dilation, groups), qw


def cpu_reference_qconv2d(x_t, w_t, b_t, stride, padding, dilation, groups, bits, mode):
    """The reference's CPU path (quantizer + torch CPU conv) on torch CPU tensors."""
    import torch
    import torch.nn.functional as F

    qw = w_t if mode == "none" else torch.from_numpy(quantize(w_t.numpy(), bits, mode))
    return F.conv2d(x_t, qw, b_t, stride, padding, dilation, groups)
