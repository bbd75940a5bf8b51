"""GPU parity: the HIP quantizer (libpo2q via the C ABI) is bit-exact with the
reference golden vectors and with the oracle.  Bar: bit-exact (NaN == NaN)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from po2_quantization_amd import _lib
from po2_quantization_amd.utils.quantizers import (PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer,
                                                   quantizer_dict)
from tests._util import bits_equal, quant_kat_items

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_every_golden_vector_bit_exact():
    d, items = quant_kat_items()
    for key, name, mode, bits, fsr, kind in items:
        x = torch.from_numpy(d["x/" + name].copy()).to(DEV)
        q = quantizer_dict[mode]
        if kind == "apply":
            y = q.apply(x, bits)
        elif kind == "fsr2":
            y = q.forward(None, x, bits, fsr)
        else:
            y = q.forward(None, x, bits=bits)
        ok = bits_equal(y.cpu().numpy(), d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


@pytest.mark.parametrize("n", [1, 7, 4096, 36864, 153600, 1 << 20, 3_000_001])
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_random_tensors_match_oracle(n, mode):
    g = torch.Generator().manual_seed(n)
    for dec in (-6, 0, 5):
        w = torch.randn(n, generator=g) * (10.0 ** dec)
        if n > 10:
            w[::97] = 0.0
        for bits in (2, 3, 4, 8):
            y = _lib.quantize(w.to(DEV), bits, mode).cpu().numpy()
            ref = O.quantize(w.numpy(), bits, mode)
            ok = bits_equal(y, ref)
            assert ok.all(), (n, dec, bits, np.nonzero(~ok)[0][:8])


@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_every_binade_threshold_neighbourhood(mode):
    """+-64 ulp around every per-binade threshold k in [-149, -1] (scale 1 and 0.7)."""
    import json

    from tests._util import GOLDEN

    tab = json.load(open(GOLDEN + "/po2_thresholds.json"))["modes"][mode]
    near = []
    for k in range(-149, 0):
        T = int(tab[str(k)]["T"], 16)
        near += [v for v in range(T - 64, T + 65) if 0 < v < 0x3F800000]
    a = np.array(near, dtype=np.uint32).view(np.float32)
    for scale in (1.0, 0.7):
        w = np.concatenate([[1.0], a]).astype(np.float32) * np.float32(scale)
        for bits in (4, 9, 16):
            y = _lib.quantize(torch.from_numpy(w).to(DEV), bits, mode).cpu().numpy()
            assert bits_equal(y, O.quantize(w, bits, mode)).all(), (scale, bits)


def test_noncontiguous_and_shapes():
    w = torch.randn(64, 64, 3, 3, device=DEV)
    wt = w.transpose(0, 1)
    y = PowerOfTwoQuantizer.apply(wt, 4)
    assert y.shape == wt.shape
    ref = O.quantize(wt.contiguous().cpu().numpy(), 4, "po2")
    assert bits_equal(y.contiguous().cpu().numpy(), ref).all()


def test_straight_through_backward():
    w = torch.randn(16, 16, 3, 3, device=DEV, requires_grad=True)
    y = PowerOfTwoPlusQuantizer.apply(w, 3)
    g = torch.randn_like(y)
    y.backward(g)
    assert torch.equal(w.grad, g)


def test_empty_and_wrong_dtype_raise():
    with pytest.raises(RuntimeError, match="numel"):
        PowerOfTwoQuantizer.apply(torch.empty(0, device=DEV), 4)
    with pytest.raises(RuntimeError, match="float32"):
        PowerOfTwoQuantizer.apply(torch.randn(8, device=DEV, dtype=torch.float64), 4)


def test_stream_semantics_no_host_sync():
    """Launches go on torch's current stream and are capturable in a HIP graph."""
    w = torch.randn(64, 32, 3, 3, device=DEV)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        y = PowerOfTwoQuantizer.apply(w, 4)
    s.synchronize()
    ref = O.quantize(w.cpu().numpy(), 4, "po2")
    assert bits_equal(y.cpu().numpy(), ref).all()
    g = torch.cuda.CUDAGraph()
    static_w = w.clone()
    s2 = torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        PowerOfTwoQuantizer.apply(static_w, 4)  # warm-up allocations
    torch.cuda.current_stream().wait_stream(s2)
    with torch.cuda.graph(g):
        out = PowerOfTwoQuantizer.apply(static_w, 4)
    static_w.copy_(w * 3.0)
    g.replay()
    torch.cuda.synchronize()
    ref = O.quantize((w * 3.0).cpu().numpy(), 4, "po2")
    assert bits_equal(out.cpu().numpy(), ref).all()
