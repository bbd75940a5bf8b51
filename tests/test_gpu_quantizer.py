"""GPU parity: the HIP quantizer (libpo2q via the C ABI) is bit-exact with the
reference golden vectors and with the oracle.  Bar: bit-exact (NaN == NaN)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from po2_quantization_amd import _lib
from po2_quantization_amd.utils.quantizers import (PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer,
                                                   quantizer_dict)
from tests._util import bits_equal, lin_kat_items, quant_kat_items

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


def test_empty_raises():
    with pytest.raises(RuntimeError, match="numel"):
        PowerOfTwoQuantizer.apply(torch.empty(0, device=DEV), 4)
    with pytest.raises(RuntimeError, match="numel"):
        PowerOfTwoQuantizer.apply(torch.empty(0, device=DEV, dtype=torch.float64), 4)


def _bit_equal(y, want, dt):
    """Bitwise equality with any NaN equal to any NaN."""
    iv = torch.int16 if dt == "bf16" else torch.int64
    nan = torch.isnan(y)
    if not torch.equal(nan, torch.isnan(want)):
        return False
    return torch.equal(y.view(iv)[~nan], want.view(iv)[~nan])


def test_fp64_bf16_on_gpu_native_bit_exact():
    """fp64 / bf16 HIP tensors take the native kernels (po2q_quant_dtypes.hip: the reference's
    decision in that dtype, tables measured from the reference): dtype and device preserved and
    every output the reference's CPU output bit for bit (tests/golden/quant_kat_dtypes.npz)."""
    from po2_quantization_amd.utils.quantizers import PowerOfTwoPlusQuantizer
    from tests.test_restated_quantizer import _load, dtype_items

    n = 0
    for d, key, dt, name, mode, bits in dtype_items():
        x = _load(d["x/%s/%s" % (dt, name)], dt).to(DEV)
        want = _load(d[key], dt)
        Q = PowerOfTwoQuantizer if mode == "po2" else PowerOfTwoPlusQuantizer
        y = Q.apply(x, bits)
        assert y.dtype == x.dtype and y.device == x.device
        assert _bit_equal(y.cpu(), want, dt), key
        n += 1
    assert n == 48


def test_fp64_bf16_native_kernels_loaded_not_restated(monkeypatch):
    """The GPU path for fp64 / bf16 is the native op, not the torch restatement."""
    monkeypatch.setattr(_lib, "restated_quantize", lambda *a, **k: (_ for _ in ()).throw(AssertionError("restated")))
    for dt in (torch.float64, torch.bfloat16):
        y = _lib.quantize(torch.randn(64, 32, 3, 3, device=DEV).to(dt), 4, "po2")
        assert y.dtype == dt


def test_fp64_bf16_on_gpu_extended_vectors():
    """tests/golden/quant_kat_dtypes2.npz (gen_golden_dtypes2.py): +-64 patterns around every fp64
    threshold of binades -12..-1, every bf16 magnitude below 1, subnormal binades and underflowing
    products, random weights over many decades, +-0 / inf / NaN / all-zero, bits 2..16, fsr 1 and 2."""
    from tests._util import load_npz
    from tests.test_restated_quantizer import _load

    d = load_npz("quant_kat_dtypes2.npz")
    n = 0
    for key in d.files:
        if not key.startswith("y/"):
            continue
        _, dt, name, mode, bits, fsr = key.split("/")
        x = _load(d["x/%s/%s" % (dt, name)], dt).to(DEV)
        y = _lib.quantize(x, int(bits), mode, int(fsr))
        assert _bit_equal(y.cpu(), _load(d[key], dt), dt), key
        n += 1
    assert n == 192


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


# ---- lin / lin+ (utils/quantizers.py:59-136) ----

def test_lin_every_golden_vector_bit_exact():
    d, items = lin_kat_items()
    for key, name, qn, bits, iters, kind in items:
        x = torch.from_numpy(d["x/" + name].copy()).to(DEV)
        q = quantizer_dict[qn]
        if kind == "apply":
            y = q.apply(x, bits)
        elif kind.startswith("it"):
            y = q.forward(None, x, bits, iters)
        else:
            y = q.forward(None, x, bits=bits)
        ok = bits_equal(y.cpu().numpy(), d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


@pytest.mark.parametrize("shape", [(16, 16, 3, 3), (64, 64, 3, 3), (960, 160, 1, 1), (96, 1, 3, 3),
                                   (5000, 2, 1, 1), (17000, 1, 1, 1), (3, 7, 5, 2), (1, 1, 1, 1)])
@pytest.mark.parametrize("qn", ["lin", "lin+"])
def test_lin_random_weights_match_oracle(shape, qn):
    """Random weights over three decades, every kernel path (channels of <= 4096, <= 16384
    and more elements): bit-exact with the oracle."""
    g = torch.Generator().manual_seed(sum(shape))
    for dec in (-3, -1, 1):
        w = torch.randn(shape, generator=g) * 10.0 ** dec
        for bits in (2, 3, 4, 8):
            y = _lib.quantize_lin(w.to(DEV), bits, qn == "lin+").cpu().numpy()
            ref = O.quantize_lin(w.numpy(), bits, qn == "lin+")
            ok = bits_equal(y, ref)
            assert ok.all(), (shape, dec, bits, np.nonzero(~ok.ravel())[0][:8])


def test_lin_errors_and_autograd():
    w = torch.randn(8, 4, 3, 3, device=DEV, requires_grad=True)
    y = quantizer_dict["lin"].apply(w, 4)
    y.sum().backward()  # straight-through (quantizers.py:93-96)
    assert torch.equal(w.grad, torch.ones_like(w))
    with pytest.raises(_lib.Po2qError, match="4-D"):
        _lib.quantize_lin(torch.randn(8, 4, device=DEV), 4, False)
    with pytest.raises(_lib.Po2qError, match="non-zero size"):
        _lib.quantize_lin(torch.randn(0, 4, 3, 3, device=DEV), 4, False)
    with pytest.raises(_lib.Po2qError, match="bits"):
        _lib.quantize_lin(torch.randn(2, 4, 3, 3, device=DEV), 0, False)
    # a CPU tensor takes the product's torch restatement of the reference ops (the CPU drop-in path):
    # the same values as the HIP kernel
    wc = torch.randn(2, 4, 3, 3)
    for plus in (False, True):
        assert torch.equal(_lib.quantize_lin(wc, 4, plus), _lib.quantize_lin(wc.to(DEV), 4, plus).cpu())
