"""CPU: the product-side torch restatement of PO2 / PO2+ (_lib.restated_quantize, the path
for CPU / fp64 / bf16 inputs) against the reference's own outputs:
quant_kat.npz (fp32, tests/golden/gen_golden.py) and quant_kat_dtypes.npz (fp64 and bf16,
tests/golden/gen_golden_dtypes.py).  Bit-exact."""
import numpy as np
import torch

from po2_quantization_amd import _lib
from po2_quantization_amd.utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer
from tests._util import bits_equal, load_npz, quant_kat_items

QUANT = {"po2": PowerOfTwoQuantizer, "po2+": PowerOfTwoPlusQuantizer}


def test_restatement_bit_exact_on_fp32_golden_vectors():
    d, items = quant_kat_items()
    for key, name, mode, bits, fsr, _ in items:
        x = torch.from_numpy(d["x/" + name])
        y = _lib.restated_quantize(x, bits, mode, fsr).numpy()
        ok = bits_equal(y, d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


def _load(arr, dt):
    if dt == "bf16":
        return torch.from_numpy(arr.view(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(arr)


def dtype_items():
    d = load_npz("quant_kat_dtypes.npz")
    for key in d.files:
        if key.startswith("y/"):
            _, dt, name, mode, bits = key.split("/")
            yield d, key, dt, name, mode, int(bits)


def test_restatement_bit_exact_on_fp64_bf16_golden_vectors():
    n = 0
    for d, key, dt, name, mode, bits in dtype_items():
        x = _load(d["x/%s/%s" % (dt, name)], dt)
        want = _load(d[key], dt)
        y = QUANT[mode].forward(None, x, bits=bits)  # routes to the restatement (not fp32 HIP)
        assert y.dtype == x.dtype
        assert torch.equal(y.view(torch.int16) if dt == "bf16" else y.view(torch.int64),
                           want.view(torch.int16) if dt == "bf16" else want.view(torch.int64)) or \
            torch.equal(torch.isnan(y), torch.isnan(want)) and torch.equal(y[~torch.isnan(y)], want[~torch.isnan(want)]), key
        n += 1
    assert n == 48


def test_restatement_bit_exact_on_extended_dtype_vectors():
    """The extended fp64 / bf16 vectors (quant_kat_dtypes2.npz, the GPU kernels' pins) through the
    CPU restatement: checks the fixture against an independent route to the reference's numbers."""
    d = load_npz("quant_kat_dtypes2.npz")
    n = 0
    for key in d.files:
        if not key.startswith("y/"):
            continue
        _, dt, name, mode, bits, fsr = key.split("/")
        x = _load(d["x/%s/%s" % (dt, name)], dt)
        y = _lib.restated_quantize(x, int(bits), mode, int(fsr))
        want = _load(d[key], dt)
        iv = torch.int16 if dt == "bf16" else torch.int64
        nan = torch.isnan(y)
        assert torch.equal(nan, torch.isnan(want)), key
        assert torch.equal(y.view(iv)[~nan], want.view(iv)[~nan]), key
        n += 1
    assert n == 192
