"""Golden PO2 / PO2+ vectors for non-fp32 inputs, made by running the REFERENCE's
quantizers (utils/quantizers.py:19-56 `forward`) on CPU in fp64 and bf16.

Build container only (needs /root/reference, read-only; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_dtypes.py

Writes quant_kat_dtypes.npz (data only): x/<dtype>/<name> inputs and
y/<dtype>/<name>/<mode>/<bits> outputs; bf16 tensors are stored as their uint16 bit
patterns, fp64 as float64.  They pin restated_quantize (po2_quantization_amd/_lib.py),
the product path for inputs the native fp32 kernel does not take.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    sys.path.insert(0, REF)
    from utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer  # noqa: E402

    g = torch.Generator().manual_seed(77)
    base = {
        "r16": torch.randn(16, 16, 3, 3, generator=g) * 0.1,
        "wide": torch.randn(4097, generator=g) * 3.0,
        "ties": torch.tensor([1.0, 0.75, 0.375, 0.1875, 0.09375, -0.75, 0.5, 0.0, -0.0, 1.5e-3]),
        "tiny": torch.randn(300, generator=g) * 1e-30,
    }
    out = {}
    for dt_name, dt in (("f64", torch.float64), ("bf16", torch.bfloat16)):
        for name, x0 in base.items():
            x = x0.to(dt)
            out["x/%s/%s" % (dt_name, name)] = store(x)
            for mode, Q in (("po2", PowerOfTwoQuantizer), ("po2+", PowerOfTwoPlusQuantizer)):
                for bits in (2, 3, 4):
                    y = Q.forward(None, x, bits=bits)
                    assert y.dtype == dt
                    out["y/%s/%s/%s/%d" % (dt_name, name, mode, bits)] = store(y)
    np.savez_compressed(os.path.join(HERE, "quant_kat_dtypes.npz"), **out)
    print("quant_kat_dtypes.npz: %d arrays" % len(out))


def store(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


if __name__ == "__main__":
    main()
