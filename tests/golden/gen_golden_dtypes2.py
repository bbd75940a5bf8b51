"""More fp64 / bf16 PO2 / PO2+ golden vectors from the REFERENCE (utils/quantizers.py:19-56 run on CPU
in the input's dtype), for the native fp64 / bf16 kernels (po2q_quant_dtypes.hip):

  f64/thr     +-64 bit patterns around every decision threshold of binades -12..-1 (scale forced
              to 1 by a leading 1.0; both signs)
  f64/sub     subnormal and near-subnormal weights (scale ~1e-300): decisions in the subnormal
              binades, products that underflow
  f64/rnd     random weights over 12 decades of scale
  bf16/all    EVERY bf16 bit pattern of magnitude below 1.0, both signs, scale forced to 1
  bf16/sub    bf16 subnormals with a subnormal scale
  */special   +-0, inf, NaN, all-zero tensors
for bits in {2, 3, 4, 8, 12, 16} and fsr in {1, 2}.

Build container only (needs /root/reference, read-only; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_dtypes2.py

Writes quant_kat_dtypes2.npz (data only): x/<dtype>/<name>, y/<dtype>/<name>/<mode>/<bits>/<fsr>; bf16 as
uint16 bit patterns.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def store(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def main():
    sys.path.insert(0, REF)
    from utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer  # noqa: E402

    thr = json.load(open(os.path.join(HERE, "po2_thresholds_dtypes.json")))
    g = torch.Generator().manual_seed(4242)
    xs = {}
    # f64 thresholds
    pats = []
    for mode in ("po2", "po2+"):
        for which in ("down", "up"):
            for k in range(-12, 0):
                t = int(thr["f64"]["modes"][mode][which][k + 1074], 16)
                pats += list(range(t - 64, t + 64))
    b = np.array(sorted(set(pats)), dtype=np.int64)
    a = b.view(np.float64)
    a = a[(a > 0) & (a < 1)]
    xs["f64/thr"] = torch.from_numpy(np.concatenate([[1.0], a, -a]))
    xs["f64/sub"] = torch.cat([torch.tensor([1e-300]), torch.rand(3000, generator=g, dtype=torch.float64) * 1e-300,
                               torch.randn(1000, generator=g, dtype=torch.float64) * 1e-310,
                               torch.tensor([5e-324, -5e-324, 1e-320])])
    xs["f64/rnd"] = (torch.randn(5000, generator=g, dtype=torch.float64)
                     * torch.pow(10.0, torch.randint(-6, 6, (5000,), generator=g).double()))
    xs["f64/special"] = torch.tensor([0.0, -0.0, 0.5, -0.25, float("inf"), 1e-3], dtype=torch.float64)
    xs["f64/nan"] = torch.tensor([0.3, float("nan"), -0.1], dtype=torch.float64)
    xs["f64/zero"] = torch.zeros(7, dtype=torch.float64)
    allb = torch.arange(1, 0x3F80, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    xs["bf16/all"] = torch.cat([torch.ones(1, dtype=torch.bfloat16), allb, -allb])
    subb = torch.arange(1, 0x0100, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    xs["bf16/sub"] = torch.cat([subb, -subb[::3]])
    xs["bf16/rnd"] = (torch.randn(3000, generator=g) * torch.pow(10.0, torch.randint(-30, 30, (3000,), generator=g).float())
                      ).to(torch.bfloat16)
    xs["bf16/special"] = torch.tensor([0.0, -0.0, 0.5, -0.25, float("inf"), 1e-3]).to(torch.bfloat16)
    xs["bf16/nan"] = torch.tensor([0.3, float("nan"), -0.1]).to(torch.bfloat16)
    xs["bf16/zero"] = torch.zeros(7, dtype=torch.bfloat16)
    out = {}
    for name, x in xs.items():
        out["x/" + name] = store(x)
        for mode, Q in (("po2", PowerOfTwoQuantizer), ("po2+", PowerOfTwoPlusQuantizer)):
            for bits in (2, 3, 4, 8, 12, 16):
                for fsr in (1, 2):
                    if fsr == 2 and bits not in (3, 8):
                        continue
                    y = Q.forward(None, x, bits=bits, fsr=fsr)
                    assert y.dtype == x.dtype
                    out["y/%s/%s/%d/%d" % (name, mode, bits, fsr)] = store(y)
    np.savez_compressed(os.path.join(HERE, "quant_kat_dtypes2.npz"), **out)
    print("quant_kat_dtypes2.npz: %d arrays" % len(out))


if __name__ == "__main__":
    main()
