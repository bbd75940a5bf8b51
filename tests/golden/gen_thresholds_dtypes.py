"""Generate the PO2 / PO2+ per-binade decision thresholds for fp64 and bf16 inputs from the
REFERENCE itself (utils/quantizers.py:19-56, run by torch on CPU in the input's dtype).

Build container only (needs /root/reference, read-only; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_thresholds_dtypes.py

The reference keeps the input's dtype, so its exponent decision is torch's
log2 / round in that dtype: for bf16 each step (w / scale, log2, a / 1.5, + 0.5) is computed in
fp32 and rounded to bf16; for fp64 it is torch's double log2.  As for fp32 (gen_thresholds.py),
within each binade k (a in [2^k, 2^(k+1))) the decision is k or k + 1 and monotone, so one
threshold T_k per binade restates it: e = k + (bits(a) >= T_k).

  bf16: EVERY positive bf16 below 1.0 is run (16,255 values) and its decision stored as a table
        (subnormal binades are not single-threshold there).
  fp64: per binade the first pattern deciding >= k (D_k) and >= k + 1 (U_k) by bisection on the
        reference's own decision (all binades at once), then checked against the reference on
        +-2^12 bit patterns around every D_k / U_k, +-2^20 around those of the binades bits <= 4
        reach (k >= -8), and 4096 random patterns in every binade.  (2^52 patterns per binade
        cannot all be run.)

Scale is forced to 1 by a leading 1.0 in each tensor; bits = 12 (clamp window [-2047, 0]) so no
decision is clamped.  Output: tests/golden/po2_thresholds_dtypes.json (data only).
"""
import json
import os
import sys
import time

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "po2_thresholds_dtypes.json")


def decisions(Q, a, dtype):
    """Unclamped exponent decision of the reference for each a (0 < a < 1) with scale 1."""
    inp = torch.cat([torch.ones(1, dtype=dtype), a])
    out = Q.forward(None, inp, 12)[1:]
    o = out.double()
    assert torch.all(o > 0), "zero output for a positive input"
    m, e = torch.frexp(o)
    assert torch.all(m == 0.5), "output not a power of two"
    return (e - 1).to(torch.int64)


def binade_bf16(bits):
    """binade k of positive bf16 bit patterns (subnormals: leading-one position)."""
    b = bits.to(torch.int64)
    ex = b >> 7
    k_norm = ex - 127
    lead = torch.floor(torch.log2(b.clamp(min=1).double())).to(torch.int64)  # subnormal leading one
    return torch.where(ex > 0, k_norm, lead - 133)


def gen_bf16(Q):
    """The reference's decision for EVERY positive bf16 below 1.0, as d = e - k + 1 (k the binade):
    bf16 subnormal binades are not single-threshold (po2+: a / 1.5 rounds to a subnormal, e.g. two
    values of binade -129 decide k - 1), so the kernel reads this table instead of a threshold."""
    bits = torch.arange(0, 0x3F80, dtype=torch.int32)
    a = bits[1:].to(torch.int16).view(torch.bfloat16)
    e = decisions(Q, a, torch.bfloat16)
    k = binade_bf16(bits[1:])
    d = e - k
    assert torch.all((d >= -1) & (d <= 1)), "bf16: decision outside {k-1, k, k+1}"
    normal = k >= -126
    same = (k[1:] == k[:-1]) & normal[1:]
    assert torch.all(~same | (d[1:] >= d[:-1])), "bf16: non-monotone decision in a normal binade"
    return [0] + (d + 1).tolist()  # entry 0 (a == 0) unused


def f64_bits(a):
    return torch.from_numpy(np.asarray(a, dtype=np.float64).view(np.int64).copy())


def f64_from_bits(b):
    return torch.from_numpy(b.numpy().astype(np.int64).view(np.float64).copy())


def binade_lo_hi_f64(k):
    """first and one-past-last bit pattern of binade k (subnormals for k < -1022)."""
    if k >= -1022:
        lo = (k + 1023) << 52
        return lo, lo + (1 << 52)
    lo = 1 << (k + 1074)
    return lo, lo << 1


def bisect_f64(Q, ks, lo, hi, level):
    """Per binade, the smallest bit pattern in [lo, hi) whose decision is >= k + level (hi: none)."""
    kk = torch.tensor(ks, dtype=torch.int64)
    L, H = lo.clone(), hi.clone()
    while bool((L < H).any()):
        mid = L + (H - L) // 2
        midc = torch.minimum(mid, hi - 1)
        d = decisions(Q, f64_from_bits(midc), torch.float64) - kk
        assert torch.all((d >= -1) & (d <= 1)), "f64: decision outside {k-1, k, k+1}"
        up = (d >= level) & (mid < hi)
        act = L < H
        H = torch.where(act & up, mid, H)
        L = torch.where(act & ~up, mid + 1, L)
    return L


def gen_f64(Q, rng):
    """Two thresholds per binade: D_k = first pattern deciding >= k (a normal binade: its first
    pattern; po2+ subnormal binades decide k - 1 below it, a / 1.5 rounding to a subnormal), U_k =
    first pattern deciding k + 1.  e = k - 1 + (bits >= D_k) + (bits >= U_k)."""
    ks = list(range(-1074, 0))
    lo = torch.tensor([binade_lo_hi_f64(k)[0] for k in ks], dtype=torch.int64)
    hi = torch.tensor([binade_lo_hi_f64(k)[1] for k in ks], dtype=torch.int64)  # exclusive
    D = bisect_f64(Q, ks, lo, hi, 0)
    U = bisect_f64(Q, ks, lo, hi, 1)
    # checks around every threshold and at random points of every binade
    for i, k in enumerate(ks):
        span = (1 << 20) if k >= -8 else (1 << 12)
        parts = [torch.from_numpy(rng.integers(int(lo[i]), int(hi[i]), size=4096, dtype=np.int64))]
        for t in (int(D[i]), int(U[i])):
            parts.append(torch.arange(max(int(lo[i]), t - span), min(int(hi[i]), t + span), dtype=torch.int64))
        b = torch.cat(parts)
        d = decisions(Q, f64_from_bits(b), torch.float64) - k
        want = (b >= int(D[i])).to(torch.int64) + (b >= int(U[i])).to(torch.int64) - 1
        assert torch.equal(d, want), "f64: binade %d is not two thresholds" % k
    return {k: (int(dv), int(uv)) for k, dv, uv in zip(ks, D.tolist(), U.tolist())}


def main():
    sys.path.insert(0, REF)
    from utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer

    rng = np.random.default_rng(2024)
    res = {"source": "reference utils/quantizers.py:19-56 run under torch %s, ATEN cpu capability %s; "
                     "scale forced to 1.0, bits=12 (no clamp)" % (torch.__version__,
                                                                  torch.backends.cpu.get_cpu_capability()),
           "bf16": {"layout": "d + 1 per bf16 bit pattern 0..0x3f7f (d = e - binade)", "modes": {}}, "f64": {"k_min": -1074, "k_max": -1, "modes": {}}}
    for name, Q in (("po2", PowerOfTwoQuantizer), ("po2+", PowerOfTwoPlusQuantizer)):
        t0 = time.time()
        tb = gen_bf16(Q)
        res["bf16"]["modes"][name] = "".join(str(v) for v in tb)
        tf = gen_f64(Q, rng)
        res["f64"]["modes"][name] = {"down": ["%016x" % tf[k][0] for k in range(-1074, 0)],
                                     "up": ["%016x" % tf[k][1] for k in range(-1074, 0)]}
        print("%s: bf16 + f64 tables in %.1f s" % (name, time.time() - t0), flush=True)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=0)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
