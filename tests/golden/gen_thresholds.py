"""Generate the PO2 / PO2+ per-binade decision thresholds from the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_thresholds.py

For every positive fp32 value a in (0, 1] it runs the reference quantizer
(`PowerOfTwoQuantizer.forward` / `PowerOfTwoPlusQuantizer.forward`,
utils/quantizers.py:19-56) on a chunk that also holds 1.0, so scale == 1 and the
normalised input is a itself.  With bits=9 (clamp window [-255, 0]) nothing is
clamped, so the output 2^e reveals the unclamped exponent decision e(a).

Within each binade k (a in [2^k, 2^(k+1))) the decision must be monotone with
exactly one step k -> k+1; the smallest a of the binade that decides k+1 is the
threshold T_k (fp32 bit pattern).  The script asserts monotonicity for EVERY
value (2^30 of them), so the table is an exact restatement of the reference's
fp32 log2/round arithmetic (torch CPU), not an approximation.

Output: tests/golden/po2_thresholds.json (committed).  The generator is the
only code that touches the reference; the JSON is data.
"""
import json
import os
import sys
import time

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "po2_thresholds.json")


def main():
    sys.path.insert(0, REF)
    from utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer

    quantizers = {"po2": PowerOfTwoQuantizer, "po2+": PowerOfTwoPlusQuantizer}
    one_bits = 0x3F800000
    chunk = 1 << 23  # one normal binade per chunk (chunk 0 = all subnormals)
    result = {
        "source": "reference utils/quantizers.py:19-56 run under torch %s, "
        "ATEN cpu capability %s; bits=9 (no clamp), scale forced to 1.0"
        % (torch.__version__, torch.backends.cpu.get_cpu_capability()),
        "k_min": -149,
        "k_max": -1,
        "modes": {},
    }
    for name, q in quantizers.items():
        t0 = time.time()
        thr = {}
        # walk a = bits 1 .. 0x3F7FFFFF (all positive floats below 1.0)
        start = 1
        while start < one_bits:
            stop = min((start // chunk + 1) * chunk, one_bits)
            ab = torch.arange(start, stop, dtype=torch.int64).to(torch.int32)
            a = ab.view(torch.float32)
            inp = torch.cat([torch.ones(1), a])
            out = q.forward(None, inp, 9)[1:]
            assert torch.all(out > 0), "zero output for positive input"
            m, e = torch.frexp(out)
            assert torch.all(m == 0.5), "output not a power of two"
            e = (e - 1).to(torch.int64)  # out = 2^e
            am, ae = torch.frexp(a)
            k = (ae - 1).to(torch.int64)  # binade of a
            d = e - k
            assert torch.all((d == 0) | (d == 1)), "decision outside {k, k+1}"
            # monotone within each binade: d must be non-decreasing along a
            # while k stays fixed
            same = k[1:] == k[:-1]
            assert torch.all(~same | (d[1:] >= d[:-1])), "non-monotone decision"
            # record first a with d == 1 per binade (chunks are walked in order)
            idx = torch.nonzero(d == 1).flatten()
            if idx.numel():
                kk = k[idx]
                first = torch.ones_like(kk, dtype=torch.bool)
                first[1:] = kk[1:] != kk[:-1]
                for kv, iv in zip(kk[first].tolist(), idx[first].tolist()):
                    if kv not in thr:
                        thr[kv] = int(ab[iv].item()) & 0xFFFFFFFF
            start = stop
        # seam check: re-verify every threshold by evaluating T-1 and T
        table = {}
        for kv in range(-149, 0):
            T = thr.get(kv)
            if T is None:
                T = ((kv + 1 + 127) << 23) if kv + 1 >= -126 else (1 << (kv + 1 + 149))
                table[kv] = {"T": "%08x" % T, "note": "no k+1 decision in binade"}
                continue
            table[kv] = {"T": "%08x" % T}
        # seam verification with the reference itself
        ts = [int(v["T"], 16) for v in table.values()]
        probe = []
        for T in ts:
            probe += [T - 1, T]
        pb = torch.tensor(probe, dtype=torch.int64).to(torch.int32).view(torch.float32)
        out = q.forward(None, torch.cat([torch.ones(1), pb]), 9)[1:]
        _, e = torch.frexp(out)
        _, ae = torch.frexp(pb)
        d = (e - ae).view(-1, 2)
        for (kv, v), (d0, d1) in zip(table.items(), d.tolist()):
            if "note" in v:
                continue
            assert (d0, d1) == (0, 1), (name, kv, v, d0, d1)
        result["modes"][name] = {str(k): v for k, v in table.items()}
        print(name, "done in %.1fs" % (time.time() - t0), flush=True)
    with open(OUT, "w") as f:
        json.dump(result, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
