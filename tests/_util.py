import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Parity contract for floating-point conv outputs (BASELINE.md "Parity contract"):
# max|y - y_ref| <= CONV_TOL * max|y_ref| per tensor (normwise relative, fp32).
CONV_TOL = 1e-5


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def quant_kat_items():
    """(key, input name, mode, bits, fsr, call form) for every quantizer golden vector."""
    d = load_npz("quant_kat.npz")
    out = []
    for key in d.files:
        kind = key.split("/")[0]
        if kind not in ("y", "apply", "fsr2"):
            continue
        _, name, mode, bits = key.split("/")
        out.append((key, name, mode, int(bits), 2 if kind == "fsr2" else 1, kind))
    return d, out


def bits_equal(a, b):
    """Bitwise equality, treating any NaN as equal to any NaN."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    same = a.view(np.uint32) == b.view(np.uint32)
    return same | (np.isnan(a) & np.isnan(b))


def normwise_err(y, ref):
    y = np.asarray(y, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    den = np.abs(ref).max()
    return float(np.abs(y - ref).max() / (den if den > 0 else 1.0))
