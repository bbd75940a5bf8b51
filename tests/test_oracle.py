"""CPU: pin the oracle (oracle/) against the golden vectors produced by running
the reference (tests/golden/gen_golden.py).  No GPU."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests._util import CONV_TOL, bits_equal, lin_kat_items, load_json, load_npz, normwise_err, quant_kat_items


def test_quantizer_bit_exact_on_every_golden_vector():
    d, items = quant_kat_items()
    assert len(items) > 400
    for key, name, mode, bits, fsr, _ in items:
        x = d["x/" + name]
        y = O.quantize(x, bits, mode, fsr)
        ok = bits_equal(y, d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_threshold_table_matches_headers(mode):
    """The C headers (product + oracle) are generated from the same reference data."""
    import os
    import re

    from tests._util import GOLDEN

    tab = load_json("po2_thresholds.json")["modes"][mode]
    want = [int(tab[str(k)]["T"], 16) for k in range(-149, 0)]
    root = os.path.dirname(os.path.dirname(GOLDEN))
    for hdr in ("oracle/po2_oracle_thresholds.h", "po2_quantization_amd/csrc/po2q_thresholds.h"):
        text = open(os.path.join(root, hdr)).read()
        blocks = re.findall(r"\{ /\* (po2\+?) \*/\n(.*?) \}", text, re.S)
        got = {m: [int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", body)] for m, body in blocks}
        assert got[mode] == want, hdr


def test_survey_threshold_rows():
    """SURVEY §8a table (k = -9..-1), cross-checked against the generated data."""
    tab = load_json("po2_thresholds.json")["modes"]
    po2 = "3b3504f0 3bb504f6 3c3504f2 3cb504f6 3d3504f2 3db504f5 3e3504f3 3eb504f4 3f3504f3".split()
    po2p = "3b3ffffc 3bc00003 3c3fffff 3cc00003 3d3fffff 3dc00001 3e3fffff 3ec00001 3f400000".split()
    assert [tab["po2"][str(k)]["T"] for k in range(-9, 0)] == po2
    assert [tab["po2+"][str(k)]["T"] for k in range(-9, 0)] == po2p


def test_quantizer_levels_and_edge_cases():
    # levels: bits=2 -> {1/2, 1}; bits=4 -> 2^-7..2^0 (times scale)
    w = np.linspace(-1, 1, 4001).astype(np.float32)
    for bits, lo in ((2, -1), (3, -3), (4, -7)):
        q = O.quantize(w, bits, "po2")
        mags = np.unique(np.abs(q[q != 0]))
        assert set(np.log2(mags).astype(int)) <= set(range(lo, 1))
    assert np.isnan(O.quantize(np.zeros(5, np.float32), 4, "po2")).all()
    y = O.quantize(np.array([0.0, -0.0, 1.0], np.float32), 4, "po2")
    assert (y.view(np.uint32)[:2] == 0).all()  # +0.0 for both signed zeros


def test_conv_oracle_against_reference_vectors():
    d = load_npz("conv_kat.npz")
    for m in load_json("conv_kat.json"):
        n = m["name"]
        b = d["b/" + n] if m["bias"] else None
        y, _ = O.qconv2d(d["x/" + n], d["w/" + n], b, m["stride"], m["pad"], m["dil"], m["groups"],
                         m["bits"], m["mode"])
        # oracle accumulates in fp64: equal to the reference's fp64 conv of its quantized weight
        assert normwise_err(y, d["y64/" + n]) < 1e-12, n
        # and within the fp32 parity contract of the reference's own fp32 output
        assert normwise_err(y, d["y/" + n]) < CONV_TOL, n


def test_sq_error():
    w = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    q = O.quantize(w, 4, "po2+")
    assert abs(O.sq_error(w, q) - float(((q.astype(np.float64) - w) ** 2).sum())) < 1e-9


def test_lin_oracle_bit_exact_on_every_golden_vector():
    """lin / lin+ restatement vs the reference's outputs (utils/quantizers.py:59-136):
    bits 2/3/4, num_iters 0/3/10, constant and NaN channels, all-zero tensor."""
    d, items = lin_kat_items()
    assert len(items) >= 200
    for key, name, qn, bits, iters, _ in items:
        y = O.quantize_lin(d["x/" + name], bits, qn == "lin+", iters)
        ok = bits_equal(y, d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


def test_log2_tables_agree():
    """The product's and the oracle's generated round(log2) tables are the same data
    (tools/gen_log2_table.py) and reproduce the PO2 rows of SURVEY §8a."""
    import re

    def read(path):
        txt = open(path).read()
        return [int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", txt)]

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    a = read(os.path.join(root, "po2_quantization_amd/csrc/po2q_log2_table.h"))
    b = read(os.path.join(root, "oracle/po2_oracle_log2_table.h"))
    assert a == b and len(a) == 254
    assert a[-1 + 126] == 0x3F3504F3 and a[-5 + 126] == 0x3D3504F2  # k = -1, -5 (PO2 T_k)
