"""Generate golden input/output vectors by running the REFERENCE on CPU.

Build container only (needs /root/reference, read-only; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Writes (all data, no reference source):
  quant_kat.npz   PO2 / PO2+ quantizer known-answer vectors
                  (utils/quantizers.py:19-56 `forward`), inputs + outputs
  conv_kat.npz    QuantizedConv2d forward vectors (models/quantized_conv.py:32-38)
                  for every distinct conv kind of the reference models
  models.npz      ResNet20 PTQ (config 1: quantize_model, quantizers.py:139-153)
                  and QAT-mode logits for ResNet20 / ResNet56 / MobileNetV2 on
                  seeded synthetic inputs; weights come from fill.seeded_fill_
  lin_kat.npz     LinearPowerOfTwo(Plus)Quantizer vectors (utils/quantizers.py:59-136),
                  inputs + outputs, bits 2/3/4, default and explicit num_iters
  models.json     state_dict key/shape lists of the reference models (checkpoint
                  compatibility of the drop-in modules)
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
from fill import seeded_fill_  # noqa: E402


def f32(bits):
    return np.asarray(bits, dtype=np.uint32).view(np.float32)


def quant_cases(thr):
    """name -> fp32 numpy input tensor."""
    cases = {}
    g = torch.Generator().manual_seed(1234)
    # weight-shaped tensors over six decades of scale
    shapes = {"r16": (16, 16, 3, 3), "r64": (64, 64, 3, 3), "ds1x1": (32, 16, 1, 1),
              "dw960": (960, 1, 3, 3), "pw": (96, 24, 1, 1), "odd": (7, 5, 3, 1)}
    for sname, shp in shapes.items():
        for dec in (-3, 0, 2):
            fan = shp[0] * shp[2] * shp[3]
            w = torch.randn(shp, generator=g) * (2.0 / fan) ** 0.5 * 10.0 ** dec
            cases["%s_e%d" % (sname, dec)] = w.numpy()
    # +/- 6 ulp around every threshold that matters for bits <= 9, both modes,
    # normalised by scale 1 (1.0 present) and by an awkward scale (0.3)
    for mode in ("po2", "po2+"):
        near = []
        for k in range(-20, 0):
            T = int(thr[mode][str(k)]["T"], 16)
            near += list(range(T - 6, T + 7))
        a = f32(near)
        sgn = np.where(np.arange(a.size) % 2 == 0, 1.0, -1.0).astype(np.float32)
        cases["near_%s_s1" % mode] = np.concatenate([[1.0], a * sgn]).astype(np.float32)
        cases["near_%s_s03" % mode] = (np.concatenate([[1.0], a * sgn]) * np.float32(0.3)).astype(np.float32)
    # exact PO2+ ties 1.5*2^k and PO2 exact sqrt-2 neighbourhood
    ties = np.array([1.0] + [1.5 * 2.0 ** k for k in range(-12, 0)] +
                    [-1.5 * 2.0 ** k for k in range(-12, 0)] +
                    [2.0 ** k for k in range(-12, 1)] + [2.0 ** (k + 0.5) for k in range(-12, 0)],
                    dtype=np.float32)
    cases["ties"] = ties
    cases["zeros_signed"] = np.array([0.0, -0.0, 0.5, -0.25, 1.0, -0.0], dtype=np.float32)
    cases["all_zero"] = np.zeros((4, 3), dtype=np.float32)
    cases["with_nan"] = np.array([0.1, np.nan, -0.5, 0.0], dtype=np.float32)
    cases["with_inf"] = np.array([np.inf, 1.0, 0.0, -2.0], dtype=np.float32)
    cases["with_neginf"] = np.array([-np.inf, 1.0, 0.0, -2.0], dtype=np.float32)
    cases["single"] = np.array([-0.7], dtype=np.float32)
    cases["subnormal"] = np.concatenate([f32([1, 2, 3, 0x7FFFF, 0x400000]), f32([0x00800000])]).astype(np.float32)
    cases["tiny_scale"] = (np.array([1.0, 0.3, -0.01, 1e-3, 0.7], dtype=np.float32) * np.float32(1e-36)).astype(np.float32)
    cases["huge_scale"] = (np.array([1.0, 0.3, -0.01, 1e-3, 0.7], dtype=np.float32) * np.float32(3e37)).astype(np.float32)
    return cases


def gen_quant(thr):
    from utils.quantizers import PowerOfTwoPlusQuantizer, PowerOfTwoQuantizer

    qs = {"po2": PowerOfTwoQuantizer, "po2+": PowerOfTwoPlusQuantizer}
    out = {}
    for name, x in quant_cases(thr).items():
        out["x/" + name] = x
        for mode, q in qs.items():
            for bits in (2, 3, 4, 5, 8):
                y = q.forward(None, torch.from_numpy(x.copy()), bits).numpy()
                out["y/%s/%s/%d" % (name, mode, bits)] = y
            # .apply(w, bits) form (fsr default) and explicit fsr=2
            y = q.apply(torch.from_numpy(x.copy()), 4).numpy()
            out["apply/%s/%s/4" % (name, mode)] = y
            y = q.forward(None, torch.from_numpy(x.copy()), 4, 2).numpy()
            out["fsr2/%s/%s/4" % (name, mode)] = y
    np.savez_compressed(os.path.join(HERE, "quant_kat.npz"), **out)
    print("quant_kat.npz:", len(out), "arrays")


CONV_CASES = [
    # name, N, C, H, W, K, R, S, stride, pad, dil, groups, bias, mode, bits
    ("r3x3s1_16", 2, 16, 10, 12, 16, 3, 3, 1, 1, 1, 1, False, "po2", 4),
    ("r3x3s1_32", 2, 32, 8, 8, 32, 3, 3, 1, 1, 1, 1, False, "po2", 4),
    ("r3x3s1_64", 1, 64, 6, 7, 64, 3, 3, 1, 1, 1, 1, False, "po2", 3),
    ("r3x3s2_16_32", 2, 16, 11, 10, 32, 3, 3, 2, 1, 1, 1, False, "po2", 4),
    ("r3x3s2_32_64", 2, 32, 8, 8, 64, 3, 3, 2, 1, 1, 1, False, "po2+", 4),
    ("r1x1s2_16_32", 2, 16, 10, 10, 32, 1, 1, 2, 0, 1, 1, False, "po2", 4),
    ("r1x1s2_32_64", 2, 32, 9, 9, 64, 1, 1, 2, 0, 1, 1, False, "po2+", 2),
    ("pw_96_24", 2, 96, 5, 5, 24, 1, 1, 1, 0, 1, 1, False, "po2+", 4),
    ("pw_24_144", 2, 24, 6, 6, 144, 1, 1, 1, 0, 1, 1, False, "po2+", 4),
    ("dw3x3s1_32", 2, 32, 8, 8, 32, 3, 3, 1, 1, 1, 32, False, "po2+", 4),
    ("dw3x3s2_96", 2, 96, 9, 9, 96, 3, 3, 2, 1, 1, 96, False, "po2+", 3),
    ("stem_3_16", 2, 3, 9, 9, 16, 3, 3, 1, 1, 1, 1, False, "none", 4),
    ("bias_3x3", 2, 8, 7, 7, 12, 3, 3, 1, 1, 1, 1, True, "po2", 4),
    ("grp2_3x3", 2, 8, 7, 7, 12, 3, 3, 1, 1, 1, 2, False, "po2", 4),
    ("dil2_3x3", 1, 8, 9, 9, 8, 3, 3, 1, 2, 2, 1, False, "po2+", 4),
    ("k5_pad2", 1, 6, 9, 9, 10, 5, 5, 1, 2, 1, 1, False, "po2", 4),
    ("nxn_fusion_2c", 2, 48, 6, 6, 24, 3, 3, 1, 1, 1, 1, False, "po2+", 2),
    ("none_3x3_16", 2, 16, 10, 12, 16, 3, 3, 1, 1, 1, 1, False, "none", 4),
]


def gen_conv():
    from models.quantized_conv import QuantizedConv2d
    from utils.quantizers import quantizer_dict

    out = {}
    meta = []
    for i, (name, N, C, H, W, K, R, S, st, pad, dil, grp, bias, mode, bits) in enumerate(CONV_CASES):
        g = torch.Generator().manual_seed(100 + i)
        qfn = None if mode == "none" else quantizer_dict[mode]
        m = QuantizedConv2d(C, K, (R, S), stride=st, padding=pad, dilation=dil, groups=grp,
                            bias=bias, quantize_fn=qfn, bits=bits)
        with torch.no_grad():
            m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / (K * R * S)) ** 0.5)
            if bias:
                m.bias.copy_(0.1 * torch.randn(K, generator=g))
        x = torch.randn(N, C, H, W, generator=g)
        with torch.no_grad():
            y = m(x)
            # reference in fp64 of the same quantized weight (conditioning probe)
            qw = m.weight if qfn is None else qfn.apply(m.weight, bits)
            y64 = torch.nn.functional.conv2d(x.double(), qw.double(), None if not bias else m.bias.double(),
                                             st, pad, dil, grp)
        out["x/" + name] = x.numpy()
        out["w/" + name] = m.weight.detach().numpy()
        if bias:
            out["b/" + name] = m.bias.detach().numpy()
        out["y/" + name] = y.numpy()
        out["y64/" + name] = y64.numpy()
        meta.append(dict(name=name, N=N, C=C, H=H, W=W, K=K, R=R, S=S, stride=st, pad=pad,
                         dil=dil, groups=grp, bias=bias, mode=mode, bits=bits))
    np.savez_compressed(os.path.join(HERE, "conv_kat.npz"), **out)
    with open(os.path.join(HERE, "conv_kat.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("conv_kat.npz:", len(meta), "cases")


LIN_SHAPES = {"r16": (16, 16, 3, 3), "r32_16": (32, 16, 3, 3), "r64": (64, 64, 3, 3), "ds1x1": (64, 32, 1, 1),
              "pw": (144, 24, 1, 1), "dw": (96, 1, 3, 3), "fusion": (24, 48, 3, 3), "odd": (7, 5, 3, 1)}


def gen_lin():
    from utils.quantizers import LinearPowerOfTwoPlusQuantizer, LinearPowerOfTwoQuantizer

    qs = {"lin": LinearPowerOfTwoQuantizer, "lin+": LinearPowerOfTwoPlusQuantizer}
    g = torch.Generator().manual_seed(4321)
    cases = {}
    for sname, shp in LIN_SHAPES.items():
        fan = shp[0] * shp[2] * shp[3]
        for dec in (-2, 0):
            cases["%s_e%d" % (sname, dec)] = (torch.randn(shp, generator=g) * (2.0 / fan) ** 0.5 * 10.0 ** dec).numpy()
    # skewed channels (min and max of different magnitude), a constant channel
    # (delta 0 -> NaN, as in the reference), a channel holding a NaN, an all-zero tensor
    w = torch.randn((8, 6, 3, 3), generator=g) * 0.05
    w[:, 1] = w[:, 1].abs() + 0.02
    w[:, 2] = 0.125
    w[3, 4, 1, 1] = float("nan")
    cases["edge"] = w.numpy()
    cases["zeros"] = np.zeros((4, 3, 3, 3), dtype=np.float32)
    out = {}
    for name, x in cases.items():
        out["x/" + name] = x
        for qn, q in qs.items():
            for bits in (2, 3, 4):
                out["y/%s/%s/%d" % (name, qn, bits)] = q.forward(None, torch.from_numpy(x.copy()), bits).numpy()
            out["apply/%s/%s/4" % (name, qn)] = q.apply(torch.from_numpy(x.copy()), 4).numpy()
            for it in (0, 3):
                out["it%d/%s/%s/4" % (it, name, qn)] = q.forward(None, torch.from_numpy(x.copy()), 4, it).numpy()
    np.savez_compressed(os.path.join(HERE, "lin_kat.npz"), **out)
    print("lin_kat.npz:", len(out), "arrays")


def gen_models():
    from models.model import get_model
    from utils.quantizers import quantize_model, quantizer_dict

    out, keys = {}, {}
    # config 1: ResNet20 PTQ po2 4-bit (test.py:118-121 -> quantizers.py:139)
    torch.manual_seed(0)
    x = torch.randn(8, 3, 32, 32, generator=torch.Generator().manual_seed(1))
    out["x/cifar8"] = x.numpy()
    # MobileViT (config 5: po2+ 2-bit, weights only) at CIFAR size (1x1 patches) and at
    # 64x64 (2x2 patches, the ImageNet-size code path; 224 raises in the reference)
    out["x/img64"] = torch.randn(4, 3, 64, 64, generator=torch.Generator().manual_seed(2)).numpy()
    specs = [("resnet20", None, 4, 10), ("resnet56", "po2", 4, 10), ("mobilenet", "po2+", 4, 10),
             ("resnet20", "po2+", 3, 10), ("mobilenet", "po2", 2, 10), ("mobilevit", "po2+", 2, 10),
             ("mobilevit", "po2", 4, 10), ("mobilevit@64", "po2+", 2, 10)]
    for mt_spec, q, bits, nc in specs:
        mt, _, sz = mt_spec.partition("@")
        sz = int(sz or 32)
        m = get_model(mt, nc, quantizer_dict[q] if q else None, bits, (sz, sz))
        seeded_fill_(m, seed=7)
        m.eval()
        keys[mt] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        xin = x if sz == 32 else torch.from_numpy(out["x/img64"])
        with torch.no_grad():
            logits = m(xin)
        tag = "%s/%s/%d" % (mt_spec, q or "none", bits)
        out["logits/" + tag] = logits.numpy()
        if q is not None:  # model-level get_quantization_error (reference quirks included)
            e, n = m.get_quantization_error()
            out["qerr/" + tag] = np.array([float(torch.as_tensor(e).detach()), float(n)], dtype=np.float64)
        if q is None:
            for qn in ("po2", "po2+", "lin", "lin+"):
                mc = get_model(mt, nc, None, bits, 32)
                mc.load_state_dict(m.state_dict())
                mc.eval()
                err = quantize_model(mc, quantizer_dict[qn], bits)
                with torch.no_grad():
                    out["ptq_logits/%s/%s/%d" % (mt, qn, bits)] = mc(x).numpy()
                out["ptq_err/%s/%s/%d" % (mt, qn, bits)] = np.array(err, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "models.npz"), **out)
    with open(os.path.join(HERE, "models.json"), "w") as f:
        json.dump(keys, f)
    print("models.npz:", sorted(out))


WIDE_SPECS = [
    # (model, image, batch, quantizer, bits, input seed): wide enough that the drop-in's eval
    # forward takes the fused-block kernels -- the stage-1 conv pair (W >= 128) and the
    # stride-2 + shortcut kernel (transition input W >= 96) -- on the reference's logits
    ("resnet56", 128, 2, "po2", 4, 3),
    ("resnet20", 224, 1, "po2+", 4, 4),
]


def gen_models_wide():
    """models_wide.npz: QAT-mode eval logits of ResNet56 @128 and ResNet20 @224 (reference
    models/resnet.py:55-71 BasicBlock, :150-163 projection shortcut, :190-201 forward)."""
    from models.model import get_model
    from utils.quantizers import quantizer_dict

    out = {}
    for mt, sz, bs, q, bits, seed in WIDE_SPECS:
        m = get_model(mt, 10, quantizer_dict[q], bits, (sz, sz))
        seeded_fill_(m, seed=7)
        m.eval()
        x = torch.randn(bs, 3, sz, sz, generator=torch.Generator().manual_seed(seed))
        with torch.no_grad():
            logits = m(x)
        tag = "%s@%d/%s/%d" % (mt, sz, q, bits)
        out["x/" + tag] = x.numpy()
        out["logits/" + tag] = logits.numpy()
    np.savez_compressed(os.path.join(HERE, "models_wide.npz"), **out)
    print("models_wide.npz:", sorted(out))


VIT256 = ("mobilevit", 256, 2, "po2+", 2, 5, 1000)  # config 5: MobileViT-XS @256 (ImageNet head), po2+ 2-bit


def gen_vit256():
    """models_vit256.npz: QAT-mode eval logits of MobileViT-XS @256x256 (BASELINE config 5, weights
    quantized: the reference quantizes no activations) -- reference models/mobile_vit.py:131-311 at
    the size the bench runs.  The input is NOT stored: the test regenerates it from the seed
    (torch CPU generator), so the fixture stays small."""
    from models.model import get_model
    from utils.quantizers import quantizer_dict

    mt, sz, bs, q, bits, seed, nc = VIT256
    m = get_model(mt, nc, quantizer_dict[q], bits, (sz, sz))
    seeded_fill_(m, seed=7)
    m.eval()
    x = torch.randn(bs, 3, sz, sz, generator=torch.Generator().manual_seed(seed))
    with torch.no_grad():
        logits = m(x)
    tag = "%s@%d/%s/%d" % (mt, sz, q, bits)
    out = {"logits/" + tag: logits.numpy(), "x_sum/" + tag: np.array(float(x.double().sum()))}
    np.savez_compressed(os.path.join(HERE, "models_vit256.npz"), **out)
    print("models_vit256.npz:", sorted(out), logits.shape)


def main():
    sys.path.insert(0, REF)
    thr = json.load(open(os.path.join(HERE, "po2_thresholds.json")))["modes"]
    torch.set_num_threads(8)
    parts = sys.argv[1:] or ["quant", "conv", "lin", "models", "wide", "vit256"]  # e.g. `gen_golden.py lin`
    if "wide" in parts:
        gen_models_wide()
    if "vit256" in parts:
        gen_vit256()
    if "quant" in parts:
        gen_quant(thr)
    if "conv" in parts:
        gen_conv()
    if "lin" in parts:
        gen_lin()
    if "models" in parts:
        gen_models()


if __name__ == "__main__":
    main()
