"""A/B of the stage-2 conv pair (32 -> 32 -> 32 @112, bs 256, po2 4-bit) across environment knobs:
each arm is a set of env settings applied around its calls (the C ABI reads them per call), the arms are
timed in interleaved rounds (HIP events, 11 launches each), medians printed as JSON lines.
  PAIR_AB_ARMS="PO2Q_PAIR_W32=0;PO2Q_PAIR_W32=2;PO2Q_PAIR_W32=3"  (';' between arms, ',' between vars)
  PAIR_AB_FORM=plain|block|general   (general: BN affine + activations, no residual; block: BN affine + ReLU, the identity residual -- BasicBlock.forward)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402


def main():
    C = int(os.environ.get("PAIR_C", "32"))
    N, H = int(os.environ.get("PAIR_N", "256")), int(os.environ.get("PAIR_H", "224" if C == 16 else "112"))
    dev = torch.device("cuda:0")
    arms = [a for a in os.environ.get("PAIR_AB_ARMS", "PO2Q_PAIR_W32=0;PO2Q_PAIR_W32=2").split(";") if a]
    form = os.environ.get("PAIR_AB_FORM", "plain")
    x = torch.relu(torch.randn(N, C, H, H, device=dev))
    w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    kw = {}
    if form == "block":
        kw = dict(post_scale1=torch.rand(C, device=dev) + 0.5, post_shift1=torch.randn(C, device=dev) * 0.1,
                  post_scale2=torch.rand(C, device=dev) + 0.5, post_shift2=torch.randn(C, device=dev) * 0.1,
                  act1="relu", act2="relu", residual=x)
    elif form == "general":  # BN affine + activations, no residual
        kw = dict(post_scale1=torch.rand(C, device=dev) + 0.5, post_shift1=torch.randn(C, device=dev) * 0.1,
                  post_scale2=torch.rand(C, device=dev) + 0.5, post_shift2=torch.randn(C, device=dev) * 0.1,
                  act1="relu", act2="relu6")
    nbytes = 4.0 * (2 * N * C * H * H + 4 * C * C * 9)
    flops = 2 * 2.0 * N * C * H * H * C * 9
    res = {}
    outs = {}
    for _ in range(int(os.environ.get("PAIR_AB_ROUNDS", "5"))):
        for arm in arms:
            env = dict(kv.split("=", 1) for kv in arm.split(",") if kv)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                res.setdefault(arm, []).append(timeit(lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2", **kw), 11))
                outs.setdefault(arm, _lib.qconv2d_pair(x, w1, w2, 4, "po2", **kw))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    base = outs[arms[0]]
    for arm in arms:
        ts = sorted(res[arm])
        ms = ts[len(ts) // 2]
        print(json.dumps({"arm": arm, "form": form, "C": C, "H": H, "batch": N, "ms": round(ms, 4),
                          "all_ms": [round(t, 4) for t in res[arm]], "hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 3),
                          "eff_mfma_frac": round(flops / (ms * 1e-3) / (2516.6e12 / 3), 3),
                          "bitwise_equal_first_arm": bool(torch.equal(outs[arm], base))}), flush=True)


if __name__ == "__main__":
    main()
