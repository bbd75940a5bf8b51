"""A/B of conv_rowsk's pipelined split (PO2Q_ROWSK_PIPE=1) against the default kernel, C = K = 64
3x3 s1 p1: every rowsk candidate plan (direct stores / TT output tile, 2 or 3 rows in flight) at the
bench's stage-3 shape (bs 256 @56) plus ragged shapes -- outputs compared bit for bit, then
interleaved timing rounds (median ms).  GPU only."""
import json
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from tools.tile_sweep import timeit  # noqa: E402


def setpipe(on):
    os.environ["PO2Q_ROWSK_PIPE"] = "1" if on else "0"


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(256, 56, 56), (3, 13, 13), (2, 20, 28), (5, 56, 56), (1, 9, 44), (4, 30, 8)]
    for n, h, w_ in shapes:
        x = torch.relu(torch.randn(n, 64, h, w_, device=dev, generator=g))
        w = torch.randn(64, 64, 3, 3, device=dev, generator=g) * 0.05
        plans = _lib.plans(n, 64, h, w_, 64, 3, 3, 1, 1)
        idx = [i for i, d in enumerate(plans) if "bf16x3_rows" in d and re.search(r"\bfp=0\b", d)
               and re.search(r"\bvr=[12]\b", d) and "CC=32" in d]
        for i in idx:
            outs = []
            for on in (False, True):
                setpipe(on)
                outs.append(_lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, "po2", plan=i))
            torch.cuda.synchronize()
            same = torch.equal(outs[0], outs[1])
            rec = {"shape": [n, 64, h, w_], "plan": i, "desc": plans[i][:120], "bitwise_equal": same}
            if n == 256:
                ts = {0: [], 1: []}
                for _ in range(int(os.environ.get("ROUNDS", "5"))):
                    for on in (0, 1):
                        setpipe(on)
                        ts[on].append(timeit(lambda: _lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, "po2", plan=i), 20))
                rec["ms_default"] = round(sorted(ts[0])[len(ts[0]) // 2], 4)
                rec["ms_pipe"] = round(sorted(ts[1])[len(ts[1]) // 2], 4)
            print(json.dumps(rec), flush=True)
            if not same:
                raise SystemExit("PIPE output differs")
    os.environ.pop("PO2Q_ROWSK_PIPE", None)


if __name__ == "__main__":
    main()
