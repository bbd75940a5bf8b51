"""Run the small-image chain kernel (po2q_qconv2d_chain_f32) a few times for rocprofv3 kernel
traces / PMC counters: config 2's stage runs (ResNet56 @32, bs = 256).

    python tools/prof_chain.py --stage 1 --iters 5
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=1, help="1: 18 x 16->16 @32, 2: 17 x 32->32 @16, 3: 17 x 64->64 @8")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from po2_quantization_amd import _lib

    C, H, n = {1: (16, 32, 18), 2: (32, 16, 17), 3: (64, 8, 17)}[args.stage]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.relu(torch.randn(args.batch, C, H, H, device=dev))
    ws = [torch.randn(C, C, 3, 3, device=dev) * 0.1 for _ in range(n)]
    print("PLAN chain stage %d: %d x %d->%d @%dx%d bs=%d" % (args.stage, n, C, C, H, H, args.batch), flush=True)
    for _ in range(args.iters):
        _lib.qconv2d_chain(x, ws, 4, "po2")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
