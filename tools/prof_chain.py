"""Driver for PMC passes over the small-image chain kernel (tools/pmc.sh via PMC_DRIVER, or rocprofv3
directly): config 2's stage-1 run (bs 256, 16 x 32 x 32, 17 layers, BasicBlock form) launched a few
times.  GPU only, tuning aid."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from po2_quantization_amd import _lib  # noqa: E402


def main():
    C, H, n = int(os.environ.get("CHAIN_C", 16)), int(os.environ.get("CHAIN_H", 32)), 17
    dev = torch.device("cuda:0")
    x = torch.relu(torch.randn(256, C, H, H, device=dev))
    ws = [torch.randn(C, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5) for _ in range(n)]
    ps = [torch.rand(C, device=dev) + 0.5 for _ in range(n)]
    pb = [torch.randn(C, device=dev) * 0.1 for _ in range(n)]
    res = [-1 if l % 2 == 0 else l - 1 for l in range(n)]
    for _ in range(3):
        _lib.qconv2d_chain(x, ws, 4, "po2", post_scales=ps, post_shifts=pb, acts=["relu"] * n, res_from=res)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
