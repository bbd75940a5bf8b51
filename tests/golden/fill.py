"""Deterministic parameter/buffer fill shared by the golden generator and the tests.

Golden model fixtures do not ship weights: both the generator (which runs the
reference models) and the parity tests (which run ours) fill every floating
state_dict entry with the same seeded values, keyed by entry name, so the two
models hold bit-identical parameters without a checkpoint in the repo.
"""
import math
import zlib

import torch


def seeded_fill_(module: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    with torch.no_grad():
        for name, t in sorted(module.state_dict().items()):
            if not t.is_floating_point():
                continue
            g = torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ seed) & 0x7FFFFFFF)
            shape = tuple(t.shape)
            if name.endswith("running_var"):
                v = torch.rand(shape, generator=g) + 0.5
            elif name.endswith("running_mean") or name.endswith("bias"):
                v = 0.1 * torch.randn(shape, generator=g)
            elif t.dim() == 4:  # conv weight [K, C/g, R, S]: kaiming fan_out scale
                fan_out = shape[0] * shape[2] * shape[3]
                v = math.sqrt(2.0 / fan_out) * torch.randn(shape, generator=g)
            elif t.dim() == 1:  # BN / LayerNorm weight
                v = 1.0 + 0.1 * torch.randn(shape, generator=g)
            else:  # Linear weights and anything else
                v = 0.05 * torch.randn(shape, generator=g)
            t.copy_(v.to(t.dtype))
    return module
