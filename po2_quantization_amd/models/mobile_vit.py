"""MobileViT-XS built on the drop-in QuantizedConv2d -- config 5's graph.

Caller of the hot path (reference models/mobile_vit.py:15-522).
The module tree reproduces the reference's nesting, so state_dict keys match:

  conv1                 Sequential(Conv2d 3->16 3x3 s2, BN, SiLU)       not quantized (:315)
  stem[0..3]            MV2Block (inverted residual, SiLU)              (:131-233, :317-360)
  trunk[i] = [MV2Block s2, MobileViTBlock]  i = 0..2                    (:362-441)
      MobileViTBlock:   conv1 = qconv nxn+BN+SiLU, conv2 = qconv 1x1+BN+SiLU (local)
                        transformer over (patch pixel, patch) tokens     (global, :101-128)
                        conv3 = qconv 1x1+BN+SiLU, cat with the block input,
                        conv4 = qconv nxn 2C->C +BN+SiLU                 (fusion, :236-311)
  to_logits             Sequential(Sequential(Conv2d 1x1, BN, SiLU), spatial mean, Linear)

Only the QuantizedConv2d layers are quantized (the reference quantizes no
Linear / attention weight, :56-128); attention, LayerNorm and the MLP stay
plain torch ops -- they are off the graded path.  nxn convs use padding 1 as
in the reference (:32), whatever kernel_size is.  einops' rearranges are
spelled as view/permute (same element order).

Note: at 224x224 the reference raises (7x7 map, 2x2 patches, :282 -- SURVEY
§7); this mirror raises the same way (a RuntimeError from the reshape).
"""
from typing import Any, Callable, Optional, Tuple

import torch
import torch.nn as nn

from .quantized_conv import (QuantizedConv2d, batched_packs, can_fuse, fusable_sequence, run_fused_sequence,
                             run_inverted_residual, run_sequence)


def quantized_conv_1x1_bn(inp, oup, quantize_fn=None, bits=4):
    return nn.Sequential(QuantizedConv2d(inp, oup, 1, 1, 0, bias=False, quantize_fn=quantize_fn, bits=bits),
                         nn.BatchNorm2d(oup), nn.SiLU())


def quantized_conv_nxn_bn(inp, oup, kernel_size=3, stride=1, quantize_fn=None, bits=4):
    return nn.Sequential(QuantizedConv2d(inp, oup, kernel_size, stride, 1, bias=False, quantize_fn=quantize_fn,
                                         bits=bits),
                         nn.BatchNorm2d(oup), nn.SiLU())


def conv_1x1_bn(inp, oup):
    return nn.Sequential(nn.Conv2d(inp, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup), nn.SiLU())


def conv_nxn_bn(inp, oup, kernel_size=3, stride=1):
    return nn.Sequential(nn.Conv2d(inp, oup, kernel_size, stride, 1, bias=False), nn.BatchNorm2d(oup), nn.SiLU())


class FeedForward(nn.Module):
    def __init__(self, dim, hidden_dim, dropout=0.0):
        super().__init__()
        self.net = nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, hidden_dim), nn.SiLU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, dim), nn.Dropout(dropout))

    def forward(self, x):
        return self.net(x)


class Attention(nn.Module):
    """Pre-norm multi-head self-attention over the tokens of each patch pixel (:68-98)."""

    def __init__(self, dim, heads=8, dim_head=64, dropout=0.0):
        super().__init__()
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.norm = nn.LayerNorm(dim)
        self.attend = nn.Softmax(dim=-1)
        self.dropout = nn.Dropout(dropout)
        self.to_qkv = nn.Linear(dim, 3 * heads * dim_head, bias=False)
        self.to_out = nn.Sequential(nn.Linear(heads * dim_head, dim), nn.Dropout(dropout))

    def forward(self, x):
        b, p, n, _ = x.shape
        # [b, p, n, 3*h*d] -> q, k, v each [b, p, h, n, d]
        q, k, v = (t.view(b, p, n, self.heads, -1).transpose(2, 3) for t in self.to_qkv(self.norm(x)).chunk(3, dim=-1))
        attn = self.dropout(self.attend(torch.matmul(q, k.transpose(-1, -2)) * self.scale))
        out = torch.matmul(attn, v).transpose(2, 3).reshape(b, p, n, -1)
        return self.to_out(out)


class Transformer(nn.Module):
    def __init__(self, dim, depth, heads, dim_head, mlp_dim, dropout=0.0):
        super().__init__()
        self.layers = nn.ModuleList(
            nn.ModuleList([Attention(dim, heads, dim_head, dropout), FeedForward(dim, mlp_dim, dropout)])
            for _ in range(depth))

    def forward(self, x):
        for attn, ff in self.layers:
            x = x + attn(x)
            x = x + ff(x)
        return x


def _quantized_error_sum(modules):
    err, n = 0.0, 0
    for m in modules:
        if isinstance(m, QuantizedConv2d):
            e, k = m.get_quantization_error()
            err, n = err + e, n + k
    return err, n


class MV2Block(nn.Module):
    """MobileNetV2 inverted residual with SiLU (:131-233)."""

    def __init__(self, inp, oup, stride=1, expansion=4, quantize_fn: Optional[Callable] = None, bits: int = 4):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError("stride must be 1 or 2")
        self.stride = stride
        hidden = int(inp * expansion)
        self.use_res_connect = stride == 1 and inp == oup

        def qconv(cin, cout, k, s, groups=1):
            return QuantizedConv2d(cin, cout, k, s, k // 2, groups=groups, bias=False, quantize_fn=quantize_fn,
                                   bits=bits)

        layers = []
        if expansion != 1:
            layers += [qconv(inp, hidden, 1, 1), nn.BatchNorm2d(hidden), nn.SiLU()]
        layers += [qconv(hidden, hidden, 3, stride, groups=hidden), nn.BatchNorm2d(hidden), nn.SiLU()]
        layers += [qconv(hidden, oup, 1, 1), nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        if can_fuse(*self.conv) and fusable_sequence(self.conv):
            return run_inverted_residual(self.conv, x, residual=x if self.use_res_connect else None)
        y = self.conv(x)
        return y + x if self.use_res_connect else y

    def get_quantization_error(self):
        return _quantized_error_sum(self.conv)


class MobileViTBlock(nn.Module):
    def __init__(self, dim, depth, channel, kernel_size, patch_size, mlp_dim, dropout: float = 0.0,
                 quantize_fn: Optional[Callable] = None, bits: int = 4):
        super().__init__()
        self.ph, self.pw = patch_size
        q = dict(quantize_fn=quantize_fn, bits=bits)
        self.conv1 = quantized_conv_nxn_bn(channel, channel, kernel_size, **q)
        self.conv2 = quantized_conv_1x1_bn(channel, dim, **q)
        self.transformer = Transformer(dim, depth, 4, 8, mlp_dim, dropout)
        self.conv3 = quantized_conv_1x1_bn(dim, channel, **q)
        self.conv4 = quantized_conv_nxn_bn(2 * channel, channel, kernel_size, **q)

    def _conv(self, seq, x):
        if can_fuse(*seq) and fusable_sequence(seq):
            return run_fused_sequence(seq, x)
        return seq(x)

    def forward(self, x):
        y = x.clone()
        x = self._conv(self.conv2, self._conv(self.conv1, x))  # local representation
        b, d, H, W = x.shape
        ph, pw = self.ph, self.pw
        h, w = H // ph, W // pw
        # "b d (h ph) (w pw) -> b (ph pw) (h w) d"
        t = x.view(b, d, h, ph, w, pw).permute(0, 3, 5, 2, 4, 1).reshape(b, ph * pw, h * w, d)
        t = self.transformer(t)  # global representation
        # "b (ph pw) (h w) d -> b d (h ph) (w pw)"
        x = t.view(b, ph, pw, h, w, d).permute(0, 5, 3, 1, 4, 2).reshape(b, d, H, W)
        return self._conv(self.conv4, torch.cat((self._conv(self.conv3, x), y), 1))  # fusion

    def get_quantization_error(self):
        err, n = 0.0, 0
        for seq in (self.conv1, self.conv2, self.conv3, self.conv4):
            e, k = _quantized_error_sum(seq)
            err, n = err + e, n + k
        return err, n


class _SpatialMean(nn.Module):
    """einops Reduce('b c h w -> b c', 'mean') (:447); holds no state."""

    def forward(self, x):
        return x.mean(dim=(2, 3))


class MobileViT(nn.Module):
    def __init__(self, image_size, dims, channels, num_classes, expansion=4, kernel_size=3, patch_size=(1, 1),
                 depths=(2, 4, 3), quantize_fn: Optional[Callable] = None, bits: int = 4):
        super().__init__()
        if len(dims) != 3:
            raise AssertionError("dims must be a tuple of 3")
        if len(depths) != 3:
            raise AssertionError("depths must be a tuple of 3")
        ih, iw = image_size
        ph, pw = patch_size
        if ih % ph or iw % pw:
            raise AssertionError("image size must be divisible by the patch size")
        q = dict(quantize_fn=quantize_fn, bits=bits)
        c = channels
        self.conv1 = conv_nxn_bn(3, c[0], stride=2)
        # stem: note the reference's 4th block is MV2Block(c[2], c[3]) (:352-360)
        self.stem = nn.ModuleList([MV2Block(c[0], c[1], 1, expansion, **q), MV2Block(c[1], c[2], 2, expansion, **q),
                                   MV2Block(c[2], c[3], 1, expansion, **q), MV2Block(c[2], c[3], 1, expansion, **q)])
        mlp_mult = (2, 4, 4)
        self.trunk = nn.ModuleList(
            nn.ModuleList([MV2Block(c[3 + 2 * i], c[4 + 2 * i], 2, expansion, **q),
                           MobileViTBlock(dims[i], depths[i], c[5 + 2 * i], kernel_size, patch_size,
                                          int(dims[i] * mlp_mult[i]), **q)])
            for i in range(3))
        self.to_logits = nn.Sequential(conv_1x1_bn(c[-2], c[-1]), _SpatialMean(),
                                       nn.Linear(c[-1], num_classes, bias=False))

    def forward(self, x):
        with batched_packs(self, x):  # eval: the single-conv layers' weight packs as batched launches
            x = run_sequence(self.conv1, x)  # unquantized stem: one native fp32 call in eval
            for blk in self.stem:
                x = blk(x)
            for mv2, vit in self.trunk:
                x = vit(mv2(x))
            x = run_sequence(self.to_logits[0], x)
        for m in list(self.to_logits)[1:]:
            x = m(x)
        return x

    def get_quantization_error(self):
        # Same value as the reference (:475-486): the stem is visited twice and the
        # trunk not at all (`_get_quantization_error_for_layer(self.stem)` twice).
        err, n = 0.0, 0
        for blk in self.stem:
            e, k = blk.get_quantization_error()
            err, n = err + e, n + k
        return 2 * err, 2 * n


def MobileVIT(*, num_classes: int = 10, quantize_fn: Optional[Callable] = None, bits: int = 4,
              image_size: Tuple[int], **kwargs: Any) -> MobileViT:
    # mobilevit_xs dims / channels (:497-505); 1x1 patches at CIFAR size, 2x2 otherwise
    channels = (16, 32, 48, 48, 64, 64, 80, 80, 96, 96, 384)
    dims = (96, 120, 144)
    patch = (1, 1) if image_size == (32, 32) else (2, 2)  # a list never equals the tuple (as in :507)
    return MobileViT(num_classes=num_classes, quantize_fn=quantize_fn, bits=bits, image_size=image_size, dims=dims,
                     channels=channels, patch_size=patch, **kwargs)
