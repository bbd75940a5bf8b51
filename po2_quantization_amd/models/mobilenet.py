"""MobileNetV2 (CIFAR head) built on the drop-in QuantizedConv2d -- config 3's graph.

Caller of the hot path (reference models/mobilenet.py:17-224).
The module tree reproduces the reference's nesting exactly, so state_dict keys
(and therefore the reference's checkpoints) match one for one:

  features[0]        Sequential(Conv2d 3->32 3x3 s2, BN, ReLU6)   not quantized (:41-46, :167)
  features[1..17]    InvertedResidual, settings (t, c, n, s) of :153-161
                     .conv = [dw3x3, BN, ReLU6, pw1x1, BN]                  (t == 1, :60-87)
                           = [pw1x1, BN, ReLU6, dw3x3, BN, ReLU6, pw1x1, BN] (t > 1,  :89-127)
                     every conv of a block is a QuantizedConv2d (depthwise: groups=C)
  conv               Sequential(Conv2d 320->1280 1x1, BN, ReLU6)  not quantized (:185)
  avgpool, classifier

On the HIP path: the depthwise 3x3 convs run `conv_depthwise`, the pointwise
1x1 convs the bf16x3 implicit GEMM (po2q_conv_x3*.hip), both fused with the
PO2/PO2+ quantizer.  BatchNorm is nn.BatchNorm2d: identical to the reference's
nn.SyncBatchNorm in eval (no collective) and the same state_dict entries.
"""
import math
from typing import Any, Callable, Optional

import torch.nn as nn

from .quantized_conv import (QuantizedConv2d, batched_packs, can_fuse, fusable_sequence, run_fused_sequence,
                             run_inverted_residual, run_sequence)

# (expand ratio t, output channels c, repeats n, first stride s) -- mobilenet.py:153-161
MOBILENET_V2_SETTINGS = ((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2),
                         (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1))


def _make_divisible(v: float, divisor: int, min_value: Optional[int] = None) -> int:
    """Round v to a multiple of divisor, never more than 10 % below v (mobilenet.py:17-24)."""
    lo = divisor if min_value is None else min_value
    r = max(lo, (int(v + divisor / 2) // divisor) * divisor)
    return r + divisor if r < 0.9 * v else r


def _plain_conv_bn(cin: int, cout: int, k: int, stride: int) -> nn.Sequential:
    """Unquantized conv + BN + ReLU6 (the stem and the last 1x1, mobilenet.py:37-50)."""
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, k // 2, bias=False), nn.BatchNorm2d(cout),
                         nn.ReLU6(inplace=True))


def quantized_conv_3x3_bn(inp, oup, stride, quantize_fn=None, bits=4):
    """QuantizedConv2d 3x3 + BN + ReLU6 (mobilenet.py:27-34; unused by MobileNetV2 itself)."""
    return nn.Sequential(QuantizedConv2d(inp, oup, 3, stride, 1, bias=False, quantize_fn=quantize_fn, bits=bits),
                         nn.BatchNorm2d(oup), nn.ReLU6(inplace=True))


class InvertedResidual(nn.Module):
    """Expand (1x1) -> depthwise 3x3 -> project (1x1), identity shortcut when shapes allow."""

    def __init__(self, inp, oup, stride, expand_ratio, quantize_fn=None, bits=4):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError("stride must be 1 or 2")
        hidden = round(inp * expand_ratio)
        self.identity = stride == 1 and inp == oup

        def qconv(cin, cout, k, s, groups=1):
            return QuantizedConv2d(cin, cout, k, s, k // 2, groups=groups, bias=False,
                                   quantize_fn=quantize_fn, bits=bits)

        layers = []
        if expand_ratio != 1:  # pointwise expansion
            layers += [qconv(inp, hidden, 1, 1), nn.BatchNorm2d(hidden), nn.ReLU6(inplace=True)]
        layers += [qconv(hidden, hidden, 3, stride, groups=hidden), nn.BatchNorm2d(hidden), nn.ReLU6(inplace=True)]
        layers += [qconv(hidden, oup, 1, 1), nn.BatchNorm2d(oup)]  # linear bottleneck
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        if can_fuse(*self.conv) and fusable_sequence(self.conv):
            return run_inverted_residual(self.conv, x, residual=x if self.identity else None)
        y = self.conv(x)
        return x + y if self.identity else y

    def get_quantization_error(self):
        err, n = 0.0, 0
        for m in self.conv:
            if isinstance(m, QuantizedConv2d):
                e, k = m.get_quantization_error()
                err, n = err + e, n + k
        return err, n


class MobileNet(nn.Module):
    def __init__(self, num_classes: int = 10, width_mult: float = 1.0, quantize_fn: Optional[Callable] = None,
                 bits: int = 4):
        super().__init__()
        self.cfgs = [list(s) for s in MOBILENET_V2_SETTINGS]
        div = 4 if width_mult == 0.1 else 8
        cin = _make_divisible(32 * width_mult, div)
        blocks = [_plain_conv_bn(3, cin, 3, 2)]
        for t, c, n, s in MOBILENET_V2_SETTINGS:
            cout = _make_divisible(c * width_mult, div)
            for i in range(n):
                blocks.append(InvertedResidual(cin, cout, s if i == 0 else 1, t, quantize_fn=quantize_fn, bits=bits))
                cin = cout
        self.features = nn.Sequential(*blocks)
        last = _make_divisible(1280 * width_mult, div) if width_mult > 1.0 else 1280
        self.conv = _plain_conv_bn(cin, last, 1, 1)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.classifier = nn.Linear(last, num_classes)
        self._initialize_weights()

    def forward(self, x):
        with batched_packs(self, x):  # eval: every layer's weight pack as batched launches
            for m in self.features:  # the unquantized stem (features[0]) natively fused in eval too
                x = run_sequence(m, x) if isinstance(m, nn.Sequential) else m(x)
            x = self.avgpool(run_sequence(self.conv, x))
        return self.classifier(x.flatten(1))

    def _initialize_weights(self):
        # mobilenet.py:205-216: N(0, sqrt(2/(k*k*out))) convs, unit BN, N(0, 0.01) Linear
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, math.sqrt(2.0 / (m.kernel_size[0] * m.kernel_size[1] * m.out_channels)))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()

    def get_quantization_error(self):
        # reference mobilenet.py:218-237: the InvertedResidual blocks of `features`.
        # The reference's `numel += numel` (:235) doubles the element count; kept so the
        # per-element error it reports (train.py) is the same number.
        err, n = 0.0, 0
        for m in self.features:
            if isinstance(m, InvertedResidual):
                e, k = m.get_quantization_error()
                err, n = err + e, n + k
        return err, 2 * n


def MobileNetV2(*, num_classes: int = 10, quantize_fn: Optional[Callable] = None, bits: int = 4,
                **kwargs: Any) -> MobileNet:
    return MobileNet(num_classes=num_classes, quantize_fn=quantize_fn, bits=bits, **kwargs)
