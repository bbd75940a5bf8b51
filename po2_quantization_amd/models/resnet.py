"""CIFAR-style ResNet20/32/44/56 built on the drop-in QuantizedConv2d.

Caller of the hot path (models/resnet.py:10-300 in the
reference): same constructors, same module names and state_dict keys, so the
reference's checkpoints load unchanged (after stripping DDP's "module."
prefix, test.py:50-55).  Structure per the reference:
  stem    3x3 conv 3->16, NOT quantized (resnet.py:99-102) + BN + ReLU
  stages  n BasicBlocks each at 16 / 32 / 64 channels, stride 1 / 2 / 2;
          block = qconv3x3 -> BN -> ReLU -> qconv3x3 -> BN (+ 1x1 qconv + BN
          projection when the shape changes) -> add -> ReLU
  head    global average pool -> Linear
BatchNorm layers are nn.BatchNorm2d: for inference (eval) this is exactly the
reference's nn.SyncBatchNorm, which issues no collective in eval mode.
"""
from typing import Callable, Optional

import torch
import torch.nn as nn

from .. import _lib
from ..utils.quantizers import NATIVE_MODES
from .quantized_conv import (QuantizedConv2d, batched_packs, can_fuse, fold_bn, plain_conv, plain_conv_fused,
                             run_fused_sequence)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, quantize_fn=None, bits=7):
        super().__init__()
        qc = dict(bias=False, quantize_fn=quantize_fn, bits=bits)
        self.conv1 = QuantizedConv2d(inplanes, planes, 3, stride=stride, padding=1, **qc)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = QuantizedConv2d(planes, planes, 3, stride=1, padding=1, **qc)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if can_fuse(self.bn1, self.bn2, self.downsample):
            # inference: conv+BN+ReLU and conv+BN+add+ReLU as single native calls
            if self._pair_ok(x):
                # conv1 -> bn1 -> relu -> conv2 -> bn2 -> + x -> relu as ONE launch, the
                # intermediate kept on chip (po2q_qconv2d_pair_f32)
                ps1, pb1 = fold_bn(self.bn1)
                ps2, pb2 = fold_bn(self.bn2)
                return _lib.qconv2d_pair(x, self.conv1.weight, self.conv2.weight, self.conv1.bits,
                                         NATIVE_MODES[self.conv1.quantize_fn], post_scale1=ps1, post_shift1=pb1,
                                         act1="relu", post_scale2=ps2, post_shift2=pb2, residual=x, act2="relu")
            if self._s2ds_ok(x):
                # conv1 -> bn1 -> relu and downsample (1x1 conv -> bn) on ONE read of x
                # (po2q_qconv2d_s2ds_f32), then conv2 -> bn2 -> + shortcut -> relu
                ps1, pb1 = fold_bn(self.bn1)
                psd, pbd = fold_bn(self.downsample[1])
                out, shortcut = _lib.qconv2d_s2ds(x, self.conv1.weight, self.downsample[0].weight, self.conv1.bits,
                                                  NATIVE_MODES[self.conv1.quantize_fn], post_scale=ps1,
                                                  post_shift=pb1, act="relu", post_scale_ds=psd, post_shift_ds=pbd)
                return self.conv2.fused(out, bn=self.bn2, residual=shortcut, act="relu")
            shortcut = x if self.downsample is None else run_fused_sequence(self.downsample, x)
            out = self.conv1.fused(x, bn=self.bn1, act="relu")
            return self.conv2.fused(out, bn=self.bn2, residual=shortcut, act="relu")
        shortcut = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out += shortcut
        return self.relu(out)

    def _pair_ok(self, x):
        """Both convs eligible for the pair kernel: identity shortcut, 16 or 32 channels, stride 1,
        the same native PO2 quantizer and bits, bf16x3 arithmetic allowed."""
        c1, c2 = self.conv1, self.conv2
        mode = NATIVE_MODES.get(c1.quantize_fn)
        geom = all(tuple(c.kernel_size) == (3, 3) and tuple(c.stride) == (1, 1) and tuple(c.padding) == (1, 1)
                   and tuple(c.dilation) == (1, 1) and c.groups == 1 and c.padding_mode == "zeros" for c in (c1, c2))
        return (self.downsample is None and geom and mode in ("po2", "po2+") and c2.quantize_fn is c1.quantize_fn
                and c1.bits == c2.bits and c1.in_channels in (16, 32) and c1.out_channels == c1.in_channels
                and c2.in_channels == c1.in_channels and c2.out_channels == c1.in_channels and c1.precision != "fp32"
                and c2.precision != "fp32" and c1.bias is None and c2.bias is None
                and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and _lib.pair_supported(x.shape, c1.bits, mode))

    def _s2ds_ok(self, x):
        """conv1 (3x3 stride 2, C -> 2C) and the projection shortcut (QuantizedConv2d 1x1 stride 2 +
        BatchNorm, models/resnet.py:100-105) eligible for the fused stride-2 kernel: same native PO2
        quantizer and bits, bf16x3 arithmetic allowed, no biases."""
        c1, ds = self.conv1, self.downsample
        if (ds is None or len(ds) != 2 or not isinstance(ds[0], QuantizedConv2d)
                or not isinstance(ds[1], nn.modules.batchnorm._BatchNorm)):
            return False
        d = ds[0]
        mode = NATIVE_MODES.get(c1.quantize_fn)
        return (mode in ("po2", "po2+") and d.quantize_fn is c1.quantize_fn and d.bits == c1.bits
                and c1.in_channels in (16, 32) and c1.out_channels == 2 * c1.in_channels
                and tuple(c1.kernel_size) == (3, 3) and tuple(c1.stride) == (2, 2) and tuple(c1.padding) == (1, 1)
                and tuple(c1.dilation) == (1, 1) and c1.padding_mode == "zeros" and d.padding_mode == "zeros"
                and tuple(d.dilation) == (1, 1)
                and d.in_channels == c1.in_channels and d.out_channels == c1.out_channels
                and tuple(d.kernel_size) == (1, 1) and tuple(d.stride) == (2, 2) and tuple(d.padding) == (0, 0)
                and c1.groups == 1 and d.groups == 1 and c1.bias is None and d.bias is None
                and c1.precision != "fp32" and d.precision != "fp32"
                and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and _lib.s2ds_supported(x.shape, c1.bits, mode))

    def get_quantization_error(self):
        e1, n1 = self.conv1.get_quantization_error()
        e2, n2 = self.conv2.get_quantization_error()
        return e1 + e2, n1 + n2


class ResNet(nn.Module):
    def __init__(self, block=BasicBlock, num_blocks=(3, 3, 3), num_filters=(16, 32, 64), num_classes=10,
                 quantize_fn: Optional[Callable] = None, bits: int = 7):
        super().__init__()
        self.inplanes = 16
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        strides = (1, 2, 2)
        for i, (planes, blocks, st) in enumerate(zip(num_filters, num_blocks, strides)):
            setattr(self, "layer%d" % (i + 1),
                    self._make_layer(block, planes, blocks, st, quantize_fn, bits))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(num_filters[2] * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride, quantize_fn, bits):
        out_planes = planes * block.expansion
        downsample = None
        if stride != 1 or self.inplanes != out_planes:
            downsample = nn.Sequential(
                QuantizedConv2d(self.inplanes, out_planes, 1, stride=stride, padding=0, bias=False,
                                quantize_fn=quantize_fn, bits=bits),
                nn.BatchNorm2d(out_planes),
            )
        layers = [block(self.inplanes, planes, stride, downsample, quantize_fn=quantize_fn, bits=bits)]
        self.inplanes = out_planes
        layers += [block(self.inplanes, planes, quantize_fn=quantize_fn, bits=bits) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        with batched_packs(self, x):  # eval: the single-conv layers' weight packs as batched launches
            if can_fuse(self.bn1) and x.is_cuda and x.dtype == torch.float32:
                # the unquantized stem conv + bn1 + relu (resnet.py:99-102, 191) as one native fp32 call
                x = plain_conv_fused(self.conv1, x, bn=self.bn1, act="relu")
            else:
                x = self.relu(self.bn1(plain_conv(self.conv1, x)))  # native forward + backward
            for layer in (self.layer1, self.layer2, self.layer3):
                x = self._stage(layer, x)
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def _stage(self, layer, x):
        """One residual stage (resnet.py:131-143 builds it).  In inference at small image sizes the
        stage's identity-shortcut blocks run as ONE chain launch (po2q_qconv2d_chain_f32: every
        block's conv1 -> bn1 -> relu -> conv2 -> bn2 -> + block input -> relu, one GPU block per
        image); its first block, when it carries the projection shortcut, runs on its own first."""
        blocks = list(layer)
        i0 = 1 if blocks and isinstance(blocks[0], BasicBlock) and blocks[0].downsample is not None else 0
        run = blocks[i0:]
        if not run or not self._chain_ok(run, x if i0 == 0 else None):
            return layer(x)
        if i0:
            x = blocks[0](x)
        if not self._chain_ok(run, x):
            for b in run:
                x = b(x)
            return x
        ws, bs, ps, pb, res = [], [], [], [], []
        for b in run:
            p1, s1 = fold_bn(b.bn1)
            p2, s2 = fold_bn(b.bn2)
            res += [-1, len(ws)]  # conv2's shortcut: the block input = conv1's input
            ws += [b.conv1.weight, b.conv2.weight]
            bs += [b.conv1.bias, b.conv2.bias]
            ps += [p1, p2]
            pb += [s1, s2]
        c = run[0].conv1
        return _lib.qconv2d_chain(x, ws, c.bits, NATIVE_MODES[c.quantize_fn], biases=bs, post_scales=ps,
                                  post_shifts=pb, acts=["relu"] * len(ws), res_from=res)

    @staticmethod
    def _chain_ok(run, x):
        """Every block a BasicBlock with an identity shortcut, eval BatchNorms, 3x3 / stride-1 C -> C
        convs with the same native PO2 quantizer and bits; with x: the chain kernel takes the shape."""
        c0 = run[0].conv1 if isinstance(run[0], BasicBlock) else None
        if c0 is None:
            return False
        mode = NATIVE_MODES.get(c0.quantize_fn)
        if mode not in ("po2", "po2+") or c0.precision == "fp32":
            return False
        for b in run:
            if not isinstance(b, BasicBlock) or b.downsample is not None or not can_fuse(b.bn1, b.bn2):
                return False
            for c in (b.conv1, b.conv2):
                if not (isinstance(c, QuantizedConv2d) and c.quantize_fn is c0.quantize_fn and c.bits == c0.bits
                        and c.precision == c0.precision and tuple(c.kernel_size) == (3, 3)
                        and tuple(c.stride) == (1, 1) and tuple(c.padding) == (1, 1) and tuple(c.dilation) == (1, 1)
                        and c.groups == 1 and c.padding_mode == "zeros" and c.in_channels == c0.in_channels
                        and c.out_channels == c0.in_channels):
                    return False
        if x is None:
            return True
        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == c0.in_channels
                and _lib.chain_supported(x.shape, 2 * len(run), c0.bits, NATIVE_MODES[c0.quantize_fn]))

    def get_quantization_error(self):
        """(sum of squared quantization error, element count) over the residual stages.

        Same value as the reference (resnet.py:203-224), quirks included so the
        per-element error train.py logs is unchanged: projection convs are not
        visited, and inside a stage the element counter is overwritten by each
        block and then doubled (`qerror, numel = ...; numel += numel`), so a
        stage contributes 2 x its last block's count."""
        err, num = 0.0, 0
        for layer in (self.layer1, self.layer2, self.layer3):
            stage_n = 0
            for blk in layer:
                if isinstance(blk, BasicBlock):
                    e, stage_n = blk.get_quantization_error()
                    err = err + e
                    stage_n = 2 * stage_n
            num += stage_n
        return err, num


def _resnet(n, num_classes=10, quantize_fn=None, bits=4, **kwargs):
    return ResNet(BasicBlock, (n, n, n), (16, 32, 64), num_classes=num_classes, quantize_fn=quantize_fn,
                  bits=bits, **kwargs)


def ResNet20(*, n=3, num_classes=10, quantize_fn=None, bits=4, **kwargs):
    return _resnet(n, num_classes, quantize_fn, bits, **kwargs)


def ResNet32(*, n=5, num_classes=10, quantize_fn=None, bits=4, **kwargs):
    return _resnet(n, num_classes, quantize_fn, bits, **kwargs)


def ResNet44(*, n=7, num_classes=10, quantize_fn=None, bits=4, **kwargs):
    return _resnet(n, num_classes, quantize_fn, bits, **kwargs)


def ResNet56(*, n=9, num_classes=10, quantize_fn=None, bits=4, **kwargs):
    return _resnet(n, num_classes, quantize_fn, bits, **kwargs)
