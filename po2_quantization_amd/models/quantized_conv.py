"""Drop-in QuantizedConv2d (mirror of the reference's models/quantized_conv.py:5-45).

Same constructor signature and defaults (padding=1, bias=False,
quantize_fn=None, bits=4), same parameters / state_dict keys (weight[, bias]),
same get_quantization_error().  forward() runs the fused libpo2q path:

  quantize_fn in {PowerOfTwoQuantizer, PowerOfTwoPlusQuantizer}
      -> one native call: absmax + quantize + pack + conv kernels
  quantize_fn None
      -> native conv of the raw weight (reference :37-38)
  any other quantize_fn (e.g. lin / lin+ or a user Function)
      -> qw = quantize_fn.apply(weight, bits), then the native conv of qw

Backward (QAT) keeps the reference's semantics: straight-through estimator on
the weight (quantizers.py:34-36), conv gradients of the quantized weight.
Inputs must be fp32 HIP tensors; there is no CPU path.
"""
import torch
import torch.nn as nn

from .. import _lib
from ..utils.quantizers import NATIVE_MODES


class _QConv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, groups, bits, mode, precision):
        y = _lib.qconv2d(x, weight, bias, stride, padding, dilation, groups, bits, mode, 1, precision)
        ctx.save_for_backward(x, weight, bias)
        ctx.conf = (stride, padding, dilation, groups, bits, mode)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, bias = ctx.saved_tensors
        stride, padding, dilation, groups, bits, mode = ctx.conf
        qw = weight if mode == "none" else _lib.quantize(weight, bits, mode)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.nn.grad.conv2d_input(x.shape, qw, gy, stride, padding, dilation, groups)
        if ctx.needs_input_grad[1]:  # STE: d qw / d w = 1
            gw = torch.nn.grad.conv2d_weight(x, weight.shape, gy, stride, padding, dilation, groups)
        if bias is not None and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3))
        return gx, gw, gb, None, None, None, None, None, None, None


class QuantizedConv2d(nn.Conv2d):
    # conv arithmetic of the native kernels: "auto" | "fp32" | "bf16x3"
    precision = "auto"

    def __init__(
        self,
        in_channels,
        out_channels,
        kernel_size,
        stride=1,
        padding=1,
        dilation=1,
        groups=1,
        bias=False,
        quantize_fn=None,
        bits=4,
    ):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.quantize_fn = quantize_fn
        self.bits = bits

    def _padding(self, x):
        if isinstance(self.padding, str):
            if self.padding == "valid":
                return (0, 0)
            # 'same' (stride 1): symmetric padding when the total is even
            pads = []
            for d, k in zip(self.dilation, self.kernel_size):
                total = d * (k - 1)
                if total % 2:
                    raise RuntimeError("po2q: padding='same' with asymmetric padding is not supported")
                pads.append(total // 2)
            return tuple(pads)
        return self.padding

    def _native(self, input, weight, mode):
        if self.padding_mode != "zeros":
            raise RuntimeError("po2q: only padding_mode='zeros' is supported (the reference uses the default)")
        unbatched = input.dim() == 3
        x = input.unsqueeze(0) if unbatched else input
        y = _QConv2dFn.apply(x, weight, self.bias, self.stride, self._padding(x), self.dilation, self.groups,
                             self.bits, mode, self.precision)
        return y.squeeze(0) if unbatched else y

    def forward(self, input):
        # reference quantized_conv.py:32-38
        if self.quantize_fn is None:
            return self._native(input, self.weight, "none")
        mode = NATIVE_MODES.get(self.quantize_fn)
        if mode is not None:
            return self._native(input, self.weight, mode)
        quantized_weight = self.quantize_fn.apply(self.weight, self.bits)
        return self._native(input, quantized_weight, "none")

    def get_quantization_error(self):
        # reference quantized_conv.py:40-45
        if self.quantize_fn is not None:
            quantized_weight = self.quantize_fn.apply(self.weight, self.bits)
            return torch.sum((quantized_weight - self.weight) ** 2), self.weight.numel()
        else:
            return 0, self.weight.numel()

