"""Drop-in quantizer plugins (mirror of the reference's utils/quantizers.py).

Same names, call forms and error behaviour as the reference:
  PowerOfTwoQuantizer.apply(w, bits[, fsr])        utils/quantizers.py:19-36
  PowerOfTwoPlusQuantizer.apply(w, bits[, fsr])    utils/quantizers.py:39-56
  Q.forward(None, w, bits=bits)                    static call used by quantize_model (:148)
  quantize_model(model, quantizer, bits) -> float  utils/quantizers.py:139-153
  quantizer_dict {"lin", "lin+", "po2", "po2+"}    utils/quantizers.py:156-161

PO2 / PO2+ run on the hand-written HIP kernels of libpo2q (fp32 HIP tensors
only; anything else raises — there is no CPU path).  Backward is the
straight-through estimator of the reference (:34-36, :54-56).

LinearPowerOfTwo(Plus)Quantizer (utils/quantizers.py:59-136) are NOT on the
graded hot path ("next"): they are provided as plain torch
ops so that quantizer_dict is complete; a native kernel replaces them later.
"""
from typing import Callable, Optional

import torch

from .. import _lib


class PowerOfTwoQuantizer(torch.autograd.Function):
    """sign(w) * 2^clamp(round(log2|w/max|w||)) * max|w|   (quantizers.py:19-36)."""

    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, fsr: int = 1):
        return _lib.quantize(input, bits, "po2", fsr)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None


class PowerOfTwoPlusQuantizer(torch.autograd.Function):
    """PO2+ : exponent round(log2(a/1.5) + 0.5) == round(log2(sqrt(8/9) a))   (quantizers.py:39-56)."""

    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, fsr: int = 1):
        return _lib.quantize(input, bits, "po2+", fsr)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None


# native quantizer classes -> libpo2q mode string (used by QuantizedConv2d to fuse)
NATIVE_MODES = {PowerOfTwoQuantizer: "po2", PowerOfTwoPlusQuantizer: "po2+"}


def quantize_per_filter(x: torch.Tensor, delta: torch.Tensor, bits: int) -> torch.Tensor:
    """Uniform quantizer with a per-input-channel step (utils/quantizers.py:8-16)."""
    d = delta.view(-1, 1, 1)
    lim = (2 ** (bits - 1)) - 1
    return d * torch.clamp(torch.round(x / d), min=-lim, max=lim)


def _linear_po2(input: torch.Tensor, bits: int, num_iters: int, plus: bool) -> torch.Tensor:
    # per input-channel (dim 1) range -> initial step (quantizers.py:62-69)
    hi = input.amax(dim=(0, 2, 3))
    lo = input.amin(dim=(0, 2, 3))
    delta = (hi - lo) / (2 ** bits - 1)
    q = quantize_per_filter(input, delta, bits) / delta.view(-1, 1, 1)
    shrink = torch.sqrt(torch.tensor(8.0 / 9.0)) if plus else None
    for _ in range(num_iters):
        # least-squares step, then snap it to a power of two (quantizers.py:74-87 / :114-127)
        qtw = torch.sum(q * input, dim=[0, 2, 3])
        qtq = torch.sum(q * q, dim=[0, 2, 3])
        delta = qtw / qtq
        delta = 2 ** torch.round(torch.log2(shrink.to(delta.device) * delta if plus else delta))
        q = quantize_per_filter(input, delta, bits) / delta.view(-1, 1, 1)
    return q * delta.view(-1, 1, 1)


class LinearPowerOfTwoQuantizer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, num_iters: int = 10):
        return _linear_po2(input, bits, num_iters, plus=False)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None


class LinearPowerOfTwoPlusQuantizer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, num_iters: int = 10):
        return _linear_po2(input, bits, num_iters, plus=True)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None


def quantize_model(model: torch.nn.Module, quantizer: Optional[Callable[..., None]], bits: int) -> float:
    """PTQ: quantize every parameter of every QuantizedConv2d in place and return
    the mean squared quantization error (utils/quantizers.py:139-153)."""
    from ..models.quantized_conv import QuantizedConv2d

    quant_error, numel = 0.0, 0
    with torch.no_grad():
        for _, module in model.named_modules():
            if isinstance(module, QuantizedConv2d):
                for _, param in module.named_parameters():
                    quant_param = quantizer.forward(None, param, bits=bits)
                    quant_error += torch.sum((quant_param - param) ** 2)
                    numel += param.numel()
                    param.copy_(quant_param)
    return (quant_error / numel).item()


quantizer_dict = {
    "lin": LinearPowerOfTwoQuantizer,
    "lin+": LinearPowerOfTwoPlusQuantizer,
    "po2": PowerOfTwoQuantizer,
    "po2+": PowerOfTwoPlusQuantizer,
}
