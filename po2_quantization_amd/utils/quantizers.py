"""Drop-in quantizer plugins (mirror of the reference's utils/quantizers.py).

Same names, call forms and error behaviour as the reference:
  PowerOfTwoQuantizer.apply(w, bits[, fsr])        utils/quantizers.py:19-36
  PowerOfTwoPlusQuantizer.apply(w, bits[, fsr])    utils/quantizers.py:39-56
  Q.forward(None, w, bits=bits)                    static call used by quantize_model (:148)
  quantize_model(model, quantizer, bits) -> float  utils/quantizers.py:139-153
  quantizer_dict {"lin", "lin+", "po2", "po2+"}    utils/quantizers.py:156-161

PO2 / PO2+ on fp32 HIP tensors run on the hand-written HIP kernels of libpo2q.
The reference's quantizers take any tensor (they are plain torch ops), so CPU,
fp64 and bf16 inputs go to _lib.restated_quantize, the product-side torch
restatement of the same threshold-table decision (bit-exact with the reference
on tests/golden/quant_kat_dtypes.npz).  Backward is the straight-through estimator of the
reference (:34-36, :54-56).

LinearPowerOfTwo(Plus)Quantizer (utils/quantizers.py:59-136)
run on the native per-channel kernel po2q_quantize_lin_f32 (po2q_lin.hip) for fp32
HIP 4-D weights, and on _lib.restated_quantize_lin (the reference's torch ops) for
CPU tensors.
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


class LinearPowerOfTwoQuantizer(torch.autograd.Function):
    """Per-input-channel uniform grid with a power-of-two step refit num_iters times
    (utils/quantizers.py:59-96)."""

    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, num_iters: int = 10):
        return _lib.quantize_lin(input, bits, plus=False, num_iters=num_iters)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output, None, None


class LinearPowerOfTwoPlusQuantizer(torch.autograd.Function):
    """lin with the step snapped as 2^round(log2(sqrt(8/9) delta)) (utils/quantizers.py:99-136)."""

    @staticmethod
    def forward(ctx, input: torch.Tensor, bits: int = 4, num_iters: int = 10):
        return _lib.quantize_lin(input, bits, plus=True, num_iters=num_iters)

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
