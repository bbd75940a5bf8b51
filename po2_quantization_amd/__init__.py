"""po2_quantization_amd — MI355X-native power-of-two quantized convolution.

Drop-in for the hot path of mschoenb97/po2_quantization:
  from po2_quantization_amd.utils.quantizers import quantizer_dict, quantize_model
  from po2_quantization_amd.models.quantized_conv import QuantizedConv2d
  from po2_quantization_amd.models.model import get_model
Kernels: po2_quantization_amd/csrc (HIP, gfx950) behind the C ABI include/po2q.h.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
