from .quantized_conv import QuantizedConv2d  # noqa: F401
