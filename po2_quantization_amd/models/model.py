"""Model factory (mirror of the reference's models/model.py:8-29)."""
from typing import Callable

from .resnet import ResNet20, ResNet32, ResNet44, ResNet56

_RESNETS = {"resnet20": ResNet20, "resnet32": ResNet32, "resnet44": ResNet44, "resnet56": ResNet56}


def get_model(model_type: str, num_classes: int, quantize_fn: Callable, bits: int, image_size=None):
    if model_type in _RESNETS:
        return _RESNETS[model_type](num_classes=num_classes, quantize_fn=quantize_fn, bits=bits)
    if model_type == "mobilenet":
        from .mobilenet import MobileNetV2

        return MobileNetV2(num_classes=num_classes, quantize_fn=quantize_fn, bits=bits)
    if model_type == "mobilevit":
        from .mobile_vit import MobileVIT

        return MobileVIT(num_classes=num_classes, quantize_fn=quantize_fn, bits=bits, image_size=image_size)
    # the reference falls through to `return model` with model unbound (model.py:29)
    raise ValueError("unknown model_type %r" % (model_type,))
