"""QAT training-step throughput (config 2: ResNet56, CIFAR 32x32,
bs=256, po2 4-bit): forward (fused native quantize + conv) + STE backward + SGD step, eager and
replayed from one HIP graph (qat.GraphedTrainStep),
against the same step with the reference's torch-op QuantizedConv2d.forward
(quantize in torch ops via the native quantizer + F.conv2d; quantized_conv.py:32-38).
GPU only; one JSON line per configuration.  Synthetic data."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import qat  # noqa: E402
from po2_quantization_amd.models import quantized_conv as QC  # noqa: E402
from po2_quantization_amd.utils.quantizers import quantizer_dict  # noqa: E402


def torch_forward(self, input):
    qw = self.quantize_fn.apply(self.weight, self.bits)
    w = self.weight + (qw - self.weight).detach()
    return F.conv2d(input, w, self.bias, self.stride, self.padding, self.dilation, self.groups)


def run(model_type, qn, bits, bs, steps=20, warmup=5, graph=False):
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    m = qat.build_model(model_type, 10, quantizer_dict[qn], bits, (32, 32), dev)
    opt, _, _, _ = qat.make_optimizer(m, 0.1, 200)
    crit = torch.nn.CrossEntropyLoss()
    x = torch.randn(bs, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (bs,), device=dev)
    if graph:  # the whole step replayed from one HIP graph (qat.GraphedTrainStep)
        gs = qat.GraphedTrainStep(m, opt, crit, x, y)
        step = lambda: gs.step(x, y)  # noqa: E731
    else:
        step = lambda: qat.train_step(m, opt, crit, x, y)  # noqa: E731
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        step()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    return ms, bs / ms * 1e3


def main():
    # MIOpen find (QAT_BENCH_FIND=1) and the po2q autotuner (always)
    torch.backends.cudnn.benchmark = os.environ.get("QAT_BENCH_FIND", "0") == "1"
    from po2_quantization_amd import _lib
    _lib.benchmark = True
    only = sys.argv[1:]  # e.g. `qat_bench.py resnet56`
    for model_type, qn, bits in (("resnet56", "po2", 4), ("resnet20", "po2", 4)):
        if only and model_type not in only:
            continue
        ms, ips = run(model_type, qn, bits, 256)
        ms_g, ips_g = run(model_type, qn, bits, 256, graph=True)
        QC.NATIVE_BACKWARD = False
        try:
            ms_a, ips_a = run(model_type, qn, bits, 256)
        finally:
            QC.NATIVE_BACKWARD = True
        orig = QC.QuantizedConv2d.forward
        QC.QuantizedConv2d.forward = torch_forward
        try:
            ms_t, ips_t = run(model_type, qn, bits, 256)
        finally:
            QC.QuantizedConv2d.forward = orig
        print(json.dumps({"model": model_type, "quantizer": qn, "bits": bits, "batch": 256, "image": 32,
                          "native_ms_per_step": round(ms, 3), "native_images_per_s": round(ips, 1),
                          "graph_ms_per_step": round(ms_g, 3), "graph_images_per_s": round(ips_g, 1),
                          "aten_backward_ms_per_step": round(ms_a, 3), "aten_backward_images_per_s": round(ips_a, 1),
                          "miopen_find": torch.backends.cudnn.benchmark,
                          "torch_forward_ms_per_step": round(ms_t, 3),
                          "torch_forward_images_per_s": round(ips_t, 1)}), flush=True)


if __name__ == "__main__":
    main()
