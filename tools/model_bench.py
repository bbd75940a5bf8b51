"""Model-level inference throughput (images/s) of the reference's model graphs on the
drop-in modules, with and without the fused conv epilogue:

    python tools/model_bench.py [--model resnet56 --image 224 --batch 256 --classes 1000]

Synthetic NCHW input, random-init weights (seeded), eval mode, torch.no_grad().
"fused": conv+BN(+add)+act as one native call per conv; "unfused": the reference's
module sequence (native conv, torch BatchNorm / ReLU / add).  GPU only."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from po2_quantization_amd import _lib  # noqa: E402
from po2_quantization_amd.models import quantized_conv  # noqa: E402
from po2_quantization_amd.models.model import get_model  # noqa: E402
from po2_quantization_amd.utils.quantizers import quantizer_dict  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet56")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--quantizer", default="po2")
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph", action="store_true",
                    help="also time the fused forward replayed from a HIP graph (small images: launch-bound)")
    ap.add_argument("--only-fused", action="store_true")
    ap.add_argument("--no-ir", action="store_true",
                    help="inverted-residual blocks as three fused layer calls instead of one block launch")
    ap.add_argument("--ir", action="store_true", help="inverted-residual blocks as one launch where it applies")
    args = ap.parse_args()
    if args.ir or args.no_ir:
        quantized_conv.IR_FUSION = bool(args.ir)
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    m = get_model(args.model, args.classes, quantizer_dict[args.quantizer], args.bits,
                  (args.image, args.image)).to(dev).eval()
    x = torch.randn(args.batch, 3, args.image, args.image, device=dev)
    _lib.benchmark = True  # autotune every conv shape once (cudnn.benchmark counterpart)
    res = {"model": args.model, "image": args.image, "batch": args.batch, "quantizer": args.quantizer,
           "bits": args.bits, "ir_fusion": quantized_conv.IR_FUSION}
    with torch.no_grad():
        for name, fuse in (("fused", True), ("unfused", False)):
            if args.only_fused and not fuse:
                continue
            quantized_conv.INFERENCE_FUSION = fuse
            t = timed(lambda: m(x), args.steps, args.warmup)
            res[name + "_ms"] = round(t * 1e3, 3)
            res[name + "_images_per_s"] = round(args.batch / t, 1)
        if args.graph:
            quantized_conv.INFERENCE_FUSION = True
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                m(x)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m(x)
            t = timed(g.replay, args.steps * 4, args.warmup)
            res["graph_fused_ms"] = round(t * 1e3, 3)
            res["graph_fused_images_per_s"] = round(args.batch / t, 1)
        if not args.only_fused:
            quantized_conv.INFERENCE_FUSION = True
            ya = m(x)
            quantized_conv.INFERENCE_FUSION = False
            yb = m(x)
            quantized_conv.INFERENCE_FUSION = True
            res["fused_vs_unfused_normwise"] = float((ya - yb).abs().max() / yb.abs().max())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
