"""Benchmark: quantized-conv forward images/s, ResNet56 224x224, bs=256 per GPU.

One step = one pass of the hot path over one batch: the 56 QuantizedConv2d
layers of ResNet56 in graph order (each a fused PO2 quantize + conv, i.e. the
reference's QuantizedConv2d.forward, models/quantized_conv.py:32-38), fed by
the previous layer's output, then the classifier head (global avg-pool + fc).
For N > 1 every rank runs its own batch shard and the logits are gathered with
an RCCL all_gather over xGMI (north_star: "inference batches shard across the
GPUs with an RCCL all-gather of outputs"; 1 MB per rank, latency-bound).
Inputs and weights are synthetic (seeded)
and resident in HBM before the timed region.  Each conv shape is autotuned
on its first (untimed, warmup) call, as the reference's cudnn.benchmark does.

  python bench.py [--gpus N --steps K --warmup W]          (N > 1: starts N ranks itself, see below)
  torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, this process starts the N ranks itself:
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py ...` as a
child process, before anything touches the GPU (importing po2_quantization_amd._lib loads no
library), relays rank 0's JSON line and exits with the launcher's status.  Under a launcher the
process group must hold exactly N ranks.
  python bench.py --image 32 --graph                     (config 2: CIFAR 32x32, hipGraph replay)
  torchrun ... bench.py --gpus 8 --global-batch 1024     (config 4: 128 images per GPU)

--graph captures one whole step (every fused quantize+conv launch of the chain + head) in
a HIP graph after the warm-up / autotune steps and times its replays: at 32x32 a layer is
a few microseconds of GPU work, less than the host's launch cost.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from po2_quantization_amd import _lib  # noqa: E402

METRIC = "quantized-conv fwd images/sec, ResNet56 224×224 bs=256; 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3      # MI355X_MICROARCH.md, FP32 matrix (= vector) peak
PEAK_BF16_MFMA_TFLOPS = 2516.6     # dense bf16
PEAK_HBM_GBS = 8000.0              # HBM3E spec


def resnet_qconv_layers(n_blocks):
    """(name, C, K, R, stride, pad, role) of every QuantizedConv2d, graph order
    (reference models/resnet.py:25-50, 150-163): role in {conv1, conv2, ds}."""
    layers, inplanes = [], 16
    for stage, (planes, stride) in enumerate(((16, 1), (32, 2), (64, 2))):
        for b in range(n_blocks):
            st = stride if b == 0 else 1
            pre = "layer%d.%d" % (stage + 1, b)
            layers.append((pre + ".conv1", inplanes, planes, 3, st, 1, "conv1"))
            layers.append((pre + ".conv2", planes, planes, 3, 1, 1, "conv2"))
            if st != 1 or inplanes != planes:
                layers.append((pre + ".downsample.0", inplanes, planes, 1, st, 0, "ds"))
            inplanes = planes
    return layers


def kaiming(K, C, R, gen, dev):
    return (torch.randn(K, C, R, R, generator=gen) * math.sqrt(2.0 / (K * R * R))).to(dev)


class QConvChain:
    def __init__(self, n_blocks, num_classes, mode, bits, precision, dev, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.layers = resnet_qconv_layers(n_blocks)
        self.weights = [kaiming(K, C, R, g, dev) for (_, C, K, R, _, _, _) in self.layers]
        self.fc_w = (torch.randn(num_classes, 64, generator=g) * 0.05).to(dev)
        self.fc_b = torch.zeros(num_classes, device=dev)
        self.mode, self.bits, self.precision = mode, bits, precision
        self.timed_layer = None      # index of the layer whose launches are timed
        self.events = []
        self.pair = True             # conv1 -> conv2 of stage-1 / stage-2 blocks as one pair launch
        self.s2ds = True             # stride-2 conv1 + its 1x1 shortcut of a stage's first block as one launch
        self.packed = None           # _lib.PackedConvs: the single-conv layers' weight packs as one batched launch
        self.packed_idx = {}         # layer index -> PackedConvs index
        self.shapes = {}             # layer index -> input shape (recorded by conv())
        self.chain = True            # small images: a stage's stride-1 run of convs as ONE launch
        self.chains = {}             # first layer index -> (layer indices, input shape) of each chain run

    def conv(self, i, x, direct=False):
        _, C, K, R, st, pad, _ = self.layers[i]
        j = None if direct else self.packed_idx.get(i)
        if j is not None:
            return self.packed.conv(j, x)
        self.shapes[i] = tuple(x.shape)
        return _lib.qconv2d(x, self.weights[i], None, st, pad, 1, 1, self.bits, self.mode, 1, self.precision)

    def pairable(self, i, x):
        """conv1 -> conv2 of block i as ONE launch (po2q_qconv2d_pair_f32): both 3x3 s1 C->C, C = 16 / 32."""
        if not self.pair:
            return False
        (_, C1, K1, R1, s1, _, _), (_, C2, K2, R2, s2, _, _) = self.layers[i], self.layers[i + 1]
        return C1 in (16, 32) and (K1, C2, K2, R1, R2, s1, s2) == (C1, C1, C1, 3, 3, 1, 1) \
            and self.mode in ("po2", "po2+") and _lib.pair_supported(x.shape, self.bits, self.mode)

    def enable_packed(self):
        """After a (autotuning) forward: every layer that ran as a single-conv launch gets its
        weight quantize + pack from one batched launch at the start of each forward
        (_lib.PackedConvs: po2q_qconv2d_plan_pack_batch), then its conv from the packed workspace."""
        idx = sorted(self.shapes)
        specs = [(self.shapes[i], self.weights[i], self.layers[i][4], self.layers[i][5]) for i in idx]
        self.packed = _lib.PackedConvs(specs, self.bits, self.mode)
        self.packed_idx = {i: j for j, i in enumerate(idx)}

    def chain_run(self, i, x):
        """Layers i, i+1, ... up to the end of i's stage (the shortcut of a transition block skipped)
        when they are all 3x3 / stride-1 C -> C convs -- the stage's stride-1 run, from its first
        block's conv2 after a transition -- and po2q_qconv2d_chain takes them on x: one launch, one
        block per image (small images)."""
        if not self.chain or self.mode not in ("po2", "po2+") or self.precision == "fp32":
            return None
        run, j = [], i
        while j < len(self.layers):
            _, C, K, R, st, _, role = self.layers[j]
            if role == "ds":  # a transition's shortcut (computed from the block input, outside the run)
                j += 1
                continue
            if st != 1 or C != K or R != 3:
                break
            if role == "conv1" and j + 2 < len(self.layers) and self.layers[j + 2][6] == "ds":
                break  # the next stage's transition block
            run.append(j)
            j += 1
        if len(run) < 2 or len(run) > _lib.CHAIN_MAX_LAYERS or not _lib.chain_supported(x.shape, len(run), self.bits,
                                                                                          self.mode):
            return None
        return run

    def run_chain(self, run, x):
        self.chains[run[0]] = (run, tuple(x.shape))
        return _lib.qconv2d_chain(x, [self.weights[j] for j in run], self.bits, self.mode)

    def forward(self, x, record=False):
        if self.packed is not None:
            self.packed.pack()  # every single-conv layer's weight, quantized + packed in one launch
        i = 0
        while i < len(self.layers):
            name, _, _, _, _, _, role = self.layers[i]
            assert role == "conv1"
            has_ds = i + 2 < len(self.layers) and self.layers[i + 2][6] == "ds"
            if has_ds:
                # stage transition: stride-2 conv1 (+ the projection shortcut, whose output feeds
                # the add), then conv2 -- with the rest of the stage as one chain where it applies
                if self.s2ds_ok(i, x):
                    # both on one read of x
                    mid, _ = _lib.qconv2d_s2ds(x, self.weights[i], self.weights[i + 2], self.bits, self.mode)
                else:
                    mid = self._timed(i, x, record)
                    self._timed(i + 2, x, record)
                run = self.chain_run(i + 1, mid)
                if run:
                    x = self.run_chain(run, mid)
                    i = run[-1] + 1
                else:
                    x = self._timed(i + 1, mid, record)
                    i += 3
                continue
            run = self.chain_run(i, x)
            if run:
                x = self.run_chain(run, x)
                i = run[-1] + 1
                continue
            if self.pairable(i, x):
                x = self._timed_pair(i, x, record)
            else:
                x = self._timed(i + 1, self._timed(i, x, record), record)
            i += 2
        pooled = x.mean(dim=(2, 3))
        return torch.nn.functional.linear(pooled, self.fc_w, self.fc_b)

    def s2ds_ok(self, i, x):
        """conv1 (3x3 s2 C -> 2C) and downsample.0 (1x1 s2 C -> 2C) of block i as ONE launch."""
        (_, C, K, R, st, _, _), (_, C3, K3, R3, st3, _, _) = self.layers[i], self.layers[i + 2]
        return self.s2ds and (K, R, st, C3, K3, R3, st3) == (2 * C, 3, 2, C, 2 * C, 1, 2) \
            and self.mode in ("po2", "po2+") and _lib.s2ds_supported(x.shape, self.bits, self.mode)

    def pair_call(self, i, x):
        return _lib.qconv2d_pair(x, self.weights[i], self.weights[i + 1], self.bits, self.mode)

    def _timed_pair(self, i, x, record):
        if record and i + 1 == self.timed_layer:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            y = self.pair_call(i, x)
            e1.record()
            self.events.append((e0, e1))
            return y
        return self.pair_call(i, x)

    def _timed(self, i, x, record):
        # HIP events around the timed layer itself (one per step: an event pair costs
        # ~10 us of queue time, so timing all 18 same-shape layers would slow the step)
        if record and i == self.timed_layer:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            y = self.conv(i, x)
            e1.record()
            self.events.append((e0, e1))
            return y
        return self.conv(i, x)


def conv_work(N, C, H, K, R, st, pad):
    P = (H + 2 * pad - R) // st + 1
    flops = 2.0 * N * K * P * P * C * R * R
    # fp32 in + out + weight read twice (absmax pass + conv) — BASELINE.md roofline table
    nbytes = 4.0 * (N * C * H * H + N * K * P * P + 2 * K * C * R * R)
    return flops, nbytes


def cpu_baseline(layers, weights_cpu, image, mode, bits, seconds, nb=2):
    """The reference's CPU path restated (oracle quantizer + torch CPU F.conv2d, the
    same oneDNN conv the reference calls) over a bounded sample of the workload: passes of
    `nb` images through the chain until `seconds` have elapsed."""
    from oracle import oracle as O

    threads = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        threads = min(threads, int(omp))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1)
    x0 = torch.relu(torch.randn(nb, 16, image, image, generator=g))

    def one_pass():
        x = x0
        i = 0
        while i < len(layers):
            has_ds = i + 2 < len(layers) and layers[i + 2][6] == "ds"
            outs = []
            for j in range(i, i + (3 if has_ds else 2)):
                _, C, K, R, st, pad, role = layers[j]
                inp = x if role != "conv2" else outs[-1]
                outs.append(O.cpu_reference_qconv2d(inp, weights_cpu[j], None, st, pad, 1, 1, bits, mode))
            x = outs[1]
            i += 3 if has_ds else 2
        return x

    one_pass()  # warm-up (oneDNN primitive creation)
    t0 = time.perf_counter()
    reps = 0
    while True:
        one_pass()
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    cpu_model = None
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name:"):
                cpu_model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return {"value": round(nb * reps / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model,
            "sample": "%d passes x %d images of the ResNet56 %dx%d quantized-conv chain (oracle quantizer "
                      "+ torch CPU F.conv2d/oneDNN, %d threads), %.1f s" % (reps, nb, image, image, threads, dt)}


def gather_logits(logits, gathered, world=None):
    """Output gather of the batch-sharded inference: rank r's logits land in rows
    [r*B, (r+1)*B) of `gathered` on every rank (RCCL all_gather over xGMI).  The collective runs
    whenever a process group exists and `gathered` was allocated for it (gather_buffer), a
    one-rank group included; without a group the logits are the output."""
    if gathered is not None:
        dist.all_gather_into_tensor(gathered, logits.contiguous())
        return gathered
    return logits


def gather_buffer(rows, classes, dev):
    """The all_gather target of gather_logits: [world * rows, classes] when a process group exists."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return torch.empty(dist.get_world_size() * rows, classes, device=dev)


def leg_steps(replay, floor, seconds, probe=20):
    """Timed steps of a graph-replayed config leg: at least `floor`, and enough for `seconds` of GPU work
    (estimated from `probe` untimed replays), so an outside sampler of GPU activity sees the leg."""
    replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(probe):
        replay()
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / probe
    return max(int(floor), int(math.ceil(seconds / max(per, 1e-6))))


def timed_steps(step, steps, warmup, world, sync, dev):
    """`warmup` untimed steps, then exactly `steps` timed ones bracketed by a barrier +
    device sync on both sides; returns the MAX wall time over ranks (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(record=True)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    return dt


def cifar_chain(args, world, rank, dev, gathered_classes=10, cpu=True):
    """Config 2 (BASELINE.json configs[1]): the ResNet56 quantized-conv chain at 32x32, bs=256 per
    GPU, po2 4-bit, replayed from a HIP graph (a layer is a few microseconds of GPU work here, less
    than the host's launch cost), measured in the same process as the headline.  Returns img/s,
    the roofline of the kernel with the largest share of the step (per distinct layer shape:
    count x average launch time from a graph of back-to-back launches) and its own CPU baseline."""
    B, Hs = 256, 32
    chain = QConvChain(9, gathered_classes, args.quantizer, args.bits, args.precision, dev, seed=0)
    x = torch.relu(torch.randn(B, 16, Hs, Hs, generator=torch.Generator().manual_seed(200 + rank))).to(dev)
    gathered = gather_buffer(B, gathered_classes, dev)
    pack_batch = args.quantizer in ("po2", "po2+") and args.precision != "fp32"
    with torch.no_grad():
        for _ in range(2):  # autotune every shape + warm the caching allocator
            chain.forward(x)
        torch.cuda.synchronize()
        if pack_batch:
            chain.enable_packed()
            chain.forward(x)
            torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain.forward(x)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            logits = chain.forward(x)
        gstep = lambda record=False: gather_logits(graph.replay() or logits, gathered, world)  # noqa: E731
        steps = leg_steps(gstep, args.cifar_steps, args.leg_seconds)
        if world > 1:  # every rank times the same number of steps
            t = torch.tensor([steps], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            steps = int(t.item())
        dt = timed_steps(gstep, steps, 5, world, torch.cuda.synchronize, dev)

        def launch_ms(fn):  # average of 20 back-to-back launches captured in a graph, 5 replays
            fn()
            torch.cuda.synchronize()
            lg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(lg):
                for _ in range(20):
                    fn()
            lg.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lg.replay()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 100

        # per distinct single-conv shape: count x average launch; per chain launch: its time
        inputs = {}
        for i, shp in chain.shapes.items():
            _, C, K, R, st, pad, _ = chain.layers[i]
            inputs.setdefault((C, K, R, st, pad, shp), []).append(i)
        cands = []
        for key, idx in inputs.items():
            C, K, R, st, pad, shp = key
            xi = torch.relu(torch.randn(shp, device=dev))
            ms = launch_ms(lambda: chain.conv(idx[0], xi, direct=True))  # noqa: B023
            flops, nbytes = conv_work(shp[0], C, shp[2], K, R, st, pad)
            plan = _lib.describe(shp[0], C, shp[2], shp[3], K, R, R, st, pad, 1, 1, args.bits,
                                 None if args.quantizer == "none" else args.quantizer, 1, args.precision)
            achieved = nbytes / (ms * 1e-3) / 1e9
            cands.append((ms * len(idx), {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                "kernel": "fused %s quantize+conv %dx%d s%d %d->%d @%dx%d bs=%d (%d layers of this shape): %s"
                          % (args.quantizer, R, R, st, C, K, shp[2], shp[3], shp[0], len(idx), plan),
                "avg_launch_ms": round(ms, 5), "algorithmic_bytes": int(nbytes), "flops": int(flops),
                "note": "a layer's 8-34 MB fit the 256 MB Infinity Cache between launches; at ~10-20 us per "
                        "launch the step is latency-bound, so the HBM fraction is low by construction"}))
        for first, (run, shp) in chain.chains.items():
            xi = torch.relu(torch.randn(shp, device=dev))
            ms = launch_ms(lambda: chain.run_chain(run, xi))  # noqa: B023
            flops = sum(conv_work(shp[0], shp[1], shp[2], shp[1], 3, 1, 1)[0] for _ in run)
            nbytes = 4.0 * 2 * shp[0] * shp[1] * shp[2] * shp[3] + sum(8.0 * chain.weights[j].numel() for j in run)
            tf = flops / (ms * 1e-3) / 1e12
            cands.append((ms, {
                "bound": "mfma", "achieved": round(tf, 2), "peak": round(PEAK_BF16_MFMA_TFLOPS / 3, 1),
                "unit": "TFLOP/s", "frac": round(tf / (PEAK_BF16_MFMA_TFLOPS / 3), 4), "traffic": None,
                "kernel": "conv_chain<%d> (po2q_qconv2d_chain_f32): %d fused %s quantize+conv 3x3 s1 %d->%d @%dx%d "
                          "bs=%d in one launch, one block per image" % (shp[1], len(run), args.quantizer, shp[1],
                                                                         shp[1], shp[2], shp[3], shp[0]),
                "avg_launch_ms": round(ms, 5), "algorithmic_bytes": int(nbytes), "flops": int(flops),
                "note": "fp32 FLOPs on the bf16x3-effective dense MFMA peak (2516.6 / 3 TFLOP/s: three bf16 "
                        "MFMAs per exact fp32 product); x in + y out + weights read twice as the bytes, the "
                        "per-layer activations stay L2-resident inside the launch"}))
        cands.sort(key=lambda c: -c[0])
        roofline = cands[0][1]
    images = world * B * steps
    out = {"workload": "resnet56 quantized-conv chain @32x32 bs=%d per GPU: 56 fused %s-%dbit quantize+conv fwd "
                       "+ head, HIP graph replay%s" % (B, args.quantizer, args.bits,
                                                       " (each stage's stride-1 run of convs as one chain launch)"
                                                       if chain.chains else ""),
           "metric": "quantized-conv fwd images/sec, ResNet56 32x32 bs=256", "value": round(images / dt, 2),
           "unit": "images/s", "n_gpus": world, "steps": steps, "ms_per_step": round(dt * 1e3 / steps, 4),
           "timed_seconds": round(dt, 3),
           "roofline": roofline, "cpu_baseline": None}
    if cpu:
        wcpu = [w.cpu() for w in chain.weights]
        out["cpu_baseline"] = cpu_baseline(chain.layers, wcpu, Hs, args.quantizer, args.bits,
                                           min(args.cpu_seconds, 10.0), nb=32)
    return out


def model_extra(args, world, rank, dev, model_type, quantizer, bits, image, batch, classes, steps, cpu, label):
    """A BASELINE.json model config measured beside the headline: the reference's model graph
    (drop-in modules, random init, eval, fused native forward) replayed from a HIP graph, bs
    `batch` per GPU, synthetic input.  The roofline is the dominant quantized conv's: every
    distinct qconv call of one forward is re-timed alone (graph of 20 back-to-back launches,
    plain conv without its epilogue) and the shape with the largest count x time is reported.
    The CPU baseline runs the same graph on the host with the oracle quantizer + torch CPU convs
    (the reference's own CPU arithmetic) over a bounded sample."""
    from po2_quantization_amd.models import quantized_conv
    from po2_quantization_amd.models.model import get_model
    from po2_quantization_amd.utils.quantizers import quantizer_dict

    torch.manual_seed(0)
    m = get_model(model_type, classes, quantizer_dict[quantizer], bits, (image, image)).eval()
    m_dev = get_model(model_type, classes, quantizer_dict[quantizer], bits, (image, image))
    m_dev.load_state_dict(m.state_dict())
    m_dev = m_dev.to(dev).eval()
    x = torch.randn(batch, 3, image, image, generator=torch.Generator().manual_seed(300 + rank)).to(dev)
    calls = {}
    real = _lib.qconv2d_fused

    def rec(xx, w, bias=None, stride=1, padding=0, dilation=1, groups=1, bits_=4, mode="po2", *a, **k):
        key = (tuple(xx.shape), tuple(w.shape), _lib._pair(stride), _lib._pair(padding), _lib._pair(dilation),
               int(groups), mode)
        calls.setdefault(key, [0, w])[0] += 1
        return real(xx, w, bias, stride, padding, dilation, groups, bits_, mode, *a, **k)

    with torch.no_grad():
        _lib.qconv2d_fused = rec
        try:
            m_dev(x)  # autotunes every conv shape; records the qconv calls
        finally:
            _lib.qconv2d_fused = real
        torch.cuda.synchronize()
        m_dev(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m_dev(x)
        torch.cuda.current_stream().wait_stream(s)
        try:
            graph = torch.cuda.CUDAGraph(keep_graph=True)  # keeps the raw graph for graph_launches
        except TypeError:
            graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            logits = m_dev(x)
        if getattr(graph, "instantiate", None) is not None:
            try:
                graph.instantiate()
            except Exception:  # noqa: BLE001 -- already instantiated
                pass
        gathered = gather_buffer(batch, classes, dev)
        gstep = lambda record=False: gather_logits(graph.replay() or logits, gathered, world)  # noqa: E731
        steps = leg_steps(gstep, steps, args.leg_seconds)
        if world > 1:  # every rank times the same number of steps
            t = torch.tensor([steps], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            steps = int(t.item())
        dt = timed_steps(gstep, steps, 5, world, torch.cuda.synchronize, dev)
        best = None
        for key, (cnt, w) in calls.items():
            xs, ws, st, pad, dil, grp, mode = key
            if mode == "none":
                continue
            xi = torch.relu(torch.randn(xs, device=dev))
            fn = lambda: _lib.qconv2d(xi, w, None, st, pad, dil, grp, bits, mode)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            lg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(lg):
                for _ in range(20):
                    fn()
            lg.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lg.replay()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 100
            if best is None or ms * cnt > best[0] * best[1]:
                best = (ms, cnt, key)
    ms, cnt, (xs, ws, st, pad, dil, grp, mode) = best
    N, C, H, W = xs
    K, Cg, R, S = ws
    P = (H + 2 * pad[0] - dil[0] * (R - 1) - 1) // st[0] + 1
    Q = (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // st[1] + 1
    nbytes = 4.0 * (N * C * H * W + N * K * P * Q + 2 * K * Cg * R * S)
    flops = 2.0 * N * K * P * Q * Cg * R * S
    achieved = nbytes / (ms * 1e-3) / 1e9
    plan = _lib.describe(N, C, H, W, K, R, S, st, pad, dil, grp, bits, mode)
    # step level: the algorithmic bytes of every conv call of the forward (fp32 x in + y out + the
    # weight read once; BN / activation / residual are fused into those) over the measured step
    step_bytes, step_flops = 0.0, 0.0
    for (xs_, ws_, st_, pad_, dil_, grp_, _), (cnt_, _) in calls.items():
        n_, c_, h_, w_ = xs_
        k_, cg_, r_, s_ = ws_
        p_ = (h_ + 2 * pad_[0] - dil_[0] * (r_ - 1) - 1) // st_[0] + 1
        q_ = (w_ + 2 * pad_[1] - dil_[1] * (s_ - 1) - 1) // st_[1] + 1
        step_bytes += cnt_ * 4.0 * (n_ * c_ * h_ * w_ + n_ * k_ * p_ * q_ + k_ * cg_ * r_ * s_)
        step_flops += cnt_ * 2.0 * n_ * k_ * p_ * q_ * cg_ * r_ * s_
    step_ms = dt * 1e3 / steps
    step_achieved = step_bytes / (step_ms * 1e-3) / 1e9
    images = world * batch * steps
    out = {"workload": "%s @%dx%d bs=%d per GPU, %s %d-bit QAT-mode weights, fused eval forward (every conv + BN + "
                       "act + residual native), HIP graph replay" % (model_type, image, image, batch, quantizer, bits),
           "metric": "%s fwd images/sec, %s %dx%d bs=%d" % (label, model_type, image, image, batch),
           "value": round(images / dt, 2), "unit": "images/s", "n_gpus": world, "steps": steps,
           "ms_per_step": round(step_ms, 4), "timed_seconds": round(dt, 3),
           "roofline": {"scope": "step", "bound": "hbm", "achieved": round(step_achieved, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(step_achieved / PEAK_HBM_GBS, 4), "traffic": None,
                        "algorithmic_bytes_per_step": int(step_bytes), "flops_per_step": int(step_flops),
                        "conv_calls_per_step": int(sum(c for c, _ in calls.values())),
                        "launches_per_step": graph_launches(graph),
                        "note": "the whole forward: every conv call's algorithmic bytes (x in + y out + weight) "
                                "over ms_per_step; at this size the step is bound by launch latency (a few us of "
                                "work per kernel), not by HBM or the matrix cores",
                        "dominant_kernel": {
                            "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": round(achieved / PEAK_HBM_GBS, 4),
                            "kernel": "fused %s quantize+conv %dx%d s%d g%d %d->%d @%dx%d bs=%d (%d calls per "
                                      "forward): %s" % (mode, R, S, st[0], grp, C, K, H, W, N, cnt, plan),
                            "avg_launch_ms": round(ms, 5), "algorithmic_bytes": int(nbytes), "flops": int(flops)}},
           "cpu_baseline": None}
    if cpu:
        out["cpu_baseline"] = model_cpu_baseline(m, image, min(args.cpu_seconds, 10.0), label)
    return out


def graph_launches(graph):
    """Kernel nodes of a captured HIP graph (hipGraphGetNodes on torch's raw graph handle), or None
    where this torch build does not expose the handle."""
    try:
        import ctypes
        h = graph.raw_cuda_graph()
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_size_t(0)
        if hip.hipGraphGetNodes(ctypes.c_void_p(h), None, ctypes.byref(n)) != 0:
            return None
        nodes = (ctypes.c_void_p * n.value)()
        if hip.hipGraphGetNodes(ctypes.c_void_p(h), nodes, ctypes.byref(n)) != 0:
            return None
        kinds = ctypes.c_int(0)
        kernels = 0
        for nd in nodes:
            if hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(kinds)) == 0 and kinds.value == 0:
                kernels += 1  # hipGraphNodeTypeKernel
        return kernels
    except Exception:  # noqa: BLE001 -- diagnostic only
        return None


def model_cpu_baseline(m, image, seconds, label):
    """The reference's CPU path for a model config: the same module graph on the host, eval, with
    the oracle quantizer (bit-exact restatement) + torch CPU F.conv2d (oneDNN) standing in for
    the native calls -- only inside this bounded timing leg."""
    from oracle import oracle as O
    from po2_quantization_amd.models import quantized_conv

    threads = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        threads = min(threads, int(omp))
    torch.set_num_threads(threads)
    F = torch.nn.functional

    def q(w, bits, mode, fsr=1):
        return torch.from_numpy(O.quantize(w.detach().numpy(), bits, mode, fsr))

    def conv(x, w, bias=None, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1, precision="auto",
             plan=None):
        return F.conv2d(x, w if mode == "none" else q(w, bits, mode, fsr), bias, stride, padding, dilation, groups)

    saved = (_lib.quantize, _lib.qconv2d, quantized_conv.INFERENCE_FUSION)
    _lib.quantize, _lib.qconv2d, quantized_conv.INFERENCE_FUSION = q, conv, False
    nb = 64 if image <= 64 else 4  # enough images per pass that the per-forward weight quantize amortizes as at bs=256
    x = torch.randn(nb, 3, image, image, generator=torch.Generator().manual_seed(1))
    try:
        with torch.no_grad():
            m(x)
            t0, reps = time.perf_counter(), 0
            while True:
                m(x)
                reps += 1
                if time.perf_counter() - t0 >= seconds:
                    break
            dt = time.perf_counter() - t0
    finally:
        _lib.quantize, _lib.qconv2d, quantized_conv.INFERENCE_FUSION = saved
    return {"value": round(nb * reps / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "%d passes x %d images of the %s graph at %dx%d on the host (oracle quantizer + torch CPU "
                      "conv / BN / act, %d threads), %.1f s" % (reps, nb, label, image, image, threads, dt)}


def launch_ranks(n, argv):
    """Start the N ranks of `bench.py argv` as one torch.distributed.run child process (one process
    per GPU, rendezvous on 127.0.0.1) and return its exit status.  Called before any GPU call: this
    parent only waits (no exec from a process that initialised the GPU)."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the box's driver supports dmabuf IPC only
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


def selftest(args, world, rank, backend):
    """--selftest: the N-rank step on the CPU over gloo, no kernels.  The global batch
    (--global-batch, default 4 images per rank) is split evenly; every rank runs its contiguous shard
    through the drop-in model's CPU path (ResNet20, po2 4-bit QAT-mode QuantizedConv2d layers: the
    reference's torch arithmetic, bs / world images per rank, --image pixels), the logits are
    all-gathered (gather_logits, the bench's collective) and the step is timed as timed_steps does
    (barrier-bracketed, max over ranks).  Rank 0 checks the gathered logits against one unsharded
    forward of the whole batch and prints one JSON line (tests/test_distributed.py runs it through the
    --gpus 2 entry)."""
    from po2_quantization_amd.models.model import get_model
    from po2_quantization_amd.utils.quantizers import quantizer_dict

    torch.set_num_threads(1)
    total = args.global_batch if args.global_batch is not None else 4 * world
    if total % world:
        raise SystemExit("--global-batch %d is not divisible by the %d ranks" % (total, world))
    B, classes, dev = total // world, 10, torch.device("cpu")
    torch.manual_seed(0)  # identical weights on every rank, as the bench's seeded weights
    m = get_model("resnet20", classes, quantizer_dict["po2"], 4, (args.image, args.image)).eval()
    x_all = torch.randn(total, 3, args.image, args.image, generator=torch.Generator().manual_seed(1))
    x = x_all[rank * B:(rank + 1) * B]
    gathered = gather_buffer(B, classes, dev)

    def step(record=False):
        with torch.no_grad():
            return gather_logits(m(x), gathered)

    dt = timed_steps(step, args.steps, args.warmup, world, lambda: None, dev)
    out = step()
    if rank == 0:
        with torch.no_grad():
            full = m(x_all)
        err = float((out - full).abs().max() / full.abs().max())
        print(json.dumps({"selftest": True, "n_gpus": world, "world_size": world, "dist_backend": backend,
                          "global_batch": total, "batch_per_rank": B, "gathered_rows": int(out.shape[0]),
                          "gathered_err": err, "gathered_ok": err <= 1e-5, "steps": args.steps, "seconds": dt}),
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~1.1 s timed at 224: long enough for an external sampler
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="images per step over all GPUs (split evenly; overrides --batch)")
    ap.add_argument("--graph", action="store_true", help="replay the step from a HIP graph")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--model", default="resnet56", choices=["resnet20", "resnet32", "resnet44", "resnet56"])
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--quantizer", default="po2", choices=["po2", "po2+", "none"])
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--precision", default="auto", choices=["auto", "fp32", "bf16x3"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pair", action="store_true",
                    help="run every conv as its own launch (no conv1->conv2 pair kernel in stages 1-2)")
    ap.add_argument("--no-s2ds", action="store_true",
                    help="run a stage's stride-2 conv1 and its 1x1 shortcut as two launches (each reads x)")
    ap.add_argument("--no-pack-batch", action="store_true",
                    help="quantize + pack each single-conv layer's weight in its own launch")
    ap.add_argument("--no-autotune", action="store_true",
                    help="use the heuristic plans instead of autotuning each conv shape on first use")
    ap.add_argument("--no-cifar", dest="cifar", action="store_false",
                    help="skip the config-2 line (ResNet56 @32x32 bs=256 chain from a HIP graph, "
                         "reported under config2_cifar32 next to the headline)")
    ap.add_argument("--cifar-steps", type=int, default=200, help="minimum timed steps of the config-2 leg")
    ap.add_argument("--leg-seconds", type=float, default=5.0,
                    help="the config-2/3/5 legs time at least this many seconds of GPU work (their step count "
                         "grows to fit); the headline keeps exactly --steps")
    ap.add_argument("--no-models", dest="models", action="store_false",
                    help="skip the model-config lines (config 3: MobileNetV2 @32 po2+ 4-bit; config 5: MobileViT-XS "
                         "@256 po2+ 2-bit), reported under config3_mobilenet32 / config5_mobilevit256")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI on ROCm)")
    ap.add_argument("--selftest", action="store_true",
                    help="N-rank plumbing only (gloo, CPU stand-in logits, no kernels): launcher, gather, timing")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the N ranks (nothing has touched the GPU in this process)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.selftest:
        args.backend = "gloo"
    # the reference runs with torch.backends.cudnn.benchmark = True (train.py:33, test.py:31);
    # the po2q counterpart times every candidate plan on a shape's first call (an untimed warmup step)
    _lib.benchmark = not args.no_autotune

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        # what the process group itself reports (the env only says what torchrun asked for)
        world, rank, backend = dist.get_world_size(), dist.get_rank(), str(dist.get_backend())
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the process group holds %d ranks" % (args.gpus, world))
    if args.selftest:
        selftest(args, world, rank, backend)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.global_batch is not None:
        if args.global_batch % world:
            raise SystemExit("--global-batch %d is not divisible by the %d ranks" % (args.global_batch, world))
        args.batch = args.global_batch // world
    n_blocks = {"resnet20": 3, "resnet32": 5, "resnet44": 7, "resnet56": 9}[args.model]
    chain = QConvChain(n_blocks, args.classes, args.quantizer, args.bits, args.precision, dev, seed=0)
    chain.timed_layer = 1  # layer1.0.conv2: 3x3 16->16 at full resolution (dominant shape)
    chain.pair = not args.no_pair
    chain.s2ds = not args.no_s2ds
    B, Hs = args.batch, args.image
    x = torch.relu(torch.randn(B, 16, Hs, Hs, generator=torch.Generator().manual_seed(100 + rank))).to(dev)
    gathered = gather_buffer(B, args.classes, dev)

    def step(record=False):
        return gather_logits(chain.forward(x, record), gathered, world)

    pack_batch = not args.no_pack_batch and args.quantizer in ("po2", "po2+") and args.precision != "fp32"
    if pack_batch:
        with torch.no_grad():  # one untimed forward: autotunes every shape and records the layers' inputs
            step()
            torch.cuda.synchronize()
        chain.enable_packed()

    graph = None
    if args.graph:
        with torch.no_grad():
            for _ in range(max(args.warmup, 1)):  # autotune + warm the caching allocator
                step()
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                chain.forward(x)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                logits = chain.forward(x)
        gstep = lambda record=False: gather_logits(graph.replay() or logits, gathered, world)  # noqa: E731

    with torch.no_grad():
        # autotuning needs one untimed pass
        dt = timed_steps(gstep if graph is not None else step, args.steps,
                         max(args.warmup, 1 if _lib.benchmark else 0), world, torch.cuda.synchronize, dev)

    # dominant op (HIP events on its stream): the stage-1 conv pair (conv1 -> conv2 of a block
    # in one launch) when the chain runs pairs, else the fused quantize+conv of the timed shape
    pair_used = chain.pairable(0, x)
    pair32_used = chain.pair and args.quantizer in ("po2", "po2+") and \
        _lib.pair_supported((B, 32, Hs // 2, Hs // 2), args.bits, args.quantizer)
    s2ds_used = chain.s2ds and args.quantizer in ("po2", "po2+") and \
        _lib.s2ds_supported((B, 16, Hs, Hs), args.bits, args.quantizer)
    xl = torch.relu(torch.randn(args.batch, 16, args.image, args.image, device=dev))

    def launch_avg_ms(fn, reps=20):
        """Average duration of `fn` from back-to-back launches: a HIP graph of `reps` launches
        replayed 5 times (--graph), else `reps` launches bracketed by events."""
        with torch.no_grad():
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if graph is not None:
                lg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(lg):
                    for _ in range(reps):
                        fn()
                lg.replay()
                e0.record()
                for _ in range(5):
                    lg.replay()
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / (5 * reps)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps

    if graph is not None:
        avg_ms = launch_avg_ms((lambda: chain.pair_call(0, xl)) if pair_used else
                               (lambda: chain.conv(chain.timed_layer, xl, direct=True)))
    else:
        ev_ms = [a.elapsed_time(b) for a, b in chain.events]
        avg_ms = sum(ev_ms) / max(len(ev_ms), 1)
    _, C, K, R, st, pad, _ = chain.layers[chain.timed_layer]
    flops, nbytes = conv_work(B, C, Hs, K, R, st, pad)
    # the conv arithmetic the library actually planned for this layer (AUTO picks
    # bf16x3 for power-of-two weights): three exact bf16 MFMA passes per fp32 product
    plan = _lib.describe(B, C, Hs, Hs, K, R, R, st, pad, 1, 1, args.bits,
                         None if args.quantizer == "none" else args.quantizer, 1, args.precision)
    prec = "bf16x3" if "kind=bf16x3" in plan else "fp32"
    peak_c = PEAK_BF16_MFMA_TFLOPS / 3.0 if prec == "bf16x3" else PEAK_FP32_MFMA_TFLOPS

    def roofline(fl, nb, ms):
        if fl / nb * PEAK_HBM_GBS / 1e3 < peak_c:  # TFLOP/s attainable from HBM below the MFMA peak
            achieved = nb / (ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 4)}
        achieved = fl / (ms * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak_c, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak_c, 4)}

    def traffic_of(key):
        traffic_file = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(traffic_file):
            try:
                tr = json.load(open(traffic_file)).get(key)
                return tr.get("hbm_bytes_per_launch") if tr else None
            except (ValueError, OSError):
                return None
        return None

    layer_kernel = ("fused %s quantize+conv %dx%d %d->%d @%dx%d bs=%d: %s"
                    % (args.quantizer, R, R, C, K, Hs, Hs, B, plan))
    if pair_used:
        # x in + y out + both weights read twice (absmax + staging); 2 convs of flops
        pflops, pbytes = 2 * flops, 4.0 * (2 * B * 16 * Hs * Hs + 4 * 16 * 16 * 9)
        roof = roofline(pflops, pbytes, avg_ms)
        roof["traffic"] = traffic_of("pair16 %dx%d bs=%d" % (Hs, Hs, B))
        roof.update({"kernel": "conv_pair_rs16 (po2q_qconv2d_pair_f32, role-split pair): conv1 -> conv2, 2 fused %s quantize+"
                               "conv 3x3 16->16 @%dx%d bs=%d in one launch, intermediate on chip"
                               % (args.quantizer, Hs, Hs, B),
                     "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes": int(pbytes), "flops": int(pflops)})
        # the single-layer kernel of the same shape (used wherever pairs do not apply)
        lms = launch_avg_ms(lambda: chain.conv(chain.timed_layer, xl, direct=True))
        layer_roof = roofline(flops, nbytes, lms)
        layer_roof["traffic"] = traffic_of(plan)
        layer_roof.update({"kernel": layer_kernel, "avg_launch_ms": round(lms, 4), "algorithmic_bytes": int(nbytes),
                           "flops": int(flops)})
    else:
        roof = roofline(flops, nbytes, avg_ms)
        roof["traffic"] = traffic_of(plan)
        roof.update({"kernel": layer_kernel, "avg_launch_ms": round(avg_ms, 4), "algorithmic_bytes": int(nbytes),
                     "flops": int(flops)})
        layer_roof = None

    images = world * B * args.steps
    out = {
        "metric": METRIC, "value": round(images / dt, 2), "unit": "images/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if prec == "fp32" else "fp32(bf16x3)", "data": "synthetic",
        "config": {"workload": "%s quantized-conv chain: %d fused %s-%dbit quantize+conv fwd + head%s%s%s%s"
                               % (args.model, len(chain.layers), args.quantizer, args.bits,
                                  (" (stage-1%s conv1->conv2 pairs as one launch each)"
                                   % (" and stage-2" if pair32_used else "")) if pair_used else "",
                                  " (stride-2 conv1 + 1x1 shortcut of stages 2-3 as one launch each)"
                                  if s2ds_used else "",
                                  " (weight packs of the single-conv layers batched: one launch per 36)"
                                  if chain.packed is not None else "",
                                  " + RCCL all_gather(logits)" if world > 1 else ""),
                   "conv_pairs": pair_used,
                   "conv_pairs_stage2": pair32_used,
                   "s2ds": s2ds_used,
                   "pack_batch": chain.packed is not None,
                   "autotune": _lib.benchmark,
                   "image": Hs, "batch_per_gpu": B, "global_batch": world * B, "quantizer": args.quantizer,
                   "bits": args.bits, "precision": prec, "parallelism": "dp%d" % world, "world_size": world,
                   "dist_backend": backend, "hip_graph": graph is not None},
        "roofline": roof,
        "layer_roofline": layer_roof,
        "cpu_baseline": None,
    }
    # the CPU baselines run on rank 0 at N = 1 only: at N > 1 the other ranks would poll the next
    # barrier beside it and skew the number
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu_baseline
    if cpu_leg:
        wcpu = [w.cpu() for w in chain.weights]
        out["cpu_baseline"] = cpu_baseline(chain.layers, wcpu, Hs, args.quantizer, args.bits, args.cpu_seconds)
    if args.cifar and Hs != 32:
        del chain, x, xl
        torch.cuda.empty_cache()
        out["config2_cifar32"] = cifar_chain(args, world, rank, dev, gathered_classes=10, cpu=cpu_leg)
    if args.models and Hs != 32:
        torch.cuda.empty_cache()
        out["config3_mobilenet32"] = model_extra(args, world, rank, dev, "mobilenet", "po2+", 4, 32, 256, 10, 200,
                                                 cpu_leg, "MobileNetV2 (config 3)")
        torch.cuda.empty_cache()
        out["config5_mobilevit256"] = model_extra(args, world, rank, dev, "mobilevit", "po2+", 2, 256, 64, 1000, 50,
                                                  cpu_leg, "MobileViT-XS (config 5)")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
