"""Quantization-aware training on the drop-in modules: the
reference's train.py loop, one process per GPU, DistributedDataParallel over RCCL.

  init(seed)                      train.py:25-34   process group ("nccl" = RCCL) + seeds
  build_model(...)                train.py:128-168 get_model, BatchNorm -> SyncBatchNorm when
                                                   distributed (the reference's models are
                                                   built with nn.SyncBatchNorm), DDP wrap,
                                                   QAT starts from full_precision.pth
  make_optimizer(...)             train.py:50-67   SGD(momentum 0.9, wd 1e-4), lr x world size,
                                                   LambdaLR warmup, MultiStepLR at 82 / 123
  train_step(...)                 train.py:79-94   forward (fused native quantize + conv), CE
                                                   loss, backward (STE + conv grads; DDP
                                                   all-reduces the gradient buckets), SGD step
  GraphedTrainStep                train.py:79-94   the same step captured once in a HIP graph and
                                                   replayed: ~1000 host launches per step become
                                                   one graph launch; under a process group the
                                                   DDP semantics (rank-0 buffer broadcast, averaged
                                                   gradients) are captured with it as coalesced
                                                   collectives (GradSync: one RCCL broadcast + one
                                                   all_reduce per dtype)
  run_train_loop(...)             train.py:37-125  epochs, per-epoch all_reduce of loss/samples,
                                                   quantization error, rows for the CSV
  write_train_csv(path, rows)     train.py:255-259 header epoch,train_loss,train_acc,quantization_error

The forward runs po2q's fused quantize + conv; the backward is the reference's autograd
(straight-through estimator for the quantizer, quantizers.py:34-36; torch's conv input /
weight gradients of the quantized weight), see models/quantized_conv.py _QConv2dFn.  The
data loader is the only departure: torchvision / CIFAR are unavailable offline, so the
training set is a tensor pair, sharded per epoch like DistributedSampler (shuffle with
seed + epoch, pad to a multiple of the world size, rank r takes every world-th index).
"""
import csv
import os
import random
from pathlib import Path
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim
from torch.nn.parallel import DistributedDataParallel
from torch.optim.lr_scheduler import LambdaLR, MultiStepLR

from .models.model import get_model

Row = Tuple[int, float, float, float]


def init(seed: int, backend: str = "nccl") -> None:
    """train.py:25-34 (backend "nccl" is RCCL on ROCm)."""
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = False
    torch.backends.cudnn.benchmark = True


def _world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def build_model(model_type: str, num_classes: int, quantize_fn: Optional[Callable], bits: int, image_size,
                device, full_precision_model_path: Optional[str] = None, sync_bn: bool = True,
                ddp: bool = True) -> nn.Module:
    """train.py:128-168: the model on `device`, DDP-wrapped when a process group exists
    (sync_bn=False keeps per-rank BatchNorm statistics, e.g. for a gloo test group).
    ddp=False under a process group: the plain module with DDP's construction step done here (rank 0's
    parameters and buffers broadcast), for GraphedTrainStep, which captures DDP's per-step collectives
    itself (GradSync) -- DDP's reducer hooks cannot be captured in a HIP graph (the capture segfaults)."""
    model = get_model(model_type=model_type, num_classes=num_classes, quantize_fn=quantize_fn, bits=bits,
                      image_size=image_size)
    _, world = _world()
    grouped = dist.is_available() and dist.is_initialized()
    if world > 1 and sync_bn:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)  # same state_dict keys
    model = model.to(device)
    if grouped and ddp:  # the reference wraps under any process group, a one-rank torchrun included
        idx = device.index if isinstance(device, torch.device) else None
        model = DistributedDataParallel(model, device_ids=[idx] if idx is not None else None,
                                        output_device=idx)
    elif grouped:
        GradSync(model).broadcast_state()
    if quantize_fn is not None and full_precision_model_path is not None:
        assert os.path.exists(full_precision_model_path), "QAT requires full precision model"
        sd = torch.load(full_precision_model_path, map_location="cpu", weights_only=True)
        if grouped and ddp:  # the reference loads the DDP state dict ("module." keys) into the DDP model
            sd = {(k if k.startswith("module.") else "module." + k): v for k, v in sd.items()}
        else:
            sd = {k.replace("module.", ""): v for k, v in sd.items()}
        model.load_state_dict(sd)
    return model


def make_optimizer(model: nn.Module, lr: float, num_epochs: int, momentum: float = 0.9,
                   weight_decay: float = 1e-4, percent_warmup_epochs: float = 0.1):
    """train.py:50-67: (optimizer, warmup scheduler, multistep scheduler, warmup epochs)."""
    _, world = _world()
    lr *= world  # scale for the larger effective batch
    warmup_epochs = int(percent_warmup_epochs * num_epochs)
    optimizer = optim.SGD(model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)
    warmup = LambdaLR(optimizer, lr_lambda=lambda epoch: (epoch + 1) / (warmup_epochs + 1))
    multistep = MultiStepLR(optimizer, milestones=[82 - warmup_epochs, 123 - warmup_epochs], gamma=0.1)
    return optimizer, warmup, multistep, warmup_epochs


class GradSync:
    """What DistributedDataParallel adds to a training step (train.py:153-155; DDP defaults), as plain
    collectives that a HIP graph can capture: before the forward, rank 0's buffers (BatchNorm statistics)
    are broadcast (broadcast_buffers=True); after the backward, every gradient is summed over the ranks
    and divided by the world size.  Both are coalesced -- one flat tensor per dtype, so one RCCL
    broadcast and one all_reduce per dtype per step instead of DDP's per-bucket calls from autograd
    hooks, which are not capturable.  Division by a power-of-two world size is exact, so the averaged
    gradient is DDP's (a/w + b/w == (a + b)/w)."""

    def __init__(self, module: nn.Module, group=None):
        self.module, self.group = module, group
        self.world = dist.get_world_size(group)

    @staticmethod
    def _by_dtype(ts):
        out = {}
        for t in ts:
            out.setdefault(t.dtype, []).append(t)
        return out.values()

    def broadcast_state(self):
        """DDP's construction step: rank 0's parameters and buffers on every rank."""
        self._broadcast(list(self.module.parameters()) + list(self.module.buffers()))

    def broadcast_buffers(self):
        self._broadcast(list(self.module.buffers()))

    def _broadcast(self, tensors):
        with torch.no_grad():
            for ts in self._by_dtype([t.detach() for t in tensors]):
                flat = torch.cat([t.reshape(-1) for t in ts])
                dist.broadcast(flat, 0, group=self.group)
                off = 0
                for t in ts:
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()

    def reduce_grads(self):
        with torch.no_grad():
            for gs in self._by_dtype([p.grad for p in self.module.parameters() if p.grad is not None]):
                flat = torch.cat([g.reshape(-1) for g in gs])
                dist.all_reduce(flat, group=self.group)
                flat.div_(self.world)
                off = 0
                for g in gs:
                    g.copy_(flat[off:off + g.numel()].view_as(g))
                    off += g.numel()


def train_step(model: nn.Module, optimizer, criterion, images: torch.Tensor, labels: torch.Tensor,
               sync: Optional[GradSync] = None):
    """One iteration (train.py:79-94); returns (loss * batch, correct) as device tensors
    (no host synchronisation inside the step).  sync: DDP's buffer broadcast + gradient average as
    explicit collectives (GraphedTrainStep on an unwrapped module under a process group)."""
    optimizer.zero_grad()
    if sync is not None:
        sync.broadcast_buffers()
    outputs = model(images)
    loss = criterion(outputs, labels)
    with torch.no_grad():
        correct = (outputs.argmax(1) == labels).sum()
    loss.backward()
    if sync is not None:
        sync.reduce_grads()
    optimizer.step()
    return loss.detach() * images.size(0), correct


class GraphedTrainStep:
    """train_step (train.py:79-94) captured in a HIP graph and replayed: forward (the fused native
    quantize + conv kernels), cross-entropy, the native backward and the SGD update as one graph
    launch.  At CIFAR size the eager step is bound by ~1000 host-side launches (BatchNorm, autograd,
    the optimizer), not by the convs; the replay issues none of them from the host.

    Same arithmetic as the eager step (the same kernels on the same tensors).  The batch is copied
    into static input buffers; step() returns (loss * batch, correct) as device tensors like
    train_step.  The learning rate is a Python float inside the SGD update, so the step is
    re-captured when a scheduler changes it (once per epoch).  The po2q autotuner runs in the eager
    warm-up steps, before capture (it synchronises the stream).

    Under a process group the step takes the plain module (qat.build_model(..., ddp=False)) and runs
    DDP's per-step semantics itself with GradSync: the rank-0 buffer broadcast and the gradient average
    as coalesced RCCL collectives captured inside the graph (tests/test_gpu_rccl.py).  A DDP-wrapped
    model is refused: DDP's reducer runs from autograd hooks on the parameters, and capturing them
    segfaults.  A model with SyncBatchNorm layers in training mode at world > 1 also issues their
    statistics collectives inside the graph."""

    def __init__(self, model: nn.Module, optimizer, criterion, images: torch.Tensor, labels: torch.Tensor,
                 warmup: int = 3):
        if isinstance(model, DistributedDataParallel):
            raise RuntimeError("GraphedTrainStep: pass the plain module (qat.build_model(..., ddp=False)); "
                               "DDP's autograd-hook reducer cannot be captured in a HIP graph")
        self.sync = GradSync(model) if dist.is_available() and dist.is_initialized() else None
        self.model, self.optimizer, self.criterion = model, optimizer, criterion
        self.x = images.clone()
        self.y = labels.clone()
        self.warmup = warmup
        self.graph = None
        self._lr = None

    def _lrs(self):
        return tuple(float(g["lr"]) for g in self.optimizer.param_groups)

    def _state(self):
        """Every tensor a step mutates: parameters, buffers (BatchNorm statistics and counters) and the
        optimizer's momentum buffers."""
        ts = list(self.model.state_dict(keep_vars=True).values())
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                buf = self.optimizer.state.get(p, {}).get("momentum_buffer")
                if buf is not None:
                    ts.append(buf)
        return [t.detach() if isinstance(t, torch.Tensor) else t for t in ts]

    def _capture(self):
        if self.graph is None:
            # eager warm-up on a side stream (po2q autotuning, lazy allocations, the optimizer's
            # momentum buffers), then every mutated tensor restored: the warm-up leaves no trace
            before = {t.data_ptr(): t.clone() for t in self._state()}  # keyed by storage: detach() is a new object
            s = torch.cuda.Stream(self.x.device)
            s.wait_stream(torch.cuda.current_stream(self.x.device))
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    train_step(self.model, self.optimizer, self.criterion, self.x, self.y, self.sync)
            torch.cuda.current_stream(self.x.device).wait_stream(s)
            with torch.no_grad():
                for t in self._state():
                    if t.data_ptr() in before:
                        t.copy_(before[t.data_ptr()])
                    else:  # a momentum buffer the warm-up created: zero gives SGD's first-step update
                        t.zero_()
        self.optimizer.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        # with a process group the RCCL watchdog thread keeps querying the eager collectives' events
        # while this thread captures: only this thread's calls may be checked against the capture
        mode = "thread_local" if self.sync is not None else "global"
        with torch.cuda.graph(g, capture_error_mode=mode):  # records only: nothing runs until replay
            self.out = train_step(self.model, self.optimizer, self.criterion, self.x, self.y, self.sync)
        self.graph = g
        self._lr = self._lrs()

    def step(self, images: torch.Tensor, labels: torch.Tensor):
        if tuple(images.shape) != tuple(self.x.shape) or tuple(labels.shape) != tuple(self.y.shape):
            raise RuntimeError("GraphedTrainStep: the batch shape changed (%s); capture another step"
                               % (tuple(images.shape),))
        self.x.copy_(images, non_blocking=True)
        self.y.copy_(labels, non_blocking=True)
        if self.graph is None or self._lrs() != self._lr:
            self._capture()
        self.graph.replay()
        return self.out[0].clone(), self.out[1].clone()


def shard_batches(images: torch.Tensor, labels: torch.Tensor, batch_size: int, epoch: int, seed: int = 0):
    """DistributedSampler(shuffle=True) order for this rank, in batches."""
    rank, world = _world()
    g = torch.Generator().manual_seed(seed + epoch)
    idx = torch.randperm(len(labels), generator=g)
    pad = (-len(idx)) % world
    idx = torch.cat([idx, idx[:pad]])[rank::world]
    return [(images[idx[i:i + batch_size]], labels[idx[i:i + batch_size]]) for i in range(0, len(idx), batch_size)]


def run_train_loop(model: nn.Module, device, images: torch.Tensor, labels: torch.Tensor, batch_size: int,
                   model_path: Optional[str], num_epochs: int, lr: float, log=print,
                   graph: bool = False) -> List[Row]:
    """train.py:37-125; returns (epoch, train_loss, train_acc, quantization_error) rows.
    graph=True (HIP device, a model built with ddp=False): full batches run as a GraphedTrainStep replay
    (under a process group with DDP's per-step collectives captured in it), a trailing partial batch
    eagerly (with the same collectives)."""
    rank, world = _world()
    optimizer, warmup, multistep, warmup_epochs = make_optimizer(model, lr, num_epochs)
    criterion = nn.CrossEntropyLoss()
    rows: List[Row] = []
    if world > 1:
        dist.barrier()
    core = model.module if isinstance(model, DistributedDataParallel) else model
    # a plain module under a process group (build_model(..., ddp=False)): DDP's per-step collectives
    sync = GradSync(model) if dist.is_available() and dist.is_initialized() and \
        not isinstance(model, DistributedDataParallel) else None
    graphed = None
    for epoch in range(num_epochs):
        total_loss = torch.zeros((), dtype=torch.float32, device=device)
        total_samples = torch.zeros((), dtype=torch.int64, device=device)
        total_correct = torch.zeros((), dtype=torch.int64, device=device)
        model.train()
        for x, y in shard_batches(images, labels, batch_size, epoch):
            x, y = x.to(device), y.to(device)
            if graph and x.is_cuda and x.size(0) == batch_size and not isinstance(model, DistributedDataParallel):
                if graphed is None:
                    graphed = GraphedTrainStep(model, optimizer, criterion, x, y)
                ls, c = graphed.step(x, y)
            else:
                ls, c = train_step(model, optimizer, criterion, x, y, sync)
            total_loss += ls
            total_correct += c
            total_samples += y.size(0)
        (warmup if epoch < warmup_epochs else multistep).step()
        if world > 1:  # sum across processes
            for t in (total_loss, total_samples, total_correct):
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
        loss = total_loss.item() / total_samples.item()
        acc = total_correct.item() / total_samples.item()
        err, numel = core.get_quantization_error()
        qerr = err / numel
        qerr = qerr.item() if isinstance(qerr, torch.Tensor) else float(qerr)
        if rank == 0:
            log(f"epoch: {epoch}, train_loss: {loss:.4f}, train_acc: {acc:.4f}, quantization_error: {qerr:.10f}")
        rows.append((epoch, loss, acc, qerr))
    if model_path is not None and rank == 0:
        Path(os.path.dirname(model_path) or ".").mkdir(parents=True, exist_ok=True)
        torch.save(model.state_dict(), model_path)
    return rows


def write_train_csv(path: str, rows: List[Row]) -> None:
    """{train_dir}/{dataset}/{model}/{seed}/{config}.csv (train.py:255-259)."""
    Path(os.path.dirname(path) or ".").mkdir(parents=True, exist_ok=True)
    with open(path, mode="w") as f:
        writer = csv.writer(f)
        writer.writerow(["epoch", "train_loss", "train_acc", "quantization_error"])
        writer.writerows(rows)
