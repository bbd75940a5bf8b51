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
                                                   replayed (single process): ~1000 host launches
                                                   per step become one graph launch
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
                device, full_precision_model_path: Optional[str] = None, sync_bn: bool = True) -> nn.Module:
    """train.py:128-168: the model on `device`, DDP-wrapped when a process group exists
    (sync_bn=False keeps per-rank BatchNorm statistics, e.g. for a gloo test group)."""
    model = get_model(model_type=model_type, num_classes=num_classes, quantize_fn=quantize_fn, bits=bits,
                      image_size=image_size)
    _, world = _world()
    if world > 1 and sync_bn:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)  # same state_dict keys
    model = model.to(device)
    if world > 1:
        idx = device.index if isinstance(device, torch.device) else None
        model = DistributedDataParallel(model, device_ids=[idx] if idx is not None else None,
                                        output_device=idx)
    if quantize_fn is not None and full_precision_model_path is not None:
        assert os.path.exists(full_precision_model_path), "QAT requires full precision model"
        sd = torch.load(full_precision_model_path, map_location="cpu", weights_only=True)
        if world > 1:  # the reference loads the DDP state dict ("module." keys) into the DDP model
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


def train_step(model: nn.Module, optimizer, criterion, images: torch.Tensor, labels: torch.Tensor):
    """One iteration (train.py:79-94); returns (loss * batch, correct) as device tensors
    (no host synchronisation inside the step)."""
    optimizer.zero_grad()
    outputs = model(images)
    loss = criterion(outputs, labels)
    with torch.no_grad():
        correct = (outputs.argmax(1) == labels).sum()
    loss.backward()
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
    re-captured when a scheduler changes it (once per epoch).  Single process only (DDP's bucketed
    all-reduce is not captured here); the po2q autotuner runs in the eager warm-up steps, before
    capture (it synchronises the stream)."""

    def __init__(self, model: nn.Module, optimizer, criterion, images: torch.Tensor, labels: torch.Tensor,
                 warmup: int = 3):
        _, world = _world()
        if world > 1 or isinstance(model, DistributedDataParallel):
            raise RuntimeError("GraphedTrainStep: single-process training only")
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
                    train_step(self.model, self.optimizer, self.criterion, self.x, self.y)
            torch.cuda.current_stream(self.x.device).wait_stream(s)
            with torch.no_grad():
                for t in self._state():
                    if t.data_ptr() in before:
                        t.copy_(before[t.data_ptr()])
                    else:  # a momentum buffer the warm-up created: zero gives SGD's first-step update
                        t.zero_()
        self.optimizer.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):  # records only: nothing runs until replay
            self.out = train_step(self.model, self.optimizer, self.criterion, self.x, self.y)
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
    graph=True (single process, HIP device): full batches run as a GraphedTrainStep replay, a
    trailing partial batch eagerly."""
    rank, world = _world()
    optimizer, warmup, multistep, warmup_epochs = make_optimizer(model, lr, num_epochs)
    criterion = nn.CrossEntropyLoss()
    rows: List[Row] = []
    if world > 1:
        dist.barrier()
    core = model.module if isinstance(model, DistributedDataParallel) else model
    graphed = None
    for epoch in range(num_epochs):
        total_loss = torch.zeros((), dtype=torch.float32, device=device)
        total_samples = torch.zeros((), dtype=torch.int64, device=device)
        total_correct = torch.zeros((), dtype=torch.int64, device=device)
        model.train()
        for x, y in shard_batches(images, labels, batch_size, epoch):
            x, y = x.to(device), y.to(device)
            if graph and world == 1 and x.is_cuda and x.size(0) == batch_size:
                if graphed is None:
                    graphed = GraphedTrainStep(model, optimizer, criterion, x, y)
                ls, c = graphed.step(x, y)
            else:
                ls, c = train_step(model, optimizer, criterion, x, y)
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
