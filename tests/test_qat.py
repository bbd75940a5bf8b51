"""QAT training on the drop-in modules (po2_quantization_amd/qat.py):
gradients of the fused native forward + STE backward equal torch autograd of the
reference formulation; the train loop runs the reference's schedule; DDP keeps ranks
in lock-step (2 processes on one GPU, gloo).  GPU only."""
import os
import socket

import pytest
import torch
import torch.nn.functional as F

from po2_quantization_amd import _lib, qat
from po2_quantization_amd.models import quantized_conv as QC
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantizer_dict
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _torch_forward(self, input):
    """The reference's QuantizedConv2d.forward in torch ops (quantized_conv.py:32-38) with
    the quantizer's straight-through backward (quantizers.py:34-36)."""
    if self.quantize_fn is None:
        return F.conv2d(input, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
    qw = self.quantize_fn.apply(self.weight, self.bits)
    w = self.weight + (qw - self.weight).detach()
    return F.conv2d(input, w, self.bias, self.stride, self.padding, self.dilation, self.groups)


@pytest.mark.parametrize("qn", ["po2", "po2+", "lin"])
def test_qat_gradients_match_torch_autograd(qn, monkeypatch):
    torch.manual_seed(0)
    m = get_model("resnet20", 10, quantizer_dict[qn], 4, (32, 32)).to(DEV).train()
    x = torch.randn(16, 3, 32, 32, device=DEV)
    y = torch.randint(0, 10, (16,), device=DEV)
    F.cross_entropy(m(x), y).backward()
    g_native = {k: p.grad.clone() for k, p in m.named_parameters()}
    m.zero_grad()
    monkeypatch.setattr(QC.QuantizedConv2d, "forward", _torch_forward)
    F.cross_entropy(m(x), y).backward()
    for k, p in m.named_parameters():
        a, b = g_native[k], p.grad
        err = ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
        assert err <= 100 * CONV_TOL, (k, err)  # gradients pass ~20 layers of backward


def test_train_loop_reference_schedule(tmp_path):
    torch.manual_seed(1)
    m = qat.build_model("resnet20", 10, quantizer_dict["po2"], 4, (32, 32), torch.device(DEV))
    images = torch.randn(96, 3, 32, 32)
    labels = (images.mean(dim=(1, 2, 3)) > 0).long()  # a learnable synthetic task
    rows = qat.run_train_loop(m, torch.device(DEV), images, labels, 32, str(tmp_path / "po2_4.pth"),
                              num_epochs=4, lr=0.02, log=lambda s: None)
    assert [r[0] for r in rows] == [0, 1, 2, 3]
    assert all(torch.isfinite(torch.tensor(r[1])) and 0.0 <= r[2] <= 1.0 and r[3] > 0 for r in rows)
    assert rows[-1][1] < rows[0][1]  # loss goes down
    qat.write_train_csv(str(tmp_path / "po2_4.csv"), rows)
    assert open(tmp_path / "po2_4.csv").readline().strip() == "epoch,train_loss,train_acc,quantization_error"
    sd = torch.load(tmp_path / "po2_4.pth", weights_only=True)
    assert set(sd) == set(m.state_dict())


def _ddp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)  # identical initial weights on every rank (DDP also broadcasts them)
    m = qat.build_model("resnet20", 10, quantizer_dict["po2+"], 4, (32, 32), torch.device(DEV), sync_bn=False)
    opt, _, _, _ = qat.make_optimizer(m, 0.01, 10)
    crit = torch.nn.CrossEntropyLoss()
    g = torch.Generator().manual_seed(5)
    images = torch.randn(32, 3, 32, 32, generator=g)
    labels = torch.randint(0, 10, (32,), generator=g)
    for x, y in qat.shard_batches(images, labels, 8, epoch=0):
        qat.train_step(m, opt, crit, x.to(DEV), y.to(DEV))
    flat = torch.cat([p.detach().flatten() for p in m.parameters()]).cpu()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    torch.distributed.all_gather(gathered, flat)
    if rank == 0:
        torch.save(torch.stack(gathered), out)
    torch.distributed.destroy_process_group()


def test_ddp_two_ranks_stay_in_lockstep(tmp_path):
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "params.pt")
    mp.spawn(_ddp_worker, args=(2, port, out), nprocs=2, join=True)
    p = torch.load(out, weights_only=True)
    assert torch.equal(p[0], p[1])  # averaged gradients -> identical updates
    assert _lib.load() is not None


def test_graphed_train_step_equals_eager_steps():
    """GraphedTrainStep (the whole QAT step -- fused native forward, native backward, SGD -- replayed
    from one HIP graph) against the same steps run eagerly from the same initial
    state: the warm-up leaves no trace and every replay is the eager step's arithmetic.  Every conv
    of the step, the unquantized stem included (models/quantized_conv.py plain_conv), runs forward and
    backward natively with fixed-order reductions, so the bar is a fixed tolerance."""
    torch.backends.cudnn.benchmark = False
    _graphed_vs_eager()


def _native_stem_ran(m):
    """One training forward + backward of the model's stem: its weight gradient came from _QConv2dFn
    (the native kernels), not from aten / MIOpen."""
    from po2_quantization_amd.models import quantized_conv as qc

    seen = []
    orig = qc._QConv2dFn.backward

    def spy(ctx, gy):
        seen.append(ctx.conf[-1])
        return orig(ctx, gy)

    qc._QConv2dFn.backward = staticmethod(spy)
    try:
        m = m.train()
        x = torch.randn(2, 3, 32, 32, device=DEV)
        y = qc.plain_conv(m.conv1, x)
        y.sum().backward()
    finally:
        qc._QConv2dFn.backward = staticmethod(orig)
    m.zero_grad(set_to_none=True)
    return seen == ["none"]


def _graphed_vs_eager():
    g = torch.Generator().manual_seed(11)
    batches = [(torch.randn(16, 3, 32, 32, generator=g).to(DEV), torch.randint(0, 10, (16,), generator=g).to(DEV))
               for _ in range(4)]

    def make():
        torch.manual_seed(3)
        m = qat.build_model("resnet20", 10, quantizer_dict["po2"], 4, (32, 32), torch.device(DEV))
        opt, _, _, _ = qat.make_optimizer(m, 0.05, 10)
        return m, opt

    crit = torch.nn.CrossEntropyLoss()
    m1, o1 = make()
    for x, y in batches:
        l1, c1 = qat.train_step(m1, o1, crit, x, y)
    m0, o0 = make()  # eager twice: the run-to-run noise of the eager step itself (reported, not a bar)
    for x, y in batches:
        qat.train_step(m0, o0, crit, x, y)
    noise = {k: (a - b).abs().max().item() for (k, a), b in zip(m1.state_dict().items(), m0.state_dict().values())
             if a.is_floating_point()}
    assert _native_stem_ran(m1), "the stem did not run through the native conv"
    m2, o2 = make()
    gs = qat.GraphedTrainStep(m2, o2, crit, batches[0][0], batches[0][1])
    for x, y in batches:
        l2, c2 = gs.step(x, y)
    torch.cuda.synchronize()
    assert gs.graph is not None
    bad = []
    for (k, a), b in zip(m1.state_dict().items(), m2.state_dict().values()):
        if a.is_floating_point():
            if not torch.allclose(a, b, rtol=1e-5, atol=1e-6):
                bad.append((k, (a - b).abs().max().item(), a.abs().max().item(), noise[k]))
        elif not torch.equal(a, b):
            bad.append((k, "int", None))
    assert not bad, bad
    assert torch.allclose(l1, l2, rtol=1e-4) and torch.equal(c1, c2)
    # a learning-rate change re-captures the step
    for grp in o2.param_groups:
        grp["lr"] *= 0.1
    first = gs.graph
    gs.step(*batches[0])
    assert gs.graph is not first

