"""N > 1 path of bench.py on CPU: world_size-2 gloo process group (127.0.0.1).

Batch-sharded inference: every rank runs its own shard, the logits are gathered
with all_gather (RCCL over xGMI on the GPU box, gloo here), and the step time is
the MAX over ranks, measured between barriers (bench.py gather_logits /
timed_steps)."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from po2_quantization_amd import qat
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantizer_dict


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    B, classes = 4, 10
    w = torch.randn(16, classes, generator=torch.Generator().manual_seed(0))  # replicated "weights"
    x = torch.randn(B, 16, generator=torch.Generator().manual_seed(100 + rank))  # this rank's shard
    gathered = torch.empty(world * B, classes)
    calls = []

    def step(record=False):
        calls.append(record)
        time.sleep(0.05 * (rank + 1))  # rank 1 is the slow one
        return bench.gather_logits(x @ w, gathered, world)

    dt = bench.timed_steps(step, 3, 2, world, lambda: None, torch.device("cpu"))
    torch.save({"dt": dt, "gathered": gathered.clone(), "calls": calls, "x": x}, os.path.join(out_dir, "r%d.pt" % rank))
    dist.destroy_process_group()


def test_sharded_gather_and_max_over_ranks_timing(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / ("r%d.pt" % r), weights_only=True) for r in range(world)]
    w = torch.randn(16, 10, generator=torch.Generator().manual_seed(0))
    expect = torch.cat([res[r]["x"] @ w for r in range(world)])
    for r in range(world):
        assert torch.equal(res[r]["gathered"], expect)        # every rank holds every shard's logits
        assert res[r]["calls"] == [False, False, True, True, True]  # W untimed, then exactly K timed steps
    assert not torch.equal(res[0]["x"], res[1]["x"])           # distinct shards
    assert res[0]["dt"] == res[1]["dt"]                        # one reported time: the max over ranks
    assert res[0]["dt"] >= 3 * 0.1                             # covers the slower rank's 3 timed steps


def _cpu_standins(setattr_=setattr):
    """Test-only: the chain's native calls replaced by the oracle's CPU restatement (the GPU
    kernels have no CPU path), so the sharding itself runs here."""
    from oracle import oracle as O
    from po2_quantization_amd import _lib

    setattr_(_lib, "qconv2d", lambda x, w, b, st, pad, d, g, bits, mode, fsr=1, precision="auto":
             O.cpu_reference_qconv2d(x, w, b, st, pad, d, g, bits, mode))
    setattr_(_lib, "pair_supported", lambda *a, **k: False)
    setattr_(_lib, "s2ds_supported", lambda *a, **k: False)
    setattr_(_lib, "chain_supported", lambda *a, **k: False)  # the chain kernel: per-layer calls instead


def _chain_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    _cpu_standins()
    chain = bench.QConvChain(3, 10, "po2", 4, "auto", torch.device("cpu"), seed=0)  # replicated weights
    x = torch.relu(torch.randn(2, 16, 8, 8, generator=torch.Generator().manual_seed(100 + rank)))
    gathered = torch.empty(world * 2, 10)
    with torch.no_grad():
        out = bench.gather_logits(chain.forward(x), gathered, world)
    torch.save({"gathered": out.clone(), "x": x}, os.path.join(out_dir, "c%d.pt" % rank))
    dist.destroy_process_group()


def test_sharded_qconv_chain_equals_full_batch(tmp_path, monkeypatch):
    """bench.py's data-parallel step: each rank runs the ResNet20 quantized-conv chain (56-layer
    chain's structure at n = 3 blocks) on its own batch shard with the same seeded weights, and
    the all_gather of the logits equals the chain run on the whole batch in one process."""
    world = 2
    mp.spawn(_chain_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / ("c%d.pt" % r), weights_only=True) for r in range(world)]
    import bench

    _cpu_standins(monkeypatch.setattr)
    chain = bench.QConvChain(3, 10, "po2", 4, "auto", torch.device("cpu"), seed=0)
    with torch.no_grad():
        full = chain.forward(torch.cat([res[r]["x"] for r in range(world)]))
    for r in range(world):
        assert torch.allclose(res[r]["gathered"], full, rtol=1e-5, atol=1e-6)


def test_bench_entry_starts_n_ranks():
    """`python bench.py --gpus 2` (the driver's command shape) starts the two ranks itself through
    torch.distributed.run and relays rank 0's line: the process group holds 2 ranks, and rank 0 holds
    both shards' outputs after the all_gather.  --selftest runs the plumbing with CPU stand-in logits
    over gloo (no kernels here); the GPU box runs the same entry over RCCL."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest", "--steps", "3",
                        "--warmup", "1"], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["world_size"] == 2 and out["n_gpus"] == 2 and out["dist_backend"] == "gloo", out
    assert out["gathered_ok"] and out["gathered_rows"] == 8, out


def test_bench_entry_global_batch_1024_split():
    """Config 4's split (--global-batch 1024 over the ranks, reference README.md:42 / train.py:25-26) through
    the --gpus 2 entry: each rank runs its 512-image shard through the drop-in ResNet20's QuantizedConv2d
    layers (CPU path, po2 4-bit), the logits are all-gathered over gloo, and rank 0 finds them equal to one
    unsharded forward of all 1024 images."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest", "--steps", "2",
                        "--warmup", "1", "--global-batch", "1024", "--image", "8"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["global_batch"] == 1024 and out["batch_per_rank"] == 512 and out["gathered_rows"] == 1024, out
    assert out["gathered_ok"], out


def test_bench_entry_rejects_world_mismatch():
    """Under an external launcher the process group must hold exactly --gpus ranks."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest"], cwd=root,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "process group holds 1 ranks" in r.stderr, r.stderr[-2000:]


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def _gradsync_worker(rank, world, port, out):
    """The same 3 training steps twice from per-rank initial weights: through DDP (the reference's wrapper)
    and through the plain module of build_model(..., ddp=False) with qat.GradSync (the collectives
    GraphedTrainStep captures)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    dev = torch.device("cpu")
    g = torch.Generator().manual_seed(9)
    images = torch.randn(24, 3, 16, 16, generator=g)
    labels = torch.randint(0, 10, (24,), generator=g)
    crit = torch.nn.CrossEntropyLoss()
    res = []
    for use_sync in (False, True):
        torch.manual_seed(rank)  # different initial weights per rank: the construction broadcast aligns them
        m = qat.build_model("resnet20", 10, quantizer_dict["po2"], 4, (16, 16), dev, sync_bn=False, ddp=not use_sync)
        core = m.module if hasattr(m, "module") else m
        if rank == 1:  # per-rank BN statistics: the buffer broadcast must make rank 0's win
            with torch.no_grad():
                for b in core.buffers():
                    if b.is_floating_point():
                        b.add_(0.25)
        sync = qat.GradSync(m) if use_sync else None
        opt, _, _, _ = qat.make_optimizer(m, 0.01, 10)
        for x, y in qat.shard_batches(images, labels, 4, epoch=0):
            qat.train_step(m, opt, crit, x, y, sync)
        res.append(torch.cat([t.detach().double().flatten() for t in core.parameters()] +
                             [t.detach().double().flatten() for t in core.buffers()]))
    flat = torch.stack(res)
    gathered = [torch.empty_like(flat) for _ in range(world)]
    torch.distributed.all_gather(gathered, flat)
    if rank == 0:
        torch.save(torch.stack(gathered), out)
    torch.distributed.destroy_process_group()


def test_gradsync_equals_ddp_two_ranks(tmp_path):
    """GradSync (coalesced rank-0 buffer broadcast + averaged-gradient all_reduce, capturable in a HIP
    graph) reproduces DistributedDataParallel's training steps bit for bit over 2 gloo ranks, the reference's
    DDP step (train.py:79-94, 153-155) on the CPU path of the drop-in convs."""
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "state.pt")
    mp.spawn(_gradsync_worker, args=(2, port, out), nprocs=2, join=True)
    p = torch.load(out, weights_only=True)  # [rank][ddp | gradsync][parameters, buffers]
    n = sum(t.numel() for t in get_model("resnet20", 10, None, 4, (16, 16)).parameters())
    # parameters in lock-step on both routes (the buffers hold each rank's last local BN update)
    assert torch.equal(p[0, 0, :n], p[1, 0, :n]) and torch.equal(p[0, 1, :n], p[1, 1, :n])
    for r in range(2):  # and each rank's whole state equal between DDP and GradSync
        assert torch.equal(p[r, 0], p[r, 1]), (r, (p[r, 0] - p[r, 1]).abs().max())
