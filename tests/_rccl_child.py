"""Child process of tests/test_gpu_rccl.py (a fresh process: a process group is process-wide state).

A one-rank RCCL process group on cuda:0 (backend "nccl" = RCCL on ROCm; init over tcp://127.0.0.1),
then:
  1. bench.py's output gather (gather_buffer / gather_logits, the all_gather_into_tensor of the
     batch-sharded inference) on device logits of the real quantized-conv chain;
  2. the reference's DDP QAT step (train.py:79-94, 153-155: qat.build_model wraps in DDP under any
     process group), eagerly through DDP, and replayed from one HIP graph with DDP's per-step
     collectives captured (qat.build_model(..., ddp=False) + qat.GraphedTrainStep + GradSync), from the
     same initial state.
Prints one JSON line."""
import faulthandler
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stage(name):
    print("stage:", name, file=sys.stderr, flush=True)


def main():
    faulthandler.enable()
    port = int(sys.argv[1])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1, device_id=dev)
    out = {"backend": str(dist.get_backend()), "world": dist.get_world_size()}

    stage("group up")
    import bench

    chain = bench.QConvChain(3, 10, "po2", 4, "auto", dev, seed=0)
    x = torch.relu(torch.randn(8, 16, 32, 32, generator=torch.Generator().manual_seed(4))).to(dev)
    with torch.no_grad():
        logits = chain.forward(x)
        gathered = bench.gather_buffer(8, 10, dev)
        got = bench.gather_logits(logits, gathered)
    torch.cuda.synchronize()
    out["gather_allocated"] = gathered is not None
    out["gather_is_buffer"] = got is gathered
    out["gather_equal"] = bool(torch.equal(got, logits))
    out["logits_finite"] = bool(torch.isfinite(logits).all())
    stage("gather done")

    from torch.nn.parallel import DistributedDataParallel

    from po2_quantization_amd import qat
    from po2_quantization_amd.utils.quantizers import quantizer_dict

    g = torch.Generator().manual_seed(11)
    batches = [(torch.randn(16, 3, 32, 32, generator=g).to(dev), torch.randint(0, 10, (16,), generator=g).to(dev))
               for _ in range(4)]
    crit = torch.nn.CrossEntropyLoss()

    def make():
        torch.manual_seed(3)
        m = qat.build_model("resnet20", 10, quantizer_dict["po2"], 4, (32, 32), dev)
        opt, _, _, _ = qat.make_optimizer(m, 0.05, 10)
        return m, opt

    m1, o1 = make()
    out["ddp_wrapped"] = isinstance(m1, DistributedDataParallel)
    for xb, yb in batches:
        l1, c1 = qat.train_step(m1, o1, crit, xb, yb)
    torch.cuda.synchronize()
    stage("eager ddp steps done")
    torch.manual_seed(3)  # the same initial state, built for the graph: no DDP wrapper (its hooks are not capturable)
    m2 = qat.build_model("resnet20", 10, quantizer_dict["po2"], 4, (32, 32), dev, ddp=False)
    o2, _, _, _ = qat.make_optimizer(m2, 0.05, 10)
    try:
        qat.GraphedTrainStep(m1, o1, crit, batches[0][0], batches[0][1])
        out["ddp_refused"] = False
    except RuntimeError:
        out["ddp_refused"] = True
    gs = qat.GraphedTrainStep(m2, o2, crit, batches[0][0], batches[0][1])
    for xb, yb in batches:
        l2, c2 = gs.step(xb, yb)
    torch.cuda.synchronize()
    stage("graphed steps done")
    out["graph_captured"] = gs.graph is not None and gs.sync is not None
    bad = []
    for (k, a), b in zip(m1.module.state_dict().items(), m2.state_dict().values()):
        if a.is_floating_point():
            if not torch.allclose(a, b, rtol=1e-5, atol=1e-6):
                bad.append([k, (a - b).abs().max().item()])
        elif not torch.equal(a, b):
            bad.append([k, "int"])
    out["graphed_vs_ddp_bad"] = bad
    out["loss_close"] = bool(torch.allclose(l1, l2, rtol=1e-4)) and bool(torch.equal(c1, c2))
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
