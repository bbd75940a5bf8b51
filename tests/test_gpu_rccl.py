"""RCCL on the MI355X (Missing #1/#2): a one-rank `nccl` process group (RCCL on ROCm)
created on the box, the bench's logits all_gather run through it, and the reference's DDP QAT step
(train.py:79-94, 153-155) run eagerly through DDP and from a HIP graph with DDP's collectives captured.
The work runs in a fresh child process (tests/_rccl_child.py): a process group is process-wide."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_gather_and_graphed_ddp_step():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "_rccl_child.py"), str(port)], cwd=root,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["backend"] == "nccl" and out["world"] == 1, out
    assert out["gather_allocated"] and out["gather_is_buffer"] and out["gather_equal"] and out["logits_finite"], out
    assert out["ddp_wrapped"] and out["graph_captured"] and out["ddp_refused"], out
    assert out["graphed_vs_ddp_bad"] == [] and out["loss_close"], out
