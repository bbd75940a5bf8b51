"""PTQ harness (po2_quantization_amd/ptq.py): the reference test.py's
checkpoint layout (DDP "module." prefixes), row order and results CSV schema.  The
CPU tests cover the file formats; the GPU test runs the whole flow on ResNet20 and
checks the PTQ errors against the reference's (tests/golden/models.npz)."""
import csv
import os
import sys

import pytest
import torch

from po2_quantization_amd import ptq
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantizer_dict
from tests._util import GOLDEN, load_npz

sys.path.insert(0, GOLDEN)
from fill import seeded_fill_  # noqa: E402


def _ddp_save(model, path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save({"module." + k: v for k, v in model.state_dict().items()}, path)


def test_load_distributed_state_dict_strips_module_prefix(tmp_path):
    src = get_model("resnet20", 10, None, 4, (32, 32))
    seeded_fill_(src, seed=3)
    _ddp_save(src, str(tmp_path / "m.pth"))
    dst = get_model("resnet20", 10, None, 4, (32, 32))
    ptq.load_distributed_state_dict(dst, str(tmp_path / "m.pth"))
    for (k, a), (k2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_results_csv_schema_and_qat_error(tmp_path):
    rows = [("full_precision", 0.5, 0.0), ("ptq_po2_3", 0.25, 1.5e-4)]
    p = str(tmp_path / "res" / "cifar" / "resnet20" / "0.csv")
    ptq.write_results(p, rows)
    with open(p) as f:
        got = list(csv.reader(f))
    assert got[0] == ["model", "test_acc", "quantization_error"]
    assert got[1] == ["full_precision", "0.5", "0.0"] and got[2][0] == "ptq_po2_3"
    q = str(tmp_path / "po2_3.csv")
    with open(q, "w") as f:  # a QAT training log (train.py writes epoch rows)
        f.write("epoch,train_loss,quantization_error\n0,1.0,0.5\n1,0.9,0.25\n")
    assert ptq._qat_error(q) == pytest.approx(0.375)


@pytest.mark.gpu
def test_ptq_flow_resnet20(tmp_path):
    """full_precision + ptq_{po2,po2+,lin,lin+}_{3,4} + qat_* rows in the reference's order;
    the 4-bit PTQ errors equal the reference's quantize_model values."""
    d = load_npz("models.npz")
    seed_dir = tmp_path / "train" / "cifar" / "resnet20" / "0"
    fp = get_model("resnet20", 10, None, 4, (32, 32))
    seeded_fill_(fp, seed=7)  # the golden generator's weights
    _ddp_save(fp, str(seed_dir / "model_state" / "full_precision.pth"))
    for qn in quantizer_dict:
        for b in ptq.bits_to_try:
            _ddp_save(fp, str(seed_dir / "model_state" / ("%s_%d.pth" % (qn, b))))
            with open(seed_dir / ("%s_%d.csv" % (qn, b)), "w") as f:
                f.write("epoch,quantization_error\n0,%g\n" % (1e-4 * b))
    x = torch.from_numpy(d["x/cifar8"])
    loader = [(x, torch.arange(8) % 10)]
    rows = ptq.evaluate_seed("resnet20", 10, (32, 32), str(seed_dir), loader, "cuda:0", log=lambda s: None)
    names = [r[0] for r in rows]
    assert names[0] == "full_precision"
    assert names[1:9] == ["ptq_%s_%d" % (q, b) for q in quantizer_dict for b in (3, 4)]
    assert names[9:] == ["qat_%s_%d" % (q, b) for q in quantizer_dict for b in (3, 4)]
    for name, acc, err in rows:
        assert 0.0 <= acc <= 1.0
        if name.startswith("ptq_") and name.endswith("_4"):
            ref = float(d["ptq_err/resnet20/%s/4" % name[4:-2]])
            assert abs(err - ref) <= 1e-5 * ref, (name, err, ref)
        if name.startswith("qat_"):
            assert err == pytest.approx(1e-4 * int(name[-1]))
    ptq.write_results(str(tmp_path / "results" / "0.csv"), rows)
    assert (tmp_path / "results" / "0.csv").exists()
