"""Post-training-quantization evaluation harness: the reference's
test.py flow on the drop-in modules, with its checkpoint layout and results CSV.

  init()                          test.py:24-31   seeds 42, cudnn.benchmark (-> po2q autotune)
  test_model(model, loader, dev)  test.py:34-47   top-1 accuracy
  load_distributed_state_dict     test.py:50-55   strips the DDP "module." prefix
  evaluate_seed(...)              test.py:96-159  full precision, ptq_{q}_{bits}, qat_{q}_{bits}
  write_results(path, rows)       test.py:161-164 header model,test_acc,quantization_error
  main(...)                       test.py:58-164  same directory layout:
      {train_dir}/{dataset}/{model_type}/{seed}/model_state/{full_precision|q_bits}.pth
      {train_dir}/{dataset}/{model_type}/{seed}/{q_bits}.csv   (QAT log, quantization_error column)
      {results_dir}/{dataset}/{model_type}/{seed}.csv

The reference builds its test loader with torchvision from downloaded CIFAR / ImageNet
(utils/dataloaders.py); neither is available offline, so main() takes the evaluation set as
a tensor file (`data_file`: {"images": [N, 3, H, W] float, "labels": [N] int64}, loaded with
weights_only=True) -- the loader is the only difference.  Checkpoints are loaded with
torch.load(weights_only=True) (the reference calls plain torch.load).
"""
import csv
import glob
import os
import random
from copy import deepcopy
from pathlib import Path
from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from .models.model import get_model
from .utils.quantizers import quantize_model, quantizer_dict

bits_to_try = [3, 4]  # test.py:21

Row = Tuple[str, float, float]


def init() -> None:
    """test.py:24-31.  cudnn.benchmark = True also switches on po2q's autotuning
    (_lib.benchmark follows torch.backends.cudnn.benchmark)."""
    random.seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    torch.cuda.manual_seed(42)
    torch.cuda.manual_seed_all(42)
    torch.backends.cudnn.deterministic = False
    torch.backends.cudnn.benchmark = True


def test_model(model: nn.Module, test_loader: Iterable, device) -> float:
    """Top-1 accuracy over (images, labels) batches (test.py:34-47)."""
    correct, total = 0, 0
    model.eval()
    with torch.no_grad():
        for images, labels in test_loader:
            images, labels = images.to(device), labels.to(device)
            outputs = model(images)
            _, predicted = torch.max(outputs.data, 1)
            total += labels.size(0)
            correct += (predicted == labels).sum().item()
    return correct / total


test_model.__test__ = False  # not a pytest test (name kept from the reference)


def load_distributed_state_dict(model: nn.Module, model_path: str) -> None:
    """Load a (possibly DistributedDataParallel-saved) state dict (test.py:50-55)."""
    state_dict = torch.load(model_path, map_location="cpu", weights_only=True)
    state_dict = {key.replace("module.", ""): value for key, value in state_dict.items()}
    model.load_state_dict(state_dict)


def _qat_error(csv_path: str) -> float:
    """Mean of the QAT log's quantization_error column (test.py:150-152)."""
    with open(csv_path) as f:
        vals = [float(r["quantization_error"]) for r in csv.DictReader(f)]
    return float(np.mean(vals)) if vals else float("nan")


def evaluate_seed(model_type: str, num_classes: int, image_size, seed_dir: str, test_loader: Sequence,
                  device, skip_qat: bool = False, bits: Sequence[int] = bits_to_try, log=print) -> List[Row]:
    """One seed's rows in the reference's order (test.py:98-159)."""
    rows: List[Row] = []
    model = get_model(model_type=model_type, num_classes=num_classes, quantize_fn=None, bits=4,
                      image_size=image_size)
    model.to(device)
    load_distributed_state_dict(model, os.path.join(seed_dir, "model_state", "full_precision.pth"))
    acc = test_model(model, test_loader, device)
    log(f"full_precision = {acc * 100:.2f}%, q_error = 0.0")
    rows.append(("full_precision", acc, 0.0))
    for quant_type, quantizer in quantizer_dict.items():  # post-training quantization
        for b in bits:
            model_copy = deepcopy(model)
            quant_error = quantize_model(model=model_copy, quantizer=quantizer, bits=b)
            acc = test_model(model_copy, test_loader, device)
            rows.append((f"ptq_{quant_type}_{b}", acc, quant_error))
            log(f"ptq_{quant_type}_{b} = {acc * 100:.2f}%, q_error = {quant_error:.10f}")
    if not skip_qat:  # quantization-aware-trained checkpoints
        for quant_type, quantizer in quantizer_dict.items():
            for b in bits:
                cfg = f"{quant_type}_{b}"
                m = get_model(model_type=model_type, num_classes=num_classes, quantize_fn=quantizer, bits=b,
                              image_size=image_size)
                m.to(device)
                load_distributed_state_dict(m, os.path.join(seed_dir, "model_state", f"{cfg}.pth"))
                acc = test_model(m, test_loader, device)
                quant_error = _qat_error(os.path.join(seed_dir, f"{cfg}.csv"))
                rows.append((f"qat_{cfg}", acc, quant_error))
                log(f"qat_{cfg} = {acc * 100:.2f}%, q_error = {quant_error:.10f}")
    return rows


def write_results(path: str, rows: Sequence[Row]) -> None:
    """results/{dataset}/{model_type}/{seed}.csv (test.py:161-164)."""
    Path(os.path.dirname(path) or ".").mkdir(parents=True, exist_ok=True)
    with open(path, mode="w") as f:
        writer = csv.writer(f)
        writer.writerow(["model", "test_acc", "quantization_error"])
        writer.writerows(rows)


def tensor_loader(data_file: str, batch_size: int):
    """(images, labels) batches from a tensor file (stands in for utils/dataloaders.py)."""
    d = torch.load(data_file, map_location="cpu", weights_only=True)
    images, labels = d["images"], d["labels"]
    return [(images[i:i + batch_size], labels[i:i + batch_size]) for i in range(0, len(labels), batch_size)]


def main(model_type: str, dataset: str, data_file: str, batch_size: int = 128, train_dir: str = "./train",
         results_dir: str = "./results", skip_qat: bool = False) -> None:
    """test.py:58-164 with the evaluation set from data_file."""
    assert torch.cuda.is_available(), "invalid hardware"
    assert model_type in ["resnet20", "resnet32", "resnet44", "resnet56", "mobilenet", "mobilevit"], \
        "invalid model type"
    assert dataset in ["cifar", "imagenet"], "invalid dataset"
    init()
    device = torch.device("cuda", 0)
    loader = tensor_loader(data_file, batch_size)
    num_classes = 10 if dataset == "cifar" else 1000
    image_size = (32, 32) if dataset == "cifar" else (224, 224)  # utils/dataloaders.py image sizes
    work_dir = f"{train_dir}/{dataset}/{model_type}"
    results_work_dir = f"{results_dir}/{dataset}/{model_type}"
    Path(results_work_dir).mkdir(parents=True, exist_ok=True)
    for seed_dir in sorted(glob.glob(f"{work_dir}/*")):
        seed = os.path.basename(seed_dir)
        rows = evaluate_seed(model_type, num_classes, image_size, seed_dir, loader, device, skip_qat)
        write_results(f"{results_work_dir}/{seed}.csv", rows)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("model_type")
    ap.add_argument("dataset")
    ap.add_argument("--data_file", required=True)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--train_dir", default="./train")
    ap.add_argument("--results_dir", default="./results")
    ap.add_argument("--skip_qat", action="store_true")
    a = ap.parse_args()
    main(a.model_type, a.dataset, a.data_file, a.batch_size, a.train_dir, a.results_dir, a.skip_qat)
