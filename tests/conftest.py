import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "torchmd-net_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


def has_gpu():
    import torch
    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def state_dict_from(npz):
    return {k[3:]: npz[k] for k in npz.files if k.startswith("sd/")}


def yaml_args(model, **kw):
    """Reference example args (tests/utils.py:7-24 semantics) from committed copies of the configs."""
    import yaml
    cfg = "tensornet_qm9.yaml" if model == "tensornet" else "et_qm9.yaml"
    with open(os.path.join(GOLDEN, "configs", cfg)) as f:
        args = yaml.safe_load(f)
    args.setdefault("precision", 32)
    args["model"] = model
    args["prior_model"] = None
    args.update(kw)
    return args
