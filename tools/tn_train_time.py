"""C3 training step timing (bench.secondary_tn_train: TensorNet-rMD17, 8 x aspirin, E + F MSE, double
backward, AdamW), eager and graph-replayed; TMDNET_TN_SECOND_ORDER=composite for the autograd
restatement of the second order (A/B).  usage (GPU box, repo root): python tools/tn_train_time.py"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402

a = SimpleNamespace(steps=40, warmup=10, graphed_train=True)
out = bench.secondary_tn_train(a, 1, 0, torch.device("cuda", 0))
out["second_order"] = os.environ.get("TMDNET_TN_SECOND_ORDER", "hip")
print(json.dumps(out))
