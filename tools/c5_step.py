"""C5 (ET, 50,001-atom periodic water box) energy+force steps exactly as bench.py's secondary line,
for rocprofv3 --kernel-trace --stats (per-kernel time of the large-system step).
usage: c5_step.py [steps]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "torchmd-net_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
a = argparse.Namespace(roofline_atoms=50001, channels=128, steps=10 * steps)
dev = torch.device("cuda", 0)
print(bench.secondary_water_box(a, 1, 0, dev))
