"""The graded C5 probe alone (bench.probe_workload: ET message forward in the pair-row layout, its
dr-form backward), HIP-event timed -- for A/B of launch switches read at import (TMDNET_ET_S, ...).
usage (GPU box): TMDNET_ET_S=4 python tools/pair_probe.py [n_atoms]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torchmd-net_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50001
dev = torch.device("cuda", 0)
launch, E, L = bench.probe_workload(n, 128, dev)
ms_p = bench._event_ms(launch.pairs, 30)
ms_b = bench._event_ms(lambda: launch.bwd(True), 10)
pb = bench.et_pair_bytes(E, n, launch.n_pairs, 128)
print(json.dumps({"S": os.environ.get("TMDNET_ET_S"), "pairs_fwd_ms": round(ms_p, 4),
                  "frac": round(pb / (ms_p * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4), "dr_bwd_ms": round(ms_b, 4)}))
