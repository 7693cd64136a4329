"""The multi-rank data-parallel training path on a GPU (VERDICT r2 "next" #5): two rank processes on
cuda:0 over gloo run the real ET-SPICE model through GraphedTrainStep (tests/multirank_worker.py).
Reference: Lightning DDP over NCCL, scripts/train.py:175-189."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_two_ranks_graphed_training_on_one_gpu(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "verdict.json"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(HERE, "multirank_worker.py"), str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    v = json.loads(out.read_text())
    print(json.dumps(v))
    assert v["world_size"] == 2
    assert v["initial_weights_differed"]  # the ranks really started from different weights ...
    assert v["all_start_from_rank0"]  # ... and the broadcast replaced them with rank 0's
    assert v["rank_grads_differ_rel"] > 1e-3  # different molecules -> different local gradients
    assert v["reduced_grad_vs_mean_of_eager_rel"] < 1e-5
    assert v["replicas_identical_after_5_steps"]
    assert v["weights_moved_rel"] > 0 and v["skipped_steps"] == 0
