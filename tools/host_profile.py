"""Host-side cost of an eager C2 energy+force evaluation (bench model, 32 QM9-like molecules), scripted
and unscripted: torch.profiler CPU self time per op, the launch count, and wall time per evaluation
with the GPU idle-waiting (host-bound when wall ~= host enqueue time).
usage (GPU box): python tools/host_profile.py [script|eager|eager_eval|both] [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "torchmd-net_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from torchmdnet.models.model import create_model
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = create_model(bench.et_args(128)).to(dev)
    z, pos, batch = bench.qm9_like(32, gen_seed=1)
    z, pos, batch = z.to(dev), pos.float().to(dev), batch.to(dev)
    forms = []
    if which in ("eager", "both"):
        forms.append(("eager", model))
    if which in ("eager_eval", "both"):  # eval mode: the C++ et_stack route (torchmd_et.CPP_EAGER)
        forms.append(("eager_eval", create_model(bench.et_args(128)).to(dev).eval()))
    if which in ("script", "both"):
        forms.append(("script", torch.jit.script(model)))
    if which in ("variants", "both"):  # the scripted model under other executor settings
        m_eval = create_model(bench.et_args(128)).to(dev).eval()
        try:
            forms.append(("script_frozen_eval", torch.jit.freeze(torch.jit.script(m_eval))))
        except Exception as e:  # noqa: BLE001
            print("freeze failed:", type(e).__name__, str(e)[:200])
        forms.append(("script_eval", torch.jit.script(m_eval)))
    if which == "noprof":  # the legacy (non-profiling) graph executor
        torch._C._jit_set_profiling_executor(False)
        forms.append(("script_legacy_executor", torch.jit.script(model)))
    for name, m in forms:
        for _ in range(5):
            m(z, pos, batch)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        host = 0.0
        for _ in range(n):
            h0 = time.perf_counter()
            y, f = m(z, pos, batch)
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n
        print(f"== {name}: wall {1e3 * wall:.3f} ms/eval, host enqueue {1e3 * host / n:.3f} ms/eval", flush=True)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            for _ in range(5):
                m(z, pos, batch)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=rows), flush=True)


if __name__ == "__main__":
    main()
