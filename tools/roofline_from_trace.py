"""Per-probe average duration of the graded edge kernel from a rocprofv3 kernel-trace CSV.

bench.py launches the graded kernel (tmdnet_et_message_fwd at C5 scale) in two back-to-back probe
loops -- `roofline` (per-edge dk/dv layout, the SURVEY formula) then `roofline.model_layout`
(pair-shared rows) -- with nothing else launched in between, while the model's own launches of the
same instantiation are interleaved with other kernels.  The run-length of consecutive launches
therefore separates the probes; their rocprof averages are what bench.py's live HIP-event figures
must agree with.  usage: roofline_from_trace.py <kernel_trace.csv> [kernel substring] [min run]"""
import csv
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_fwd<float, 4, 1, 1, false>"
min_run = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
runs, cur = [], []
for r in rows:
    if name in r["Kernel_Name"]:
        cur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    elif cur:
        runs.append(cur)
        cur = []
if cur:
    runs.append(cur)
everything = [d for run in runs for d in run]
print(f"kernel: {name}")
print(f"all launches: {len(everything)}, average {sum(everything) / max(1, len(everything)) / 1e6:.4f} ms")
for i, run in enumerate(r for r in runs if len(r) >= min_run):
    label = ["roofline (per-edge layout, graded)", "roofline.model_layout (pair rows)"][i] if i < 2 else "run"
    print(f"probe run {i}: {label}: {len(run)} consecutive launches, average {sum(run) / len(run) / 1e6:.4f} ms")
