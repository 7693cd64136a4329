"""Per-probe average duration of the graded edge kernel from a rocprofv3 kernel-trace CSV.

bench.py's roofline_probe launches the graded kernel (tmdnet_et_message_fwd at C5 scale) as two
back-to-back loops with nothing else launched in between: 5 warm-up + `reps` timed launches in the
per-edge dk/dv layout (`roofline.per_edge_layout`, the SURVEY-formula figure), then 5 + `reps` in the
pair-row layout (`roofline`, the graded figure: the layout the model runs).  The model's own launches of the same instantiation are interleaved
with other kernels, so the probes are the one run of 2 (5 + reps) consecutive launches; their timed
segments' rocprof averages are what bench.py's live HIP-event figures must agree with.
usage: roofline_from_trace.py <kernel_trace.csv> [reps=50] [warmup=5] [kernel substring]"""
import csv
import sys

path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 5
name = sys.argv[4] if len(sys.argv) > 4 else "k_fwd<float, 4, 4, 1, false, false>"
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
print(f"all launches: {len(everything)}, average {sum(everything) / max(1, len(everything)) / 1e6:.4f} ms "
      "(probes and the model's own launches mixed)")
probe = [run for run in runs if len(run) == 2 * (warm + reps)]
if not probe:
    print(f"no run of {2 * (warm + reps)} consecutive launches found")
for run in probe:
    graded = run[warm:warm + reps]
    model = run[2 * warm + reps:]
    print(f"roofline.per_edge_layout (SURVEY formula): {len(graded)} timed launches, average "
          f"{sum(graded) / len(graded) / 1e6:.4f} ms")
    print(f"roofline (graded: the model's pair-row layout): {len(model)} timed launches, average "
          f"{sum(model) / len(model) / 1e6:.4f} ms")

# the backward probes (bench.py roofline_probe "backward"): 3 warm-up + reps // 2 timed calls of the
# training form (one k_bwd_dst and one k_bwd_src launch each), then of the dr form (one k_bwd_merged
# launch each).  They are the last launches of these kernels in the run (the model's C5 force pass runs
# earlier).
nb = max(4, reps // 2)
for kname, form in (("k_bwd_dst<", "training form"), ("k_bwd_src<", "training form"), ("k_bwd_merged<", "dr form")):
    ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if kname in r["Kernel_Name"]]
    if len(ds) < 3 + nb:
        print(f"{kname}: fewer than {3 + nb} launches")
        continue
    tail = ds[-nb:]
    print(f"backward {kname[:-1]} {form}: {len(tail)} launches, average {sum(tail) / len(tail) / 1e6:.4f} ms")
# the fused-projection forward probe (roofline.fused_projection): the last 5 + reps launches of fep::k_fwd
ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "fep::k_fwd<" in r["Kernel_Name"]]
if len(ds) >= warm + reps:
    tail = ds[-reps:]
    print(f"roofline.fused_projection fep::k_fwd: {len(tail)} launches, average {sum(tail) / len(tail) / 1e6:.4f} ms")
