"""Per-probe average duration of the graded edge kernel from a rocprofv3 kernel-trace CSV.

bench.py's roofline_probe launches the graded kernel (tmdnet_et_message_fwd at C5 scale) as two
back-to-back loops with nothing else launched in between: 5 warm-up + `reps` timed launches in the
per-edge dk/dv layout (`roofline`, the graded SURVEY-formula figure), then 5 + `reps` in the pair-row
layout (`roofline.model_layout`).  The model's own launches of the same instantiation are interleaved
with other kernels, so the probes are the one run of 2 (5 + reps) consecutive launches; their timed
segments' rocprof averages are what bench.py's live HIP-event figures must agree with.
usage: roofline_from_trace.py <kernel_trace.csv> [reps=50] [warmup=5] [kernel substring]"""
import csv
import sys

path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 5
name = sys.argv[4] if len(sys.argv) > 4 else "k_fwd<float, 4, 1, 1, false>"
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
    print(f"roofline (per-edge layout, graded): {len(graded)} timed launches, average "
          f"{sum(graded) / len(graded) / 1e6:.4f} ms")
    print(f"roofline.model_layout (pair rows): {len(model)} timed launches, average "
          f"{sum(model) / len(model) / 1e6:.4f} ms")

# the backward probes (bench.py roofline_probe "backward"): 3 warm-up + reps // 2 timed calls of the
# training form, then of the dr form; each call is one k_bwd_dst and one k_bwd_src launch.  They are the
# last launches of these kernels in the run (the model's C5 force pass runs earlier).
nb = max(4, reps // 2)
for kname in ("k_bwd_dst<", "k_bwd_src<"):
    ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if kname in r["Kernel_Name"]]
    if len(ds) < 2 * (3 + nb):
        print(f"{kname}: fewer than {2 * (3 + nb)} launches")
        continue
    tail = ds[-2 * (3 + nb):]
    tr, dr = tail[3:3 + nb], tail[3 + nb + 3:]
    print(f"backward {kname[:-1]} training form: {len(tr)} launches, average {sum(tr) / len(tr) / 1e6:.4f} ms; "
          f"dr form: {len(dr)} launches, average {sum(dr) / len(dr) / 1e6:.4f} ms")
