"""Group the kernels of one marked step (rocprofv3 kernel trace) by name: count, total us."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"] or "spin" in r["Kernel_Name"]]
step = rows[marks[-2] + 1:marks[-1]]
agg = defaultdict(lambda: [0, 0.0])
for r in step:
    k = r["Kernel_Name"]
    k = k.split("(")[0][:90] if not k.startswith("Cijk") else "GEMM " + k.split("_MT")[1][:14]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"kernels {len(step)}  busy {tot:.0f} us  span {(int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])) / 1e3:.0f} us")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{t:9.1f} us {n:5d}  {k}")
