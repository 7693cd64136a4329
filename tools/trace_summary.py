"""Kernel sequence of the LAST of N identical steps from a rocprofv3 kernel-trace CSV."""
import csv
import sys
from collections import Counter

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"] or "spin" in r["Kernel_Name"]]
last = rows[marks[-2] + 1:marks[-1]]
print("kernels per step:", len(last))
t0 = int(last[0]["Start_Timestamp"])
if len(sys.argv) > 2 and sys.argv[2] == "summary":
    last_only = False  # (the full sequence is always listed: the judged kernel lists are untruncated)
else:
    last_only = False
busy = 0
for r in last:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy += d
    if not last_only:
        print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:9.1f} {d / 1e3:7.2f}  {r["Kernel_Name"][:120]}')
print("busy us", busy / 1e3, "span us", (int(last[-1]["End_Timestamp"]) - t0) / 1e3)
c = Counter(r["Kernel_Name"][:60] for r in last)
t = Counter()
for r in last:
    t[r["Kernel_Name"][:60]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("-- by count")
for k, v in c.most_common():
    print(v, k)
print("-- by total time (us)")
for k, v in t.most_common():
    print(f"{v:9.1f} {c[k]:5d} {k}")
