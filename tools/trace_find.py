"""Find kernels whose name matches argv[2] in the marked step of a kernel trace; print neighbours."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"] or "spin" in r["Kernel_Name"]]
step = rows[marks[-2] + 1:marks[-1]]
print("kernels in step", len(step))
keys = [k for k in rows[0].keys()]
print(keys)
for i, r in enumerate(step):
    if sys.argv[2] in r["Kernel_Name"]:
        print("----", i, r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", ""))
        for j in range(max(0, i - 4), min(len(step), i + 3)):
            rr = step[j]
            print("   ", j, rr.get("Grid_Size", rr.get("Grid_Size_X", "")), rr["Kernel_Name"][:110])
