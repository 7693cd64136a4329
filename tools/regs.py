"""Register / LDS / spill table of every kernel of one .hip file, from the compiler's remarks:
    python3 tools/regs.py torchmd-net_amd/csrc/et_fused.hip [extra hipcc flags]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Iinclude",
       "-Itorchmd-net_amd/csrc", "-Wno-unused-function", *sys.argv[2:], "-c", sys.argv[1], "-o", "/tmp/regs_tmp.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = m.group(2)
    if "error" in line:
        print(line)
for r in rows:
    g = lambda k: r.get(k, "?")  # noqa: E731
    print(f"{g('VGPRs'):>4} vgpr {g('VGPRs Spill'):>4} spill {g('Occupancy [waves/SIMD]'):>2} occ "
          f"{g('LDS Size [bytes/block]'):>7} lds  {r['name']}")
