# Kernel-trace stats of tools/fep_time.py (fused vs unfused ET edge kernels on the C5 water box).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fep_tr -o run -- python3 $R/tools/fep_time.py 50001 ${1:-64} > $R/gpurun_out/fep_trace_run.log 2>&1 || { tail -20 $R/gpurun_out/fep_trace_run.log; exit 1; }
f=$(find /tmp/fep_tr -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us avg  x{r["Calls"]:>4}  {r["Name"][:110]}')
PY
