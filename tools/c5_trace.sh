# Kernel-trace stats of the C5 energy + force evaluation (tools/c5_time.py) under one edge-kernel variant.
# usage: bash tools/c5_trace.sh <TMDNET_FEP> <TMDNET_FEP_BWD> <tag>
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TMDNET_FEP=$1 TMDNET_FEP_BWD=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c5_tr_$3 -o run -- python3 $R/tools/c5_time.py 50001 3 > $R/gpurun_out/c5_trace_$3.run.log 2>&1 || { tail -20 $R/gpurun_out/c5_trace_$3.run.log; exit 1; }
f=$(find /tmp/c5_tr_$3 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over the run")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms  {float(r["AverageNs"])/1e3:9.1f} us avg  x{r["Calls"]:>4}  {r["Name"][:100]}')
PY
