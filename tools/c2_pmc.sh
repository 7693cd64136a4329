# PMC passes over the graph-replayed C2 step (tools/graph_trace.py et: the bench workload), one rocprofv3
# run per pass within the per-block counter slots; per-kernel means (one dispatch = one launch of a
# replay).  usage (GPU box, repo root): bash tools/c2_pmc.sh [tag] [et|train]
set -o pipefail
tag=${1:-c2}
what=${2:-et}
out=gpurun_out/${tag}_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/$out/p$i -o run -- python3 $R/tools/graph_trace.py $what > $R/$out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$out/p$i.log; exit 1; }
done
cd $R && python3 - $out > $out/summary.txt <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "").split("(")[0].replace("void ", "")
        acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
names = sorted({k for k, _ in acc})
for kn in names:
    vals = {c: sum(v) / len(v) for (k, c), v in acc.items() if k == kn}
    n = max(len(v) for (k, c), v in acc.items() if k == kn)
    wc = vals.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{kn[:70]:70s} n={n:5d} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items()))
          + f" | wait/wave={vals.get('SQ_WAIT_ANY', 0) / wc:.3f} valu/wave={vals.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}")
PY
cat $out/summary.txt; rm -rf $out/p1 $out/p2 $out/p3 $out/p4
