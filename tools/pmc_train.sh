# PMC counters of the captured training step's kernels (GPU box, repo root): one pass per counter set,
# per-kernel averages over the replays of tools/graph_trace.py train.  bash tools/pmc_train.sh <tag>
set -e -o pipefail
root=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  rm -rf /tmp/pmc_tr_$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc_tr_$i -o run -- \
    python3 "$root/tools/graph_trace.py" train > /dev/null 2> "$root/gpurun_out/$1_pmc_$i.err"
  python3 - "$(find /tmp/pmc_tr_$i -name '*counter_collection*.csv' | head -1)" "$set" >> "$root/gpurun_out/$1_pmc.txt" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:70]
    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
print("== " + sys.argv[2])
for (k, c), v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    if any(s in k for s in ("k_bwd2", "k_bwd_both", "k_gemm", "k_fwd", "k_ln_bwd", "k_adj", "MT64x32", "Cijk")):
        print(f"{c:16s} {sum(v) / len(v):16.1f} n={len(v):4d}  {k}")
PY
done
head -80 "$root/gpurun_out/$1_pmc.txt"
