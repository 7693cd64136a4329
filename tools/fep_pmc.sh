# PMC passes over the fused forward kernel alone (one rocprofv3 run per pass; each pass within the
# per-block counter slots).  Usage on the box: bash tools/fep_pmc.sh <mode>
set -o pipefail
mkdir -p gpurun_out/fep_pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
m=${1:-2}
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE"; do
  i=$((i+1))
  TMDNET_FEP_MODE=$m timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/fep_pmc/p$i -o run -- python3 $R/tools/fep_time.py 50001 64 fused_only > $R/gpurun_out/fep_pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/fep_pmc/p$i.log; exit 1; }
done
cd $R && python3 - > gpurun_out/fep_pmc/summary.txt <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/fep_pmc/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "k_fwd" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f.split("/")[2], k, "per-dispatch mean", sum(v) / max(1, len(v)), "n", len(v))
PY
cat gpurun_out/fep_pmc/summary.txt; rm -rf gpurun_out/fep_pmc/p1 gpurun_out/fep_pmc/p2 gpurun_out/fep_pmc/p3
