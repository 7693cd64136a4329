# PMC passes over the fused kernels alone (one rocprofv3 run per pass; each pass within the per-block
# counter slots).  Usage on the box: bash tools/fep_pmc.sh [fused_only|fused_bwd_only] [tag]
set -o pipefail
what=${1:-fused_only}
tag=${2:-fep}
out=gpurun_out/${tag}_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_VMEM_WR" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/$out/p$i -o run -- python3 $R/tools/fep_time.py 50001 64 $what > $R/$out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$out/p$i.log; exit 1; }
done
cd $R && python3 - $out > $out/summary.txt <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
for f in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "fep::" in k:
            name = k.split("(")[0].split("fep::")[1]
            acc[(name, row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (kn, c), v in sorted(acc.items()):
        print(f.split("/")[2], kn, c, "per-dispatch mean", sum(v) / max(1, len(v)), "n", len(v))
PY
cat $out/summary.txt; rm -rf $out/p1 $out/p2 $out/p3 $out/p4
