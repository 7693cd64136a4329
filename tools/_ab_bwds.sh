set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
for S in 8 4; do
  cd /tmp && rm -rf /tmp/prof_b$S
  TMDNET_ET_BWD_S=$S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_b$S -o run -- python3 $R/tools/graph_trace.py et > /dev/null 2>&1
  python3 $R/tools/trace_summary.py "$(find /tmp/prof_b$S -name '*kernel_trace.csv')" > $R/gpurun_out/bwds_S$S.txt
  echo "S=$S"; grep -E "kernels per step|busy" $R/gpurun_out/bwds_S$S.txt; grep -E "^ +[0-9.]+ +[0-9]+ .*k_bwd_both" $R/gpurun_out/bwds_S$S.txt
done
