set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
TMDNET_TN_EBD_S=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_tn_kernels.py tests/test_gpu_parity.py -k "tn or tensor" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ebd_tests.log 2>&1 || { tail -30 gpurun_out/ebd_tests.log; exit 1; }
tail -1 gpurun_out/ebd_tests.log
for S in 8 4; do
  cd /tmp && rm -rf /tmp/prof_e$S
  TMDNET_TN_EBD_S=$S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_e$S -o run -- python3 $R/tools/graph_trace.py tn > /dev/null 2>&1
  python3 $R/tools/trace_summary.py "$(find /tmp/prof_e$S -name '*kernel_trace.csv')" > $R/gpurun_out/ebd_S$S.txt
  echo "EBD S=$S"; grep -E "kernels per step|busy" $R/gpurun_out/ebd_S$S.txt; grep -E "^ +[0-9.]+ +[0-9]+ .*k_embed_bwd_dst" $R/gpurun_out/ebd_S$S.txt
done
