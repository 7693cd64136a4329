set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tn_kernels.py tests/test_gpu_tn_padding.py tests/test_gpu_parity.py tests/test_gpu_periodic_oracle.py tests/test_gpu_train_parity.py tests/test_torchscript.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tns_tests.log 2>&1 || { tail -40 gpurun_out/tns_tests.log; exit 1; }
tail -1 gpurun_out/tns_tests.log
export TMPDIR=/tmp
R=$(pwd)
for S in 1 2 4; do
  cd /tmp && rm -rf /tmp/prof_tn$S
  TMDNET_TN_S=$S timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn$S -o run -- python3 $R/tools/graph_trace.py tn > /dev/null 2>&1
  python3 $R/tools/trace_summary.py "$(find /tmp/prof_tn$S -name '*kernel_trace.csv')" > $R/gpurun_out/tns_c3_S$S.txt
  echo "S=$S"; grep -E "kernels per step|busy" $R/gpurun_out/tns_c3_S$S.txt; grep -E "tn::k_" $R/gpurun_out/tns_c3_S$S.txt | grep -v "^[0-9] " | head -12
done
