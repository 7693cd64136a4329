set -e -o pipefail
root=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- python3 "$root/tools/graph_trace.py" tn > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_tn -name '*kernel_trace.csv' | head -1)" > "$root/gpurun_out/tn_c3_graph_step_kernels.txt"
