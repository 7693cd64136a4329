set -o pipefail
mkdir -p gpurun_out/prof_r04
export TMPDIR=/tmp
R=$(pwd)
bash tools/r04_bench_evidence.sh || exit 1
cd /tmp && rm -rf /tmp/prof_tn
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- python3 $R/tools/graph_trace.py tn > /dev/null 2>&1
python3 $R/tools/trace_summary.py "$(find /tmp/prof_tn -name '*kernel_trace.csv')" > $R/gpurun_out/prof_r04/tn_c3_graph_step_kernels.txt
grep -E "kernels per step|busy" $R/gpurun_out/prof_r04/tn_c3_graph_step_kernels.txt
