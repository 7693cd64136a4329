# Kernel trace of one replay of the captured ET-QM9 training step (GPU box, repo root):
#   bash tools/prof_train.sh <tag>  ->  gpurun_out/<tag>_train_step_kernels.txt
set -e -o pipefail
root=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && rm -rf /tmp/prof_train
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_train -o run -- \
  python3 "$root/tools/graph_trace.py" train > /dev/null 2> "$root/gpurun_out/prof_train.err"
csv=$(find /tmp/prof_train -name '*kernel_trace.csv' | head -1)
python3 "$root/tools/trace_summary.py" "$csv" summary > "$root/gpurun_out/$1_train_step_kernels.txt"
python3 "$root/tools/trace_summary.py" "$csv" > "$root/gpurun_out/$1_train_step_sequence.txt"
head -80 "$root/gpurun_out/$1_train_step_kernels.txt"
