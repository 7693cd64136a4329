#!/bin/bash
# Regenerates the judged GPU evidence under gpurun_out/prof_<tag>/ (copy into profiles/ afterwards):
#   bench.json               -- the full default bench line (CPU baseline, PMC traffic, graphed training)
#   bench_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats of a bench run (no PMC / CPU legs)
#   bench_under_rocprof.json -- that run's own JSON line (its live HIP-event roofline figure)
#   roofline_from_trace.txt  -- the same run's per-probe rocprof average of the graded kernel
#   et_c2_graph_step_kernels.txt / tn_c3_graph_step_kernels.txt -- kernel sequence of one replay
#   graphed_train_check.json -- bench-scale GraphedTrainStep vs eager (loss / gradients, time)
# usage (GPU box, from the repo root): bash tools/refresh_profiles.sh r01 [stats-only]
set -e -o pipefail
tag=${1:-r01}
root=$(pwd)
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
[ "$2" = "stats-only" ] || timeout -k 10 600 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
cd /tmp
rm -rf /tmp/prof_stats /tmp/prof_et /tmp/prof_tn
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_stats -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --no-pmc > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err"
cp "$(find /tmp/prof_stats -name '*kernel_stats.csv' | head -1)" "$out/bench_kernel_stats.csv"
python3 "$root/tools/roofline_from_trace.py" "$(find /tmp/prof_stats -name '*kernel_trace.csv' | head -1)" \
  > "$out/roofline_from_trace.txt"
[ "$2" = "stats-only" ] && exit 0
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_et -o run -- \
  python3 "$root/tools/graph_trace.py" et > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_et -name '*kernel_trace.csv' | head -1)" \
  > "$out/et_c2_graph_step_kernels.txt"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- \
  python3 "$root/tools/graph_trace.py" tn > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_tn -name '*kernel_trace.csv' | head -1)" \
  > "$out/tn_c3_graph_step_kernels.txt"
cd "$root"
timeout -k 10 240 python3 tools/graphed_train_check.py 30 > "$out/graphed_train_check.json" 2> "$out/gtr.err"
echo done
