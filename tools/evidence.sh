#!/bin/bash
# The judged evidence of a round (GPU box, repo root), in two GPU calls: the -m gpu suite, the full bench line (CPU
# baseline, PMC traffic), a rocprofv3 --kernel-trace --stats run of the bench (no PMC / CPU legs) with the
# per-probe trace average of the graded kernel, the kernel lists of one C2 / C3 graph replay and of one
# captured ET training step, the C5 per-kernel breakdown, the C2 PMC passes.
# Output: gpurun_out/prof_<tag>/ (copy into profiles/ as <tag>_*).
#   bash tools/evidence.sh <tag> part1 [skip-tests]   (tests, bench, bench under rocprof)
#   bash tools/evidence.sh <tag> part2                (graph-step traces, C5 breakdowns, training check, C2 PMC)
#   bash tools/evidence.sh <tag> part3                (the C5 fused kernels' PMC passes)
set -o pipefail
root=$(pwd)
tag=${1:?round tag}
shift
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ "$1" = "part3" ]; then  # the C5 fused kernels' PMC passes (forward, backward)
  timeout -k 10 600 bash tools/fep_pmc.sh fused_only ${tag}fwd > /dev/null 2>&1 && cp gpurun_out/${tag}fwd_pmc/summary.txt "$out/fep_fwd_pmc.txt"
  timeout -k 10 600 bash tools/fep_pmc.sh fused_bwd_only ${tag}bwd > /dev/null 2>&1 && cp gpurun_out/${tag}bwd_pmc/summary.txt "$out/fep_bwd_pmc.txt"
  ls "$out"
  exit 0
fi
if [ "$1" = "part1" ]; then
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1 || { tail -30 "$out/gputest.log"; exit 1; }
  tail -1 "$out/gputest.log"
fi
timeout -k 10 900 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));s=d['secondary'];r=d['roofline'];print('C2',d['ms_per_step'],d['value'],'roof',r['frac'],r.get('traffic'),'train',s['et_train_step']['graphed']['ms_per_step'],'tn_train',s['tn_train_step_c3'],'C5',s['et_water_box_c5']['ms_per_step'],'C5scr',s['et_scripted_c5'].get('ms_per_step'),'C3',s['tensornet_c3']['ms_per_step'],'scr',s['et_scripted_c2']['ms_per_step'],'cpu',d['cpu_baseline']['value'])"
cd /tmp && rm -rf /tmp/prof_stats /tmp/prof_et /tmp/prof_tn /tmp/prof_train
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_stats -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --no-pmc --no-secondary > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err" || { echo "rocprof bench failed"; tail -5 "$out/rocprof.err"; exit 1; }
cp "$(find /tmp/prof_stats -name '*kernel_stats.csv' | head -1)" "$out/bench_kernel_stats.csv"
python3 "$root/tools/roofline_from_trace.py" "$(find /tmp/prof_stats -name '*kernel_trace.csv' | head -1)" > "$out/roofline_from_trace.txt"
head -5 "$out/roofline_from_trace.txt"
exit 0
fi
cd /tmp && rm -rf /tmp/prof_et /tmp/prof_tn /tmp/prof_train
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_et -o run -- python3 "$root/tools/graph_trace.py" et > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_et -name '*kernel_trace.csv' | head -1)" > "$out/et_c2_graph_step_kernels.txt"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- python3 "$root/tools/graph_trace.py" tn > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_tn -name '*kernel_trace.csv' | head -1)" > "$out/tn_c3_graph_step_kernels.txt"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_train -o run -- python3 "$root/tools/graph_trace.py" train > /dev/null 2>&1
csv=$(find /tmp/prof_train -name '*kernel_trace.csv' | head -1)
python3 "$root/tools/trace_summary.py" "$csv" > "$out/train_step_kernels.txt"
grep -h "kernels per step\|busy" "$out/et_c2_graph_step_kernels.txt" "$out/tn_c3_graph_step_kernels.txt" "$out/train_step_kernels.txt"
cd "$root"
timeout -k 10 360 bash tools/c5_profile.sh ${tag}ev > /dev/null 2>&1 && cp gpurun_out/${tag}ev_c5_kernel_stats.csv "$out/c5_kernel_stats.csv" && cp gpurun_out/${tag}ev_c5time.json "$out/c5_time.json"
timeout -k 10 240 python3 tools/graphed_train_check.py 30 > "$out/graphed_train_check.json" 2> "$out/gtr.err" || echo "graphed train check failed"
timeout -k 10 420 bash tools/c2_pmc.sh ${tag}ev > /dev/null 2>&1 && cp gpurun_out/${tag}ev_pmc/summary.txt "$out/c2_pmc.txt"
# TensorNet: the captured C3 training step's kernels, the C5 water box breakdown
cd /tmp && rm -rf /tmp/prof_tntrain
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tntrain -o run -- python3 "$root/tools/graph_trace.py" tn_train > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_tntrain -name '*kernel_trace.csv' | head -1)" > "$out/tn_train_step_kernels.txt"
grep -h "kernels per step\|busy" "$out/tn_train_step_kernels.txt"
cd "$root"
timeout -k 10 400 bash tools/tn_c5_profile.sh ${tag}tn > /dev/null 2>&1 && cp gpurun_out/${tag}tn_tn_c5_kernel_stats.csv "$out/tn_c5_kernel_stats.csv" && cp gpurun_out/${tag}tn_tnc5time.json "$out/tn_c5_time.json"
echo done
