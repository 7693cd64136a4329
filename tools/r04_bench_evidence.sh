#!/bin/bash
# The bench line (CPU baseline + PMC traffic) and a rocprofv3 --kernel-trace --stats run of the same bench
# with the per-probe trace average of the graded kernel, into gpurun_out/prof_r04/ (GPU box, repo root).
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/prof_r04
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));s=d['secondary'];r=d['roofline'];print('C2',d['ms_per_step'],d['value'],'roof',r['frac'],r.get('traffic'),'train',s['et_train_step']['graphed']['ms_per_step'],'C5',s['et_water_box_c5']['ms_per_step'],'C3',s['tensornet_c3']['ms_per_step'],'scr',s['et_scripted_c2']['ms_per_step'],'cpu',d['cpu_baseline']['value'])"
cd /tmp && rm -rf /tmp/prof_stats
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_stats -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --no-pmc > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err" || { echo "rocprof bench failed"; tail -5 "$out/rocprof.err"; exit 1; }
cp "$(find /tmp/prof_stats -name '*kernel_stats.csv')" "$out/bench_kernel_stats.csv"
python3 "$root/tools/roofline_from_trace.py" "$(find /tmp/prof_stats -name '*kernel_trace.csv')" > "$out/roofline_from_trace.txt"
head -8 "$out/roofline_from_trace.txt"
