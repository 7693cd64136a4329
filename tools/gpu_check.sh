# Full -m gpu suite, a bench line without the CPU / PMC legs, and the kernel list of one captured C2
# energy+force replay: bash tools/gpu_check.sh <tag> [first-test-file]   (GPU box, repo root)
# The optional first file runs alone before the suite (a test just fixed: stop there if it fails).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-chk}
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest "$2" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_first.log 2>&1 || { tail -40 gpurun_out/${tag}_first.log; exit 1; }
  tail -1 gpurun_out/${tag}_first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gputest.log 2>&1 || { tail -40 gpurun_out/${tag}_gputest.log; exit 1; }
tail -1 gpurun_out/${tag}_gputest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));s=d['secondary'];print('C2',d['ms_per_step'],'train',s['et_train_step']['graphed']['ms_per_step'],'ddp',d['ddp_train']['ms_per_step'],'C5',s['et_water_box_c5']['ms_per_step'],'C3',s['tensornet_c3']['ms_per_step'],'C4',s['et_spice_c4']['ms_per_step'])"
export TMPDIR=/tmp
root=$(pwd)
cd /tmp && rm -rf /tmp/prof_et_chk
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_et_chk -o run -- python3 "$root/tools/graph_trace.py" et > /dev/null 2>&1
python3 "$root/tools/trace_summary.py" "$(find /tmp/prof_et_chk -name '*kernel_trace.csv' | head -1)" > "$root/gpurun_out/${tag}_et_c2_kernels.txt"
grep -E "kernels per step|busy" "$root/gpurun_out/${tag}_et_c2_kernels.txt"
