set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tn_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tnk.log 2>&1 || { tail -40 gpurun_out/tnk.log; exit 1; }
tail -1 gpurun_out/tnk.log
for s in 1 4; do
  TMDNET_ET_S=$s timeout -k 10 200 python -u tools/pair_probe.py > gpurun_out/pp.json 2>&1 || { tail -5 gpurun_out/pp.json; exit 1; }
  tail -1 gpurun_out/pp.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/r04e_gputest.log 2>&1 || { tail -40 gpurun_out/r04e_gputest.log; exit 1; }
tail -1 gpurun_out/r04e_gputest.log
timeout -k 10 300 bash tools/prof_train.sh r04 > /dev/null 2>&1 || { echo "prof_train failed"; tail -5 gpurun_out/prof_train.err; exit 1; }
head -3 gpurun_out/r04_train_step_kernels.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { tail -30 gpurun_out/r04e_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04e_bench.json'));s=d['secondary'];print('C2',d['ms_per_step'],'train',s['et_train_step']['graphed']['ms_per_step'],'C5',s['et_water_box_c5']['ms_per_step'],'C3',s['tensornet_c3']['ms_per_step'],'C4',s['et_spice_c4']['ms_per_step'],'scr',s['et_scripted_c2']['ms_per_step']);print(json.dumps(d['roofline']['fused_projection']))"
export TMPDIR=/tmp
R=$(pwd)
cd /tmp && rm -rf /tmp/prof_tn
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- python3 $R/tools/graph_trace.py tn > /dev/null 2>&1
python3 $R/tools/trace_summary.py "$(find /tmp/prof_tn -name '*kernel_trace.csv' | head -1)" > $R/gpurun_out/r04e_tn_c3_kernels.txt
grep -E "kernels per step|busy" $R/gpurun_out/r04e_tn_c3_kernels.txt
