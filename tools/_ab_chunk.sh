set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_second_order.py tests/test_eq_head.py tests/test_gpu_fit_graphed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/first.log 2>&1 || { tail -40 gpurun_out/first.log; exit 1; }
tail -1 gpurun_out/first.log
timeout -k 10 300 python -u tools/tn_time.py > gpurun_out/tn_time.txt 2>&1 || { tail -20 gpurun_out/tn_time.txt; exit 1; }
cat gpurun_out/tn_time.txt
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/r04f_gputest.log 2>&1 || { tail -40 gpurun_out/r04f_gputest.log; exit 1; }
tail -1 gpurun_out/r04f_gputest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -30 gpurun_out/r04f_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04f_bench.json'));s=d['secondary'];print('C2',d['ms_per_step'],'train',s['et_train_step']['graphed']['ms_per_step'],'C5',s['et_water_box_c5']['ms_per_step'],'C3',s['tensornet_c3']['ms_per_step'],'C4',s['et_spice_c4']['ms_per_step'],'scr',s['et_scripted_c2']['ms_per_step'],s['et_scripted_c2']['train_mode_ms_per_step'],s['et_scripted_c2']['eager_unscripted_ms_per_step'],'fit',s['et_fit_data_path']['ms_per_step'])"
export TMPDIR=/tmp
R=$(pwd)
cd /tmp && rm -rf /tmp/prof_tn /tmp/prof_et
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tn -o run -- python3 $R/tools/graph_trace.py tn > /dev/null 2>&1
python3 $R/tools/trace_summary.py "$(find /tmp/prof_tn -name '*kernel_trace.csv')" > $R/gpurun_out/r04f_tn_c3_kernels.txt
grep -E "kernels per step|busy" $R/gpurun_out/r04f_tn_c3_kernels.txt
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_et -o run -- python3 $R/tools/graph_trace.py et > /dev/null 2>&1
python3 $R/tools/trace_summary.py "$(find /tmp/prof_et -name '*kernel_trace.csv')" > $R/gpurun_out/r04f_et_c2_kernels.txt
grep -E "kernels per step|busy" $R/gpurun_out/r04f_et_c2_kernels.txt
cd $R
timeout -k 10 300 bash tools/prof_train.sh r04f > /dev/null && grep -E "kernels per step|busy" gpurun_out/r04f_train_step_kernels.txt
