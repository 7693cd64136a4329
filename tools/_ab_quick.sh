set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_fit_graphed.py tests/test_eq_head.py tests/test_gpu_second_order.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/first.log 2>&1 || { tail -40 gpurun_out/first.log; exit 1; }
tail -1 gpurun_out/first.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -30 gpurun_out/r04f_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04f_bench.json'));s=d['secondary'];print('C2',d['ms_per_step'],'train',s['et_train_step']['graphed']['ms_per_step'],'C5',s['et_water_box_c5']['ms_per_step'],'C3',s['tensornet_c3']['ms_per_step'],'C4',s['et_spice_c4']['ms_per_step'],'scr',s['et_scripted_c2']['ms_per_step'],s['et_scripted_c2']['train_mode_ms_per_step'],s['et_scripted_c2']['eager_unscripted_ms_per_step'],'fit',s['et_fit_data_path']['ms_per_step'])"
timeout -k 10 300 bash tools/prof_train.sh r04f > /dev/null && grep -E "kernels per step|busy" gpurun_out/r04f_train_step_kernels.txt
