set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_second_order.py -k "tn_gemm or tn " -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tn_tests.log 2>&1 || { tail -40 gpurun_out/tn_tests.log; exit 1; }
tail -1 gpurun_out/tn_tests.log
timeout -k 10 300 python -u tools/tn_time.py > gpurun_out/tn_time.txt 2>&1 || { tail -20 gpurun_out/tn_time.txt; exit 1; }
cat gpurun_out/tn_time.txt
TMDNET_TN_V=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_train_parity.py tests/test_eq_head.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tn_parity.log 2>&1 || { tail -40 gpurun_out/tn_parity.log; exit 1; }
tail -1 gpurun_out/tn_parity.log
TMDNET_TN_V=4 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/tn4_bench.json 2> gpurun_out/tn4_bench.err || { tail -30 gpurun_out/tn4_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tn4_bench.json'));s=d['secondary'];print('TN_V=4: C2',d['ms_per_step'],'train',s['et_train_step']['graphed']['ms_per_step'],'fit',s['et_fit_data_path']['ms_per_step'])"
