set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_periodic_oracle.py tests/test_gpu_capture.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
timeout -k 10 200 python -u tools/fep_time.py 50001 64 > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('default', 'fwd',d['fused_ms'],'bwd',d['fused_bwd_ms'],'unf',d['unfused_total_ms'],d['unfused_bwd_total_ms'],'err',d['max_rel_err_x'],max(d['bwd_max_rel_err'].values()))"
timeout -k 10 300 python -u tools/c5_time.py 50001 5 > gpurun_out/c5.json 2>&1 || { tail -5 gpurun_out/c5.json; exit 1; }
tail -1 gpurun_out/c5.json
