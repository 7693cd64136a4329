# Second-order iteration on the box: the second-order / head / training GPU tests, the bench line
# (no CPU baseline / PMC), then the kernel trace of one captured training-step replay.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02_so}
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_second_order.py tests/test_eq_head.py tests/test_gpu_parity.py -k "adjoint or second_order or double or train or graphed or fit or force or head or neighbor_embedding or tn_gemm" > gpurun_out/${tag}_tests.log 2>&1; rc=$?
tail -5 gpurun_out/${tag}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-roofline --no-pmc --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));s=d['secondary'];print('C2',d['ms_per_step'],'train',s['et_train_step']['ms_per_step'],s['et_train_step']['graphed']['ms_per_step'],'ddp',d['ddp_train']['ms_per_step'])"
bash tools/prof_train.sh $tag | head -40
