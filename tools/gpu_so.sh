set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_second_order.py tests/test_gpu_parity.py -k "adjoint or second_order or double or train or graphed or fit or force" > gpurun_out/r02_so_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r02_so_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-roofline --no-pmc --steps 20 --warmup 5 > gpurun_out/r02_bench_so.json 2> gpurun_out/r02_bench_so.err || { tail -30 gpurun_out/r02_bench_so.err; exit 1; }
cat gpurun_out/r02_bench_so.json
