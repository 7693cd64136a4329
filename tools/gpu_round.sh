# One GPU round trip: the -m gpu suite, the capture tests on the index-checking debug build, the
# default bench line.  Usage on the box: bash tools/gpu_round.sh [skip-tests]
set -o pipefail
mkdir -p gpurun_out
if [ "$1" != "skip-tests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1 || { tail -30 gpurun_out/r03_gputest.log; exit 1; }
tail -1 gpurun_out/r03_gputest.log
fi
TMDNET_LIB=debug timeout -k 10 300 python -u -m pytest tests/test_gpu_capture.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r03_gputest_debug.log; exit 1; }
tail -1 gpurun_out/r03_gputest_debug.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -30 gpurun_out/r03_bench.err; exit 1; }
cat gpurun_out/r03_bench.json
