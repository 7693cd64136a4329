# Run a subset of the -m gpu tests on the box: bash tools/gpu_tests.sh <log-name> <pytest args...>
set -o pipefail
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1
rc=$?
tail -40 gpurun_out/$name.log
exit $rc
