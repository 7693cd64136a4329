# Interleaved A/B of one environment switch on the headline C2 line (bench.py without secondary lines),
# plus the captured C2 step's kernel list under each value.
# usage: bash tools/c2_ab.sh <tag> VAR valueA valueB   (GPU box, repo root)
set -o pipefail
tag=$1; var=$2; a=$3; b=$4
mkdir -p gpurun_out
export TMPDIR=/tmp
root=$(pwd)
for rep in 1 2; do
  for v in "$a" "$b"; do
    env "$var=$v" timeout -k 10 240 python -u bench.py --no-secondary --no-roofline --no-cpu-baseline --no-ddp-train --no-pmc --steps 100 > "gpurun_out/${tag}_${v}_${rep}.json" 2> "gpurun_out/${tag}_${v}_${rep}.err" || { tail -20 "gpurun_out/${tag}_${v}_${rep}.err"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${tag}_${v}_${rep}.json'));print('$var=$v', d['ms_per_step'])"
  done
done
for v in "$a" "$b"; do
  rm -rf "/tmp/prof_${tag}_$v"
  (cd /tmp && env "$var=$v" timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "/tmp/prof_${tag}_$v" -o run -- python3 "$root/tools/graph_trace.py" et > /dev/null 2>&1) || { echo "trace failed"; exit 1; }
  python3 tools/trace_summary.py "$(find "/tmp/prof_${tag}_$v" -name '*kernel_trace.csv' | head -1)" > "gpurun_out/${tag}_${v}_kernels.txt"
  grep -E "kernels per step|busy" "gpurun_out/${tag}_${v}_kernels.txt"
done
