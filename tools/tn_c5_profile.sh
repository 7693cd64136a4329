# C5 TensorNet arm (tools/tn_c5_time.py) under rocprofv3 --kernel-trace --stats: the per-kernel breakdown of
# eager energy + force evaluations.  usage: bash tools/tn_c5_profile.sh <tag> [n_atoms] [static 0|1]  (GPU box)
set -o pipefail
tag=${1:-tnc5}
n=${2:-50001}
st=${3:-1}
mkdir -p gpurun_out
export TMPDIR=/tmp
root=$(pwd)
rm -rf "/tmp/prof_$tag"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$tag" -o run -- python3 "$root/tools/tn_c5_time.py" "$n" 5 "$st" > "$root/gpurun_out/${tag}_tnc5time.json" 2> "$root/gpurun_out/${tag}_tnc5time.err" || { tail -20 "$root/gpurun_out/${tag}_tnc5time.err"; exit 1; }
cp "$(find "/tmp/prof_$tag" -name '*kernel_stats.csv' | head -1)" "$root/gpurun_out/${tag}_tn_c5_kernel_stats.csv"
cat "$root/gpurun_out/${tag}_tnc5time.json"
