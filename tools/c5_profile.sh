# C5 water-box energy + forces (tools/c5_time.py) under rocprofv3 --kernel-trace --stats: the per-kernel
# breakdown of one eager evaluation.  usage: bash tools/c5_profile.sh <tag> [n_atoms]   (GPU box, repo root)
set -o pipefail
tag=${1:-c5}
n=${2:-50001}
mkdir -p gpurun_out
export TMPDIR=/tmp
root=$(pwd)
rm -rf "/tmp/prof_$tag"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$tag" -o run -- python3 "$root/tools/c5_time.py" "$n" 5 > "$root/gpurun_out/${tag}_c5time.json" 2> "$root/gpurun_out/${tag}_c5time.err" || { tail -20 "$root/gpurun_out/${tag}_c5time.err"; exit 1; }
cp "$(find "/tmp/prof_$tag" -name '*kernel_stats.csv' | head -1)" "$root/gpurun_out/${tag}_c5_kernel_stats.csv"
cat "$root/gpurun_out/${tag}_c5time.json"
