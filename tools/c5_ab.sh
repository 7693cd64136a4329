# C5 energy + forces A/B of one environment switch, interleaved runs in separate processes.
# usage: bash tools/c5_ab.sh VAR "valA" "valB" [rounds]
set -o pipefail
mkdir -p gpurun_out
var=$1; a=$2; b=$3; n=${4:-2}
for i in $(seq $n); do
  for v in "$a" "$b"; do
    env $var=$v timeout -k 10 300 python -u tools/c5_time.py 50001 5 2>/dev/null | sed "s/^/$var=$v /" || exit 1
  done
done
