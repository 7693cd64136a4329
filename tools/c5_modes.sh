# C5 energy + forces under each edge-kernel variant (separate processes: the switches are read at import).
set -o pipefail
mkdir -p gpurun_out
for v in "0 off" "auto off" "auto rows" "auto fused" "auto lazy"; do
  set -- $v
  TMDNET_FEP=$1 TMDNET_FEP_BWD=$2 timeout -k 10 300 python -u tools/c5_time.py 50001 5 2>&1 | grep -v amdgpu.ids || exit 1
done
