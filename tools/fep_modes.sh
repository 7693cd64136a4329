# Fused-projection forward: the kernel variants (TMDNET_FEP_MODE) timed on the C5 water box.
set -o pipefail
mkdir -p gpurun_out
for m in 2; do
  TMDNET_FEP_MODE=$m timeout -k 10 300 python -u tools/fep_time.py 50001 ${1:-64} 2>&1 | grep -v amdgpu.ids | sed "s/^/mode $m: /" || exit 1
done
