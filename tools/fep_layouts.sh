set -o pipefail
for lay in plain strided; do
  FEP_TIME_QKV=$lay timeout -k 10 300 python -u tools/fep_time.py 50001 64 2>&1 | grep -v amdgpu.ids | sed "s/^/$lay: /" || exit 1
done
