# Round-4 probe 1 (GPU box, repo root): C5 kernel trace (fused path default), fused-kernel PMC passes,
# host profile of the eager / scripted C2 evaluation.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/host_profile.py both 40 > gpurun_out/r04_host_profile.txt 2>&1 || { tail -20 gpurun_out/r04_host_profile.txt; exit 1; }
grep "==" gpurun_out/r04_host_profile.txt
cd /tmp && rm -rf /tmp/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c5 -o run -- python3 $R/tools/c5_time.py 50001 3 > $R/gpurun_out/r04_c5_time.json 2>&1 || { tail -20 $R/gpurun_out/r04_c5_time.json; exit 1; }
cp $(find /tmp/prof_c5 -name '*kernel_stats.csv' | head -1) $R/gpurun_out/r04_c5_kernel_stats.csv
tail -1 $R/gpurun_out/r04_c5_time.json
cd $R
timeout -k 10 400 bash tools/fep_pmc.sh fused_only r04fwd > /dev/null 2>&1 || echo "fwd pmc failed"
timeout -k 10 400 bash tools/fep_pmc.sh fused_bwd_only r04bwd > /dev/null 2>&1 || echo "bwd pmc failed"
ls gpurun_out/r04fwd_pmc gpurun_out/r04bwd_pmc
