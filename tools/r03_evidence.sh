#!/bin/bash
# Round-3 evidence refresh, part 2 (part 1 = tools/refresh_profiles.sh r03): the captured training
# step's kernel list and the one-GPU rehearsal of the multi-rank bench path (2 ranks on cuda:0 over
# gloo, TMDNET_BENCH_REHEARSAL).  GPU box, repo root: bash tools/r03_evidence.sh
set -e -o pipefail
mkdir -p gpurun_out
bash tools/prof_train.sh r03 > /dev/null
head -3 gpurun_out/r03_train_step_kernels.txt
TMDNET_BENCH_REHEARSAL=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-pmc > gpurun_out/r03_bench_rehearsal_2ranks.json 2> gpurun_out/r03_bench_rehearsal.err
python -c "import json;d=json.loads(open('gpurun_out/r03_bench_rehearsal_2ranks.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d['ms_per_step'],d.get('ddp_train',{}).get('ms_per_step'))"
