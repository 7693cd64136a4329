# A/B of the force-pass recording (TMDNET_ET_RECORD) on the captured training step: kernel traces of
# one replay each (GPU box, repo root): bash tools/ab_record.sh <tag>
set -e -o pipefail
mkdir -p gpurun_out
TMDNET_ET_RECORD=0 bash tools/prof_train.sh $1_rec0 > /dev/null
TMDNET_ET_RECORD=1 bash tools/prof_train.sh $1_rec1 > /dev/null
head -2 gpurun_out/$1_rec0_train_step_kernels.txt gpurun_out/$1_rec1_train_step_kernels.txt
