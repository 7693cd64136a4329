# A/B of an environment switch on the captured training step: kernel traces of one replay per value
# (GPU box, repo root): bash tools/ab_env.sh <tag> <VAR> <value>...
set -e -o pipefail
mkdir -p gpurun_out
tag=$1; var=$2; shift 2
for v in "$@"; do
  env "$var=$v" bash tools/prof_train.sh ${tag}_$v > /dev/null
  echo "$var=$v: $(head -2 gpurun_out/${tag}_${v}_train_step_kernels.txt | tr '\n' ' ')"
done
