# Kernel-time profile of model training steps: tools/model_step.py under
# rocprofv3 --kernel-trace --stats for each model spec in $@ (e.g. "dlrm --bf16")
set -o pipefail
mkdir -p gpurun_out/mprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in "$@"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mprof/$tag -o run -- python3 tools/model_step.py --model $m --steps 6 --warmup 3 > gpurun_out/mprof/$tag.log 2>&1 || { tail -5 gpurun_out/mprof/$tag.log; exit 1; }
  tail -1 gpurun_out/mprof/$tag.log
done
