# Round-2 measurement sweep: model training steps (configs[1..4] shapes) and
# the dominant kernel's PMC traffic (FETCH_SIZE / WRITE_SIZE in separate passes)
set -o pipefail
mkdir -p gpurun_out/models
for m in "dlrm --bf16" "dlrm" "deepfm --dim 64 --rows 10000000" "din" "dcn" "wdl"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python -u tools/model_step.py --model $m > gpurun_out/models/$tag.log 2>&1 || { tail -5 gpurun_out/models/$tag.log; exit 1; }
  tail -1 gpurun_out/models/$tag.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --no-graph --steps 2 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --no-deepfm"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/stats -o run -- python3 $B > gpurun_out/pmc_stats.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o run -- python3 $B > gpurun_out/pmc_write.log 2>&1 || exit 1
ls gpurun_out/pmc/*
