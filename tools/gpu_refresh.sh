# Round-2 refresh: kernel roofline survey, CrossNet roofline, model steps (configs[1..4] shapes + WDL)
set -o pipefail
mkdir -p gpurun_out/refresh
timeout -k 10 300 python -u tools/kernel_roofline.py > gpurun_out/refresh/kernel_roofline.log 2>&1 || { tail -5 gpurun_out/refresh/kernel_roofline.log; exit 1; }
grep '"op"' gpurun_out/refresh/kernel_roofline.log | cut -c1-160
for m in "dlrm --bf16" "dlrm" "deepfm --dim 64 --rows 10000000" "din" "dcn" "wdl"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python -u tools/model_step.py --model $m > gpurun_out/refresh/model_$tag.log 2>&1 || { tail -5 gpurun_out/refresh/model_$tag.log; exit 1; }
  tail -1 gpurun_out/refresh/model_$tag.log | cut -c1-200
done
