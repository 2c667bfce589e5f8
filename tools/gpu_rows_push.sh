# Block-aggregated worklist pushes: rows / fused-SGD / parity tests, then the
# WDL and DeepFM bf16 steps and the bench's train step.  Tag $1.
set -o pipefail
T=${1:-push}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_wdl.py tests/test_gpu_din.py -x -q --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for M in wdl wdl; do
  A="--model $M --bf16"; [ $M = deepfm ] && A="$A --rows 10000000 --dim 64"
  timeout -k 10 300 python tools/model_step.py $A --steps 8 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "$M $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
timeout -k 10 300 python tools/model_step.py --model din --steps 8 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
echo "din $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
MS_ARGS="--model wdl --bf16" bash tools/gpu_dlrm_prof.sh $T/prof
