# rows backward: one-position fast path + narrow lane groups for dim <= 4
# (wide tables).  Rows / parity tests, then the DeepFM bf16 step and its
# kernel stats.  Tag $1.
set -o pipefail
T=${1:-wide}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_rows_sgd_fused.py tests/test_gpu_parity.py tests/test_gpu_modelzoo.py -x -q --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for F in "--bf16" "--bf16"; do  # after the emit change
  timeout -k 10 300 python tools/model_step.py --model deepfm --rows 10000000 --dim 64 $F --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "$F $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
MS_ARGS="--model deepfm --rows 10000000 --dim 64 --bf16" bash tools/gpu_dlrm_prof.sh $T/prof
