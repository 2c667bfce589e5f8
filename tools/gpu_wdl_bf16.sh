# WDL --bf16 on the MFMA tower + bf16 head: tests, then the model step fp32
# vs --bf16 (B = 65 536) and the kernel stats of the bf16 step.  Tag $1.
set -o pipefail
T=${1:-wdl}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_wdl.py -x -q -k "wdl" --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for F in "--bf16" "--bf16"; do
  timeout -k 10 300 python tools/model_step.py --model wdl $F --steps 6 --warmup 2 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "$F $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
MS_ARGS="--model wdl --bf16" bash tools/gpu_dlrm_prof.sh $T/prof
