# DeepFM --bf16 on the MFMA towers: test, then the model step fp32 vs bf16.  Tag $1.
set -o pipefail
T=${1:-dfm}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q -k "deepfm" --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for F in "" "--bf16" "" "--bf16"; do
  timeout -k 10 300 python tools/model_step.py --model deepfm --rows 10000000 --dim 64 $F --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "$F $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
