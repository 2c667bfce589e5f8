# DeepFM --bf16 on the MFMA towers: tests, then the model step with the fused
# FM + bf16 dnn-input node and without it (DR_DEEPFM_FUSE_FM_COPY=0), and the
# kernel stats of the fused step.  Tag $1.
set -o pipefail
T=${1:-dfm}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_parity.py tests/test_gpu_modelzoo.py -x -q -k "deepfm or fm2 or mlp or model" --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for V in 1 0 1 0; do
  DR_DEEPFM_FUSE_HEAD=$V timeout -k 10 300 python tools/model_step.py --model deepfm --rows 10000000 --dim 64 --bf16 --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "fuse_head=$V $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
MS_ARGS="--model deepfm --rows 10000000 --dim 64 --bf16" bash tools/gpu_dlrm_prof.sh $T/prof
