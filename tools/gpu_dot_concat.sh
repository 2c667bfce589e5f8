# DLRM --bf16: fused dot + concat + cast (DotConcatBf16) vs the composed path.
# Tests, then the model step both ways and its kernel stats.  Tag $1.
set -o pipefail
T=${1:-dcat}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_modelzoo.py tests/test_gpu_parity.py -x -q -k "dot or dlrm or DLRM or mlp or gemm" --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for V in 1 1; do  # fused dot-concat + head
  DR_DLRM_FUSE_DOT_CONCAT=$V timeout -k 10 300 python tools/model_step.py --model dlrm --bf16 --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "fuse=$V $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
bash tools/gpu_dlrm_prof.sh $T/prof_fused
for V in 1; do
  DR_DLRM_FUSE_HEAD=$V timeout -k 10 300 python tools/model_step.py --model dlrm --bf16 --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "fuse_head=$V $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
