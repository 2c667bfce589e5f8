# TN weight-gradient GEMM (dr_gemm_tn_bf16): MLP tests, then the DLRM bf16
# step with it and with the transposes + NT path (DR_TOWER_TN_DW=0).  Tag $1.
set -o pipefail
T=${1:-tn}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for V in 1 0 1 0; do
  DR_TOWER_TN_DW=$V timeout -k 10 300 python tools/model_step.py --model dlrm --bf16 --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
  echo "tn=$V $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
done
bash tools/gpu_dlrm_prof.sh $T/prof
