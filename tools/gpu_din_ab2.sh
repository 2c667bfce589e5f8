# DIN step: default build vs the ab build (measurement)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/din_tests.log 2>&1
rc=$?; tail -2 gpurun_out/din_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in base ab; do
  if [ $v = ab ]; then export DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so; else unset DEEPREC_AMD_LIB; fi
  echo -n "$v "; timeout -k 10 200 python3 tools/model_step.py --model din 2>/dev/null | tail -1 || exit 1
done; done
