# A/B of two library builds on the training-step probe (measurement only)
set -o pipefail
mkdir -p gpurun_out
AB=deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base ab; do
    if [ $v = ab ]; then export DEEPREC_AMD_LIB=$PWD/$AB; else unset DEEPREC_AMD_LIB; fi
    echo -n "$v: "
    timeout -k 10 200 python -u tools/train_probe.py --graph "$@" 2>/dev/null | tail -1 || exit $?
  done
done
