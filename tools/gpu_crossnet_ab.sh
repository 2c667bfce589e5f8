# CrossNet A/B (measurement): default build vs the ab build, layer roofline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crossnet_tests.log 2>&1
rc=$?; tail -3 gpurun_out/crossnet_tests.log; [ $rc -ne 0 ] && exit $rc
for v in base ab; do
  if [ $v = ab ]; then export DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so; else unset DEEPREC_AMD_LIB; fi
  echo "== $v"
  timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet 2>/dev/null | grep '"crossnet_layer_bf16\|with_lin' || exit 1
done
