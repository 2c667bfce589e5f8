# CrossNet: tests (incl. repeated-launch determinism), then the layer roofline
# for the default kernel and the variants named in $@ (DR_CROSSNET_VARIANT)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py tests/test_gpu_parity.py -k "crossnet or dcn" -x -q --timeout 120 --timeout-method thread > gpurun_out/crossnet_tests.log 2>&1
rc=$?; tail -4 gpurun_out/crossnet_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet > gpurun_out/crossnet_default.log 2>&1
rc=$?; cat gpurun_out/crossnet_default.log; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  echo "== variant $v"
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet 2>/dev/null | grep '"crossnet_' || exit 1
done
