# CrossNet variant check: the dcn/crossnet tests under DR_CROSSNET_VARIANT=$1,
# then the layer roofline for each variant named in $@
set -o pipefail
mkdir -p gpurun_out
V=$1
DR_CROSSNET_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py tests/test_gpu_parity.py -k "crossnet or dcn" -x -q --timeout 120 --timeout-method thread > gpurun_out/crossnet_tests_v$V.log 2>&1
rc=$?; tail -4 gpurun_out/crossnet_tests_v$V.log; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  echo "== variant $v"
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet 2>/dev/null | grep '"crossnet_\|torch_' || exit 1
done
