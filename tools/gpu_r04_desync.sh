# CrossNet desynchronised-epilogue variant (13) vs the default (8): DCN tests
# under each, then the crossnet roofline lines, alternating
set -o pipefail
O=gpurun_out/r04desync
mkdir -p $O
for v in 13 8; do
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "variant $v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for v in 8 13 8 13; do
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet > $O/roof_$v.log 2>&1 || exit 1
  echo "== $v"; grep '"crossnet_layer_bf16\|with_lin\|crossnet_dx' $O/roof_$v.log | grep "B 65536"
done
