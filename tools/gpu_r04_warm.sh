# CrossNet epilogue warming: DCN tests, roofline lines (B = 65 536) x 2
set -o pipefail
O=gpurun_out/r04warm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py tests/test_gpu_configs.py -k "crossnet or dcn or cross" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet > $O/roof_$i.log 2>&1 || exit 1
  grep "B 65536" $O/roof_$i.log | grep '"crossnet_layer_bf16\|with_lin\|composed\|crossnet_dx\|addmm_dx'
done
