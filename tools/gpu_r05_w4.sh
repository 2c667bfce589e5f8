# Round 5: one-wave-per-SIMD CrossNet kernel (crossnet_w4_kernel) -- the
# crossnet / dcn tests under DR_CROSSNET_VARIANT 14 and 16, then the layer
# roofline for 8 (the 8-phase default), 14, 15 (14's loop alone), 16, 17.
set -o pipefail
T=${1:-r05w4}
mkdir -p gpurun_out/$T
for v in 14 16; do
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests_v$v.log 2>&1
  rc=$?; echo "tests v$v: $(tail -1 gpurun_out/$T/tests_v$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for v in 8 14 15 16 17 8 16; do
  echo "== variant $v"
  DR_CROSSNET_VARIANT=$v timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet > gpurun_out/$T/roof_v$v.log 2>&1 || { tail -5 gpurun_out/$T/roof_v$v.log; exit 1; }
  grep '"crossnet_\|torch_' gpurun_out/$T/roof_v$v.log | cut -c1-200
done
