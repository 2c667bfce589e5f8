# Round 5: the DIN weight-gradient pass at 3 waves per SIMD (launch bounds),
# 32-position chunks (10 loads in flight: one round trip) vs 24 -- tests and
# kernel stats each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05y11}
mkdir -p gpurun_out/$T
for c in 32 24; do
  DR_DIN_WGRAD_CH=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py -k "fused_attention" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests$c.log 2>&1
  rc=$?; echo "CH=$c: $(tail -1 gpurun_out/$T/tests$c.log)"; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests$c.log | head -10
  [ $rc -ne 0 ] && exit $rc
  DR_DIN_WGRAD_CH=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof$c -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof$c.log 2>&1 || exit 1
done
echo profiled
