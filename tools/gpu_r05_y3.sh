# Round 5: the DIN weight-gradient pass on the matrix cores, 32- vs 64-position
# chunks with the one-list staging, vs the library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05y7}
mkdir -p gpurun_out/$T
for c in 32 64; do
  DR_DIN_WGRAD_CH=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py -k "fused_attention" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests_$c.log 2>&1
  rc=$?; echo "CH=$c: $(tail -1 gpurun_out/$T/tests_$c.log)"; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests_$c.log | head -10
  [ $rc -ne 0 ] && exit $rc
done
for e in "DR_DIN_WGRAD=hand" "DR_DIN_WGRAD=hand DR_DIN_WGRAD_BLOCKS=512" "DR_DIN_WGRAD=hand DR_DIN_WGRAD_BLOCKS=1024" "DR_DIN_WGRAD=lib"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/$T/din.log | grep -o '"ms_per_step": [0-9.]*')"
done
for c in 512 768; do
  DR_DIN_WGRAD=hand DR_DIN_WGRAD_BLOCKS=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof$c -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof$c.log 2>&1 || exit 1
done
echo profiled
