# Round 5: the DIN weight-gradient pass on the matrix cores vs VALU vs library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05y4}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py -k "fused_attention" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
for e in "DR_DIN_WGRAD=hand" "DR_DIN_WGRAD=lib" "DR_DIN_WGRAD=hand DR_DIN_WGRAD_VALU=1"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/$T/din.log | grep -o '"ms_per_step": [0-9.]*')"
done
DR_DIN_WGRAD=hand timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
echo profiled
