# Round 5, batch Q: DIN with the target and history items in one lookup
# (DR_DIN_ONE_ITEM_LOOKUP) -- the DIN tests, then the step with it on / off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05q}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_configs.py -k "din or config3" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in 1 0 1 0; do
  DR_DIN_ONE_ITEM_LOOKUP=$e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din$e.log 2>&1 || { tail -5 gpurun_out/$T/din$e.log; exit 1; }
  echo "din one_item_lookup=$e: $(tail -1 gpurun_out/$T/din$e.log)"
done
