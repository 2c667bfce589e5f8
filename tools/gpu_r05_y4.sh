# Round 5: the DIN weight-gradient pass with blocks rounded to whole 32-position
# chunks (753 blocks at DIN's cap) -- tests, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05y10}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py -k "fused_attention" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/din_prof.log | tail -1 || true
