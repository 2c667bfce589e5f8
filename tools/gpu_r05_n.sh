# Round 5, batch N: the segment walk of long runs (DR_GRAD_SEG_SCAN) -- the
# rows / DIN parity tests, the DIN step with it on and off, and a kernel
# trace of the step.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05n}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_din.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in 4096 0 4096; do
  DR_GRAD_SEG_SCAN=$e timeout -k 10 300 python -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din$e.log 2>&1 || { tail -5 gpurun_out/$T/din$e.log; exit 1; }
  echo "din seg=$e: $(tail -1 gpurun_out/$T/din$e.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || { tail -5 gpurun_out/$T/din_prof.log; exit 1; }
echo "din under rocprof: $(tail -1 gpurun_out/$T/din_prof.log)"
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
grep -E "rows_seg|rows_serial" "$f" | cut -c1-200
