# Round 5, batch R: KV Adam on device beta powers (every Adam test), the DIN
# merged lookup A/B, and the DIN step captured as hipGraphs (bit-equal to
# eager, timed).  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05r}
mkdir -p gpurun_out/$T
FILES=$(grep -ln "AdamOptimizer\|din" tests/test_gpu_*.py | tr '\n' ' ')
timeout -k 10 900 python -u -m pytest $FILES -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in 1 0; do
  DR_DIN_ONE_ITEM_LOOKUP=$e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din$e.log 2>&1 || { tail -5 gpurun_out/$T/din$e.log; exit 1; }
  echo "din one_item_lookup=$e: $(tail -1 gpurun_out/$T/din$e.log)"
done
timeout -k 10 300 python -u tools/din_graph_probe.py --steps 20 > gpurun_out/$T/graph.log 2>&1; rc=$?
tail -6 gpurun_out/$T/graph.log
exit $rc
