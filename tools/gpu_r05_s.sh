# Round 5, batch S: the fused-SGD tests (side-stream aware), the DIN merged
# lookup A/B, and the DIN step captured as hipGraphs.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05s}
mkdir -p gpurun_out/$T
for e in ${DIN_AB:-}; do
  DR_DIN_ONE_ITEM_LOOKUP=$e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din$e.log 2>&1 || { tail -5 gpurun_out/$T/din$e.log; exit 1; }
  echo "din one_item_lookup=$e: $(tail -1 gpurun_out/$T/din$e.log)"
done
timeout -k 10 300 python -u tools/din_graph_probe.py --steps 20 > gpurun_out/$T/graph.log 2>&1; rc=$?
[ $rc -eq 0 ] && { timeout -k 10 400 python -u bench.py --cpu-seconds 0 --steps 3 --warmup 1 --train-steps 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --din-steps 20 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; rc=$?; grep "din leg" gpurun_out/$T/bench.err | cut -c1-600; }
tail -8 gpurun_out/$T/graph.log
exit $rc
