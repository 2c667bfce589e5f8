# Round 6: ordering / coherence of replayed graph nodes (standalone HIP probe).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06l}
mkdir -p gpurun_out/$T
for m in plain memset memcpy; do
  timeout -k 10 60 ./tools/graph_order_probe $m | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 60 ./tools/graph_order_probe $m | sed 's/^/[nopc] /' | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
done
exit 0
