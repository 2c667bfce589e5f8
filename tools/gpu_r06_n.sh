# Round 6: memset node -> counting kernel in a replayed graph (torch's
# multi-block reduction pattern), with and without graph packet capture.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06n}
mkdir -p gpurun_out/$T
for m in memset memsetd32; do
  timeout -k 10 60 ./tools/graph_memset_probe $m | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 60 ./tools/graph_memset_probe $m | sed 's/^/[nopc] /' | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
done
exit 0
