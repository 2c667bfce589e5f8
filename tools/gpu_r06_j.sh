# Round 6: dynamic LDS under hipGraph replay (standalone HIP probe), with and
# without the runtime's graph packet capture.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06j}
mkdir -p gpurun_out/$T
for w in 612 4096 16384; do
  timeout -k 10 60 ./tools/dynlds_graph_probe $w 4096 | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 60 ./tools/dynlds_graph_probe $w 4096 | sed 's/^/[nopc] /' | tee -a gpurun_out/$T/probe.log; rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit $rc
done
exit 0
