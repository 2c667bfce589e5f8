# Round 6: churn = allocations or kernel launches?  And the runtime's graph
# packet capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) / kernarg placement.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06h}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/$n.log 2>&1 || { tail -5 gpurun_out/$T/$n.log; exit 1; }
  echo "$n: $(grep -E '^LOSSES' gpurun_out/$T/$n.log)"
}
run attn_alloc GPP_PIECE=attn GPP_CHURN=1 GPP_CHURN_KIND=alloc
run attn_launch GPP_PIECE=attn GPP_CHURN=1 GPP_CHURN_KIND=launch
run attn_fill_nopc GPP_PIECE=attn GPP_CHURN=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run fwdbwd_nopc GPP_PIECE=fwdbwd GPP_CHURN=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run full_nopc GPP_PIECE=full GPP_CHURN=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run attn_fill_devka GPP_PIECE=attn GPP_CHURN=1 HIP_FORCE_DEV_KERNARG=1
run attn_fill_hostka GPP_PIECE=attn GPP_CHURN=1 HIP_FORCE_DEV_KERNARG=0
