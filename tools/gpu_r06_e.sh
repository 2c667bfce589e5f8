# Round 6: graph + allocator churn by piece; the DIN switches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06e}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/$n.log 2>&1 || { tail -5 gpurun_out/$T/$n.log; exit 1; }
  echo "$n: $(grep -E '^LOSSES' gpurun_out/$T/$n.log)"
}
run lookup_c GPP_PIECE=lookup GPP_CHURN=1
run attn_c GPP_PIECE=attn GPP_CHURN=1
run fwd_nofused_c GPP_PIECE=fwd GPP_CHURN=1 DR_DIN_FUSED_ATTENTION=0
run fwdbwd_nofused GPP_PIECE=fwdbwd GPP_CHURN=0 DR_DIN_FUSED_ATTENTION=0
run fwd_twolookups_c GPP_PIECE=fwd GPP_CHURN=1 DR_DIN_ONE_ITEM_LOOKUP=0
run fwdbwd_noside GPP_PIECE=fwdbwd GPP_CHURN=0 DR_ROWS_SIDE_STREAM=0
run fwd_b512_c GPP_PIECE=fwd GPP_CHURN=1 GPP_BATCH=512
