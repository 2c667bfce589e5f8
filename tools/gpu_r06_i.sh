# Round 6: which kernel of the attention trips the graph packet capture?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06i}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/$n.log 2>&1 || { tail -5 gpurun_out/$T/$n.log; exit 1; }
  echo "$n: $(grep -E '^LOSSES' gpurun_out/$T/$n.log)"
}
run attn_mlp GPP_PIECE=attn_mlp GPP_CHURN=1
run attn_pool GPP_PIECE=attn_pool GPP_CHURN=1
run attn_mlp_b1024 GPP_PIECE=attn_mlp GPP_CHURN=1 GPP_BATCH=1024
run attn_mlp_b2048 GPP_PIECE=attn_mlp GPP_CHURN=1 GPP_BATCH=2048
