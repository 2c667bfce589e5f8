# Round 6: the pool kernel alone in a graph (fixed inputs), and the pool in torch ops.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06m}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/$n.log 2>&1 || { tail -5 gpurun_out/$T/$n.log; exit 1; }
  echo "$n: $(grep -E '^LOSSES' gpurun_out/$T/$n.log)"
}
run const_pool GPP_PIECE=const_pool
run const_pool_sum GPP_PIECE=const_pool_sum
run attn_pool_torch GPP_PIECE=attn_pool_torch GPP_CHURN=1
