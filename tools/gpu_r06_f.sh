# Round 6: graph + churn by piece, with the copy engines off (HSA_ENABLE_SDMA=0:
# captured memcpy / memset nodes run as blit kernels instead of SDMA).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06f}
mkdir -p gpurun_out/$T
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/$n.log 2>&1 || { tail -5 gpurun_out/$T/$n.log; exit 1; }
  echo "$n: $(grep -E '^LOSSES' gpurun_out/$T/$n.log)"
}
run attn_c_nosdma GPP_PIECE=attn GPP_CHURN=1 HSA_ENABLE_SDMA=0
run fwdbwd_nosdma GPP_PIECE=fwdbwd GPP_CHURN=0 HSA_ENABLE_SDMA=0
run full_c_nosdma GPP_PIECE=full GPP_CHURN=1 HSA_ENABLE_SDMA=0
run full_nosdma GPP_PIECE=full GPP_CHURN=0 HSA_ENABLE_SDMA=0
