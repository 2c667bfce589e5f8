# Round 5, batch U: DIN graph divergence, more bisection (dense update only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05u2}
mkdir -p gpurun_out/$T
run() {
  env "$@" DGP_ORDER=0,0,1,1 DGP_SKIP=ev timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 > gpurun_out/$T/g.log 2>&1
  echo "== $* rc=$?"; grep -v Warning gpurun_out/$T/g.log | grep -E "differs: loss|==|param .* differs" | head -4
}
run DR_DIN_FUSED_ATTENTION=0
run DR_DIN_ONE_ITEM_LOOKUP=0
run DR_CROSSNET_DW=lib
