# Round 5, batch V: DIN graph divergence -- zero_grad outside the capture;
# also the whole-graph with only the EV update.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05v2}
mkdir -p gpurun_out/$T
run() {
  env "$@" DGP_ORDER=0,0,1,1 timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 > gpurun_out/$T/g.log 2>&1
  echo "== $* rc=$?"; grep -v Warning gpurun_out/$T/g.log | grep -E "differs: loss|eager ==|param .* differs" | head -3
}
run DGP_ZERO_OUTSIDE=1
run DGP_ZERO_OUTSIDE=1 DGP_SKIP=ev
