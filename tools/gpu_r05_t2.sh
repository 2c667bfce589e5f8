# Round 5: bisecting the twin-model interference with DIN graph replays.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05tw}
mkdir -p gpurun_out/$T
for op in none fwd lookup fwdbwd dense apply; do
  DGP_TWIN_OP=$op timeout -k 10 200 python -u tools/din_graph_probe.py --steps 2 > gpurun_out/$T/$op.log 2>&1
  echo "== $op rc=$?"; grep -E "twin op" gpurun_out/$T/$op.log | head -2
done
