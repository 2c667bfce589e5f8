# Round 5, batch T: bisecting the DIN graph replays (tools/din_graph_probe.py):
# the same batch captured twice, with the EV update or the dense update left out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05t4}
mkdir -p gpurun_out/$T
for cfg in "0,0,1,1:" "0,0,1,1:ev" "0,0,1,1:dense"; do
  o=${cfg%%:*}; k=${cfg##*:}
  DGP_ORDER=$o DGP_SKIP=$k timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 > gpurun_out/$T/g_$k.log 2>&1
  echo "== order $o skip '$k' rc=$?"; grep -v Warning gpurun_out/$T/g_$k.log | grep -E "captured|differs|==|step [0-9]+:" | head -12
done
