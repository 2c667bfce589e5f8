# Round 6: DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 against the original failures --
# the 4-graph churned replays and the twin model's eager steps interleaved
# with the replays (round 5's symptom) -- and the graph step's time with it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06k}
mkdir -p gpurun_out/$T
export DGP_FILE=/tmp/dgp_eager.pt
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 8 --batch 4096 > gpurun_out/$T/eager.log 2>&1 || { tail -5 gpurun_out/$T/eager.log; exit 1; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 8 > gpurun_out/$T/churn_nopc.log 2>&1 || { tail -5 gpurun_out/$T/churn_nopc.log; exit 1; }
grep -E "replay|all replays" gpurun_out/$T/churn_nopc.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u tools/din_graph_probe.py --steps 12 --batch 4096 > gpurun_out/$T/twin_nopc.log 2>&1; rc=$?
grep -E "differs|eager == graph|din_step|storage" gpurun_out/$T/twin_nopc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/din_graph_probe.py --steps 12 --batch 4096 > gpurun_out/$T/twin_pc.log 2>&1; rc=$?
grep -E "differs|eager == graph|din_step" gpurun_out/$T/twin_pc.log; exit 0
