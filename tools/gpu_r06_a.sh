# Round 6: the hipGraph corruption -- default-pool blocks freed inside a
# capture (allocator history), zero-poisoned free blocks and small-pool
# churn before each replay, every replay compared with the eager run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06a}
mkdir -p gpurun_out/$T
export DGP_FILE=/tmp/dgp_eager.pt
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 8 --batch 4096 > gpurun_out/$T/eager.log 2>&1 || { tail -5 gpurun_out/$T/eager.log; exit 1; }
for m in none default graph; do
  GMP_POISON=$m timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 8 > gpurun_out/$T/poison_$m.log 2>&1 || { tail -5 gpurun_out/$T/poison_$m.log; exit 1; }
  tail -9 gpurun_out/$T/poison_$m.log
done
GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 8 > gpurun_out/$T/churn.log 2>&1 || { tail -5 gpurun_out/$T/churn.log; exit 1; }
tail -9 gpurun_out/$T/churn.log
