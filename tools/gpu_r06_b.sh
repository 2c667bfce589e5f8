# Round 6: the hipGraph corruption, bisected -- what is non-finite after the
# first churned replay; zero vs NaN churn; large-pool churn; rocBLAS instead
# of hipBLASLt (eager reference rerun with the same library).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06b}
mkdir -p gpurun_out/$T
export DGP_FILE=/tmp/dgp_eager.pt
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 --batch 4096 > gpurun_out/$T/eager.log 2>&1 || { tail -5 gpurun_out/$T/eager.log; exit 1; }
for c in small small0 large; do
  GMP_REPORT=1 GMP_CHURN=$c timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 4 > gpurun_out/$T/churn_$c.log 2>&1 || { tail -5 gpurun_out/$T/churn_$c.log; exit 1; }
  grep -E "replay|non-finite" gpurun_out/$T/churn_$c.log
done
export DGP_FILE=/tmp/dgp_eager_rocblas.pt GMP_BLAS=rocblas
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 --batch 4096 > gpurun_out/$T/eager_rocblas.log 2>&1 || { tail -5 gpurun_out/$T/eager_rocblas.log; exit 1; }
GMP_REPORT=1 GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 4 > gpurun_out/$T/churn_rocblas.log 2>&1 || { tail -5 gpurun_out/$T/churn_rocblas.log; exit 1; }
grep -E "replay|non-finite" gpurun_out/$T/churn_rocblas.log
