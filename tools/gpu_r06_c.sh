# Round 6: the hipGraph corruption, bisected further -- no empty_cache at
# capture; graph 1 replayed first; torch's BLAS = hipBLAS (rocBLAS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06c}
mkdir -p gpurun_out/$T
export DGP_FILE=/tmp/dgp_eager.pt
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 --batch 4096 > gpurun_out/$T/eager.log 2>&1 || { tail -5 gpurun_out/$T/eager.log; exit 1; }
GMP_NO_EMPTY_CACHE=1 GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 4 > gpurun_out/$T/noempty.log 2>&1 || { tail -5 gpurun_out/$T/noempty.log; exit 1; }
echo "== no empty_cache"; grep -E "replay" gpurun_out/$T/noempty.log
GMP_REPLAY=1,1 GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 2 > gpurun_out/$T/g1first.log 2>&1 || { tail -5 gpurun_out/$T/g1first.log; exit 1; }
echo "== graph 1 first (compare replay 0 with eager step 1 by eye)"; grep -E "replay" gpurun_out/$T/g1first.log
export DGP_FILE=/tmp/dgp_eager_hipblas.pt GMP_BLAS=cublas
DGP_MODE=eager timeout -k 10 240 python -u tools/din_graph_probe.py --steps 4 --batch 4096 > gpurun_out/$T/eager_hipblas.log 2>&1 || { tail -5 gpurun_out/$T/eager_hipblas.log; exit 1; }
GMP_CHURN=small timeout -k 10 240 python -u tools/graph_mem_probe.py --steps 4 > gpurun_out/$T/hipblas.log 2>&1 || { tail -5 gpurun_out/$T/hipblas.log; exit 1; }
echo "== hipblas"; grep -E "replay" gpurun_out/$T/hipblas.log
