# DLRM dot interaction on the f32 MFMA (dot_mfma_kernel) vs the LDS-tiled
# VALU kernel (DR_DOT_VALU=1), MFMA loads plain vs nontemporal (DR_DOT_NT=1):
# parity tests, kernel roofline each way, rocprof kernel times, the DLRM
# bf16 model step.  Tag $1.
set -o pipefail
T=${1:-dotm}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modelzoo.py tests/test_gpu_torch_ops.py -x -q -k "dot or dlrm or DLRM" --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for V in pf2 one e1 pf3 pf2 one; do
  unset DR_DOT_VALU DR_DOT_PF DR_DOT_BLOCKS_PER_CU DR_DOT_EXP
  [ $V = valu ] && export DR_DOT_VALU=1
  [ $V = one ] && export DR_DOT_PF=0
  [ $V = pf2 ] && export DR_DOT_BLOCKS_PER_CU=2
  [ $V = pf4 ] && export DR_DOT_BLOCKS_PER_CU=4
  [ $V = e1 ] && export DR_DOT_EXP=1 DR_DOT_BLOCKS_PER_CU=2
  [ $V = e2 ] && export DR_DOT_EXP=2 DR_DOT_BLOCKS_PER_CU=2
  timeout -k 10 200 python tools/kernel_roofline.py --only dot > gpurun_out/$T/kr.log 2>&1 || exit 1
  echo "$V $(grep '^{' gpurun_out/$T/kr.log)" | tee -a gpurun_out/$T/ab.log
done
unset DR_DOT_VALU DR_DOT_PF
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/kernel_roofline.py --only dot > gpurun_out/$T/prof.log 2>&1 || exit 1
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:5]:
    print("%-90s %6s %10.1f us avg %8.1f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 300 python tools/model_step.py --model dlrm --bf16 --steps 10 --warmup 3 > gpurun_out/$T/ms.log 2>&1 || exit 1
echo "mfma $(grep '^{' gpurun_out/$T/ms.log)" | tee -a gpurun_out/$T/ab.log
