# Round 6: CrossNet dW with the XCD-region tile order: dW tests, timing per order, FETCH_SIZE
# (order 4 vs xcd) and MFMA busy of the hand kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ak}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -q -k "dw" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
DR_CROSSNET_DW_KERNEL=w4 timeout -k 10 300 python -u tools/cross_dw_probe.py > gpurun_out/$T/probe.log 2>&1 || { tail -5 gpurun_out/$T/probe.log; exit 1; }
grep -E "crossnet_dw|matmul" gpurun_out/$T/probe.log
for o in 4 xcd; do
DR_CROSSNET_DW_KERNEL=w4 DR_CROSSNET_DW_ORDER=$o timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/fetch_$o -o run -- python3 tools/cross_dw_probe.py --hand-only > gpurun_out/$T/fetch_$o.log 2>&1 || { tail -5 gpurun_out/$T/fetch_$o.log; exit 1; }
DR_CROSSNET_DW_KERNEL=w4 DR_CROSSNET_DW_ORDER=$o timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/mfma_$o -o run -- python3 tools/cross_dw_probe.py --hand-only > gpurun_out/$T/mfma_$o.log 2>&1 || { tail -5 gpurun_out/$T/mfma_$o.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, statistics
T = "gpurun_out/r06ak"
for o in ("4", "xcd"):
    for q in ("fetch", "mfma"):
        f = glob.glob("%s/%s_%s/**/*counter_collection.csv" % (T, q, o), recursive=True)[0]
        vals = {}
        for r in csv.DictReader(open(f)):
            if "crossnet_dw_w4_kernel" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        print(o, q, {k: statistics.median(v) for k, v in vals.items()})
PY
