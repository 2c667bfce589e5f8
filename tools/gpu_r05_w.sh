# Round 5, batch W: which kernels run while the DIN step is being captured
# (they run eagerly instead of into the graph).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05w2}
mkdir -p gpurun_out/$T
DGP_CAPTURE_ONLY=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o cap -- python3 -u tools/din_graph_probe.py --steps 1 > gpurun_out/$T/cap.log 2>&1 || { tail -5 gpurun_out/$T/cap.log; exit 1; }
f=$(find gpurun_out/$T/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the capture window: after the last >250 ms gap
gaps = [(int(rows[i+1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]), i) for i in range(len(rows)-1)]
big = [i for g, i in gaps if g > 250e6]
print("kernels", len(rows), "big gaps after index", big)
if big:
    s = big[0] + 1
    e = big[1] if len(big) > 1 else len(rows) - 1
    print("kernels inside the capture window:", e - s + 1)
    for r in rows[s:e+1][:40]:
        print("  ", r["Kernel_Name"][:110])
PY
