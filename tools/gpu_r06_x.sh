# Round 6: rounds walk with the DPP scan: tests, per-mode kernel times, device rounds count.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06x
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py > gpurun_out/r06x/tests.log 2>&1; tail -3 gpurun_out/r06x/tests.log
grep -q " passed" gpurun_out/r06x/tests.log && ! grep -q "failed\|error" gpurun_out/r06x/tests.log &&
DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so timeout -k 10 200 python -u tools/seg_walk_probe.py --modes rounds --iters 1 > gpurun_out/r06x/debug.log 2>&1 &&
grep roundswalk gpurun_out/r06x/debug.log | awk '{n+=1; s+=$3; r+=$5} END {print n, "walks", s, "segments", r, "rounds"}' &&
grep segwalk gpurun_out/r06x/debug.log | head -10 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06x/prof -o run -- python3 tools/seg_walk_probe.py --iters 10 > gpurun_out/r06x/prof.log 2>&1 &&
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/r06x/prof/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for n in ('rows_serial_plain_kernel', 'rows_serial_seg_kernel', 'rows_seg_kernel'):
    print(n, [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if n in r['Kernel_Name']])
"
