# Round 6: rounds walk cycle split on trained-model DIN terms (debug build) + kernel times per mode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06af
DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so timeout -k 10 200 python -u tools/seg_walk_probe.py --terms din_pad_terms_s200.npz --modes rounds --iters 1 > gpurun_out/r06af/debug.log 2>&1 &&
grep "roundswalk" gpurun_out/r06af/debug.log | head -24 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06af/prof -o run -- python3 tools/seg_walk_probe.py --terms din_pad_terms_s200.npz --iters 5 > gpurun_out/r06af/prof.log 2>&1 &&
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/r06af/prof/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for n in ('rows_serial_plain_kernel', 'rows_serial_seg_kernel'):
    print(n, [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if n in r['Kernel_Name']])
"
