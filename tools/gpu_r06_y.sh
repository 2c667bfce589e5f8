# Round 6: where the rounds walk's cycles go (debug build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06y
DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so timeout -k 10 200 python -u tools/seg_walk_probe.py --modes rounds --iters 1 > gpurun_out/r06y/debug.log 2>&1 &&
grep "walk run" gpurun_out/r06y/debug.log | head -60
