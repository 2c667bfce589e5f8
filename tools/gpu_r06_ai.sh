# Round 6: serial segment walk cycle split (debug build), first-step and trained terms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06ai
for f in din_pad_terms.npz din_pad_terms_s200.npz; do
DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so timeout -k 10 200 python -u tools/seg_walk_probe.py --terms $f --modes seg-rep_add --iters 1 > gpurun_out/r06ai/debug_$f.log 2>&1 || exit 1
echo $f; grep "segwalk" gpurun_out/r06ai/debug_$f.log | head -10
done
