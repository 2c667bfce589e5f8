# Round 6: DIN's padding-id segment terms saved for host replays of the walk
# (first step, and after 20 / 200 training steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06u
for n in 20 200; do
  DTP_STEPS=$n DTP_SAVE=gpurun_out/r06u/din_terms_s$n.npz timeout -k 10 200 python -u tools/din_term_probe.py || exit 1
done
