# FETCH_SIZE calibration (tools/fetch_calib.hip): timings, then one --pmc pass
# per counter set, each under its own kill timeout.
set -o pipefail
mkdir -p gpurun_out/calib
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/fetch_calib > gpurun_out/calib/timing.log 2>&1 || exit 1
cat gpurun_out/calib/timing.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run -- ./tools/fetch_calib > gpurun_out/calib/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib/req -o run -- ./tools/fetch_calib > gpurun_out/calib/req.log 2>&1
echo "req rc=$?"
echo calibrated
