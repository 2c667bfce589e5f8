# Round 6: the graph fix under test -- interleave tests, the DIN graph test,
# then the bench with its in-bench DIN / DLRM graph checks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06p}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_interleave.py tests/test_gpu_din_graph.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$T/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log > gpurun_out/$T/bench.json
grep -E "din leg|dlrm model step" gpurun_out/$T/bench.log | cut -c1-600
python3 -c "import json;d=json.load(open('gpurun_out/$T/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print(json.dumps(d.get('cpu_baseline'))[:600])"
