# Round 6: DIN / graph / sharded-capture tests, then the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06aa}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py tests/test_gpu_graph_interleave.py tests/test_gpu_sharded_capture.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.log || { tail -5 gpurun_out/$T/bench.log; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value', 'ms_per_step')}, d['roofline']['frac'])
for k in ('train_step', 'dlrm_train_step', 'din_config', 'native_engine', 'cpu_baseline'):
    print(k, json.dumps(d.get(k))[:700])
"
