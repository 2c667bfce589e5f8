# Round 6: the default bench line (what the driver runs), twice, for the record.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06bench}
mkdir -p gpurun_out/$T
for i in 1 2; do
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench_$i.json 2> gpurun_out/$T/bench_$i.log || { tail -5 gpurun_out/$T/bench_$i.log; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/$T/bench_$i.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value', 'ms_per_step')}, d['roofline']['frac'], d['roofline'].get('traffic_round'))
for k in ('train_step', 'dlrm_train_step', 'din_config', 'cpu_baseline'):
    v = d.get(k) or {}
    print(k, {kk: v.get(kk) for kk in ('ms_per_step', 'value', 'spread', 'graph_check', 'hipgraph')})
ne = d.get('native_engine') or {}
print('native', {k: (ne.get(k) or {}).get('ms_per_step') for k in ('xgmi', 'rccl', 'fixed')})
"
done
