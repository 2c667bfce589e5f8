"""The sharded C entries (dr_comm_init with a callback table,
dr_sharded_forward / dr_sharded_backward -- SURVEY 8b's "sharded variants
taking a dr_comm*") across PROCESSES: 2 and 3 ranks, each its own process on
cuda:0, the all-to-all behind the dr_comm callback a gloo process group
(sharded.Comm.host_staged).  tools/sharded_c_check.py checks every rank's
forward (one-hot forward-only / with gradient, multi-hot mean, bf16 EVs with
fp32 and bf16 outputs) bit-exact against one GPU's lookup of the same batch
in full local tables, and every owner's backward IndexedSlices bit-exact
against the oracle's Unique + SparseSegment*Grad of every source rank's
batch, concatenated in source-rank order.  The RCCL form of the comm runs on
the driver's multi-GPU node."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_c_entries_multiprocess(world):
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sharded_c_check.py"),
                        "--world", str(world)], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=170)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert sorted(x["rank"] for x in lines) == list(range(world))
    bad = [(x["rank"], c[0]) for x in lines for c in x["checks"] if not c[1]]
    assert not bad, bad
    assert all(x["ok"] for x in lines)
