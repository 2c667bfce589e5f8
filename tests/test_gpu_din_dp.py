"""Data-parallel DIN (BASELINE configs[3], 1 -> N GPUs): replicated EVs,
dense gradients all-reduced, EV gradient slices gathered in rank order
(modelzoo.din_train_step(world=N)), 2 and 3 processes on one GPU against one
process running the same step over every rank's slice (tools/din_dp_check.py;
Dice normalises over a replica's batch, so each slice's forward is its own): loss,
dense weights and all three tables within 1e-5 relative after each of three
steps, replicas bit-identical across ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_din_data_parallel_matches_one_process(world):
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "din_dp_check.py"),
                        "--world", str(world)], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=170)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert sorted(x["rank"] for x in lines) == list(range(world))
    assert all(x["ok"] for x in lines), lines
