"""The DIN training step (modelzoo.din_train_step: merged item lookup, fused
attention, capturable dense Adam, KV Adam with HBM beta powers) captured as
hipGraphs, one per batch shape, replays bit-equal to the eager steps: the
eager run and the graph run each alone in a process (tools/din_graph_probe.py
DGP_MODE=eager / graph), losses of every step and the final parameters and
EV contents compared bitwise."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_din_graph_replays_equal_eager(tmp_path):
    probe = os.path.join(ROOT, "tools", "din_graph_probe.py")
    env = dict(os.environ, DGP_FILE=str(tmp_path / "eager.pt"))
    for mode in ("eager", "graph"):
        env["DGP_MODE"] = mode
        r = subprocess.run([sys.executable, probe, "--steps", "8", "--batch", "512"], env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (mode, r.stdout[-2000:], r.stderr[-2000:])
    assert "== eager run: True" in r.stdout, r.stdout[-2000:]
