"""CPU: the oracle's KV FTRL restatement (oracle/deeprec_oracle.c
orc_ev_apply_ftrl) against a direct numpy transcription of COMPUTE_FTRL
(core/kernels/training_ali_ops.cc:279-307) in float32, element order
ascending.  Both evaluate the same scalar formula in the same order; the
tolerance (2e-6 rel) only absorbs an ulp between C powf / sqrtf and numpy."""
import numpy as np
import pytest


def _ftrl_np(var, accum, linear, g, lr, l1, l2, lr_power, shr):
    f = np.float32
    var, accum, linear = var.copy(), accum.copy(), linear.copy()
    gu = (g + f(2.0) * f(shr) * var).astype(np.float32) if shr > 0 else g
    na = (accum + gu * gu).astype(np.float32)
    if lr_power == -0.5:
        p_new, p_old = np.sqrt(na), np.sqrt(accum)
    else:
        p_new = np.power(na, f(-lr_power)).astype(np.float32)
        p_old = np.power(accum, f(-lr_power)).astype(np.float32)
    t = ((p_new - p_old) / f(lr) * var).astype(np.float32)
    linear = (linear + (gu - t)).astype(np.float32)
    nsq = np.float32(0)
    for x in linear:
        nsq = np.float32(nsq + x * x)
    norm = np.sqrt(nsq)
    if norm > l1:
        eta = (p_new / f(lr)).astype(np.float32)
        coef = ((f(l1) - norm) / ((eta + f(2.0) * f(l2)) * norm)).astype(np.float32)
        var = (coef * linear).astype(np.float32)
    else:
        var = np.zeros_like(var)
    accum = (accum + g * g).astype(np.float32)
    return var, accum, linear


@pytest.mark.parametrize("lr_power,shr,l1", [(-0.5, 0.0, 0.0), (-0.5, 0.0, 0.3), (-0.7, 0.05, 0.01)])
def test_oracle_ftrl_matches_numpy(orc, lr_power, shr, l1):
    rng = np.random.default_rng(3)
    D, lr, l2 = 5, 0.2, 0.01
    ev = orc.EV(D, 0.4)
    acc, lin = ev.create_slot(1, 0.1), ev.create_slot(2, 0.0)
    var = np.full(D, 0.4, np.float32)
    a = np.full(D, 0.1, np.float32)
    li = np.zeros(D, np.float32)
    for step in range(5):
        g = (rng.standard_normal((1, D)) * 0.5).astype(np.float32)
        ev.apply_ftrl(acc, lin, lr, l1, l2, lr_power, shr, g, np.array([9]), step)
        var, a, li = _ftrl_np(var, a, li, g[0], lr, l1, l2, lr_power, shr)
        np.testing.assert_allclose(ev.gather(np.array([9]))[0], var, rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(acc.gather(np.array([9]))[0], a, rtol=1e-6)
