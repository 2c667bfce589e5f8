"""CPU: the oracle's KvSparseApplyAdamAsync / KvSparseApplyAdagradDecay
restatements (oracle/deeprec_oracle.c orc_ev_apply_adam_async /
orc_ev_apply_adagrad_decay) pinned by the reference's own known-answer
tests: python/training/adam_async_test.py:39-105 (adam_update_numpy over 3
steps, beta powers 0.9^t / 0.999^t) and python/training/adagrad_decay_test.py
:98-153 (4 steps, decay_step 3, rate 0.9: the accumulator decays once, on the
third step, when global_step + 1 = 3).  Tolerances are the reference tests'
assertAllCloseAccordingToType for float32 (1e-6 rel / abs)."""
import numpy as np
import pytest


def _adam_update_numpy(param, g, t, m, v, alpha=0.001, beta1=0.9, beta2=0.999, eps=1e-8):
    alpha_t = alpha * np.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    return param - alpha_t * m / (np.sqrt(v) + eps), m, v


def test_oracle_adam_async_matches_reference_kat(orc):
    var0, g0 = np.array([1.0, 2.0]), np.array([0.1, 0.1], np.float32)
    ev = orc.EV(1, 0.0)
    m_ev, v_ev = ev.create_slot(1, 0.0), ev.create_slot(2, 0.0)
    ev.insert(np.array([0, 1]), var0.astype(np.float32).reshape(2, 1))
    m0 = v0 = 0.0
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    for t in range(1, 4):
        np.testing.assert_allclose(b1p, 0.9 ** t, rtol=1e-6)
        ev.apply_adam_async(m_ev, v_ev, float(b1p), float(b2p), 0.001, 0.9, 0.999, 1e-8,
                            g0.reshape(2, 1), np.array([0, 1]))
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
        var0, m0, v0 = _adam_update_numpy(var0, g0.astype(np.float64), t, m0, v0)
        np.testing.assert_allclose(ev.gather(np.array([0, 1]))[:, 0], var0, rtol=1e-6, atol=1e-6)


def test_oracle_adam_async_rmsprop_formula(orc):
    """apply_sparse_rmsprop (training_ali_ops.cc:1506-1513) in float64."""
    rng = np.random.default_rng(5)
    D = 4
    ev = orc.EV(D, 0.5)
    m_ev, v_ev = ev.create_slot(1, 0.0), ev.create_slot(2, 0.0)
    w, m, v = np.full(D, 0.5), np.zeros(D), np.zeros(D)
    for _ in range(4):
        g = (rng.standard_normal((1, D)) * 0.3).astype(np.float32)
        ev.apply_adam_async(m_ev, v_ev, 0.0, 0.0, 0.01, 0.9, 0.999, 1e-8, g, np.array([3]),
                            rmsprop=True)
        gd = g[0].astype(np.float64)
        v = v * 0.999 + gd * gd * (1 - 0.999)
        m = m * 0.9 + 1.0 / np.sqrt(v + 1e-8) * 0.01 * gd
        w = w - m
        np.testing.assert_allclose(ev.gather(np.array([3]))[0], w, rtol=1e-5, atol=1e-6)


def test_oracle_adagrad_decay_matches_reference_kat(orc):
    ev = orc.EV(1, 0.0)
    acc, pw = ev.create_slot(1, 0.1), ev.create_slot(2, 0.0)
    ev.insert(np.array([0, 1]), np.array([[1.0], [2.0]], np.float32))
    v0_expect, v0_accum = 1.0, 0.1
    for step in range(4):
        # global_step before the step; the optimizer feeds global_step + 1
        ev.apply_adagrad_decay(acc, pw, 1.0, 3, 0.9, 0.1, np.array([[0.1]], np.float32),
                               np.array([0]), step + 1)
        if step == 2:
            v0_accum = v0_accum * 0.9
        v0_accum = v0_accum + 0.1 * 0.1
        v0_expect = v0_expect - 1.0 / np.sqrt(v0_accum) * 0.1
    got = ev.gather(np.array([0, 1]))[:, 0]
    np.testing.assert_allclose(got, [v0_expect, 2.0], rtol=1e-6, atol=1e-6)
    assert pw.gather(np.array([0]))[0, 0] == 1.0       # decayed exactly once


def test_oracle_adagrad_decay_baseline_floor(orc):
    """accum = max(accum * rate, baseline): a small accumulator is floored."""
    ev = orc.EV(2, 0.0)
    acc, pw = ev.create_slot(1, 0.1), ev.create_slot(2, 0.0)
    g = np.zeros((1, 2), np.float32)
    ev.apply_adagrad_decay(acc, pw, 1.0, 1, 0.5, 0.1, g, np.array([7]), 5)
    np.testing.assert_array_equal(acc.gather(np.array([7]))[0], np.float32(0.1))
    np.testing.assert_array_equal(pw.gather(np.array([7]))[0], [1.0, 0.0])
    with pytest.raises(Exception):
        ev.apply_adagrad_decay(acc, pw, 1.0, 0, 0.5, 0.1, g, np.array([7]), 5)


def test_adagrad_decay_constructor_checks():
    """AdagradDecayOptimizer's argument checks (adagrad_decay.py:64-72)."""
    import deeprec_amd as dr
    for kw in ({"initial_accumulator_value": 0.0}, {"accumulator_decay_step": 0},
               {"accumulator_decay_rate": 1.0}, {"accumulator_decay_rate": 0.0}):
        with pytest.raises(ValueError):
            dr.AdagradDecayOptimizer(0.1, **kw)
    o = dr.AdamAsyncOptimizer(apply_sparse_rmsprop=True)
    assert o._opt == 4 and dr.AdamAsyncOptimizer()._opt == 3
