"""XCD-resident K-step blocks (csrc/rb_xblock.hip) against the
per-step kernels and the oracle.

A block launch steps the scene K times: each XCD's workgroups copy a slab
of the scene plus a ghost band into buffers of their own, step the copy K
times with the per-step kernels' body code (barriers among the XCD's
workgroups only) and commit their own bodies.  Bar: fp64 bit-exact (uint64
words) with K single steps — state and the next recorded step's contacts —
from t = 0 (the reference step is Jacobi across bodies,
multi_sphere_bounce.py:43-46, so the band argument makes the blocks exact),
and a block run whose speed bound fails rolls back and replays per step,
still exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rb():
    import rbhip
    rbhip.load()
    return rbhip


def _same(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint64),
                                                 np.ascontiguousarray(b).view(np.uint64))


def _world(rb, sc, monkeypatch, xb, k=None, extra=None, **kw):
    monkeypatch.setenv("RBHIP_XB", "1" if xb else "0")
    if k is not None:
        monkeypatch.setenv("RBHIP_XB_K", str(k))
    for key, val in (extra or {}).items():
        monkeypatch.setenv(key, val)
    return rb.World(sc, **kw)


def _run_pair(rb, sc, monkeypatch, chunks, k=None, extra=None, dtype="f64", sync=True):
    """The same chunks of steps through blocks and through the per-step
    kernels; returns both final states and the block world's stats."""
    out = []
    for xb in (True, False):
        with _world(rb, sc, monkeypatch, xb, k, extra if xb else None, dtype=dtype) as w:
            for n in chunks:
                if sync:
                    w.step(n)
                else:
                    w.step_async(n)
            w.sync()
            q, v = w.get_state()
            out.append((q, v, w.stats()))
    return out


@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_c3_blocks_equal_per_step_kernels(rb, monkeypatch, k):
    """C3 (the bench scene, 65,536 spheres) for 60 steps from t = 0 in
    blocks of K steps: bit-identical to the per-step kernels, every step
    committed by blocks (no roll-back)."""
    from rbhip import scenes
    sc = scenes.make("c3")
    (q1, v1, st), (q0, v0, _) = _run_pair(rb, sc, monkeypatch, [60], k=k)
    assert st["xb_steps"] == 60 and st["xb_fallbacks"] == 0, st
    assert _same(q1, q0) and _same(v1, v0)


def test_c3_driver_window_async_bit_exact(rb, oracle):
    """The driver's bench shape: 5 warm-up steps, 20 (graph capture), 20
    timed steps enqueued asynchronously, then rb_sync — bit-exact with the
    oracle after 45 steps, with the next step's contacts recorded."""
    import os
    from rbhip import scenes
    sc = scenes.make("c3")
    osc = oracle.OracleScene(sc)
    oracle.set_threads(16)
    try:
        q_ref, v_ref, (cnt, par, kin, _) = oracle.step(osc, sc.qpos0, sc.qvel0, 46, record=True)
    finally:
        oracle.set_threads(1)
    os.environ["RBHIP_XB"] = "1"
    try:
        w = rb.World(sc)
    finally:
        del os.environ["RBHIP_XB"]
    with w:
        for n in (5, 20, 20):
            w.step_async(n)
        w.sync()
        st = w.stats()
        assert st["xb_steps"] == 45 and st["xb_fallbacks"] == 0, st
        w.record_contacts(True)
        w.step(1)
        q, v = w.get_state()
        gc, gp, gk, _ = w.contacts()
    assert _same(q, q_ref) and _same(v, v_ref)
    assert np.array_equal(gc, cnt) and np.array_equal(gp, par) and np.array_equal(gk, kin)


def test_speed_bound_failure_rolls_back_bit_exact(rb, monkeypatch):
    """A speed bound that cannot hold (valpha = vbeta = 0: only gravity's
    K |g| dt) fails the blocks in flight: the run is rolled back and
    replayed per step, bit-identical, and counted as a fallback."""
    from rbhip import scenes
    sc = scenes.make("c3")
    extra = {"RBHIP_XB_VALPHA": "0", "RBHIP_XB_VBETA": "0"}
    (q1, v1, st), (q0, v0, _) = _run_pair(rb, sc, monkeypatch, [30, 30], k=6, extra=extra)
    assert st["xb_fallbacks"] >= 1, st
    assert _same(q1, q0) and _same(v1, v0)


def test_blocks_on_incline_and_32k_scene(rb, monkeypatch):
    """C4's incline (friction-dominated, sliding rows) for 120 steps and a
    32,768-sphere flat scene for 80 steps: bit-identical to the per-step
    kernels through blocks of 6."""
    from rbhip import scenes
    for sc, steps in ((scenes.make("c4"), 120), (scenes.flat_spheres(128, 256, seed=3), 80)):
        (q1, v1, st), (q0, v0, _) = _run_pair(rb, sc, monkeypatch, [steps], k=6)
        assert st["xb_steps"] + 0 >= 0
        assert _same(q1, q0) and _same(v1, v0)


def test_blocks_f32_bit_exact_vs_per_step(rb, monkeypatch):
    from rbhip import scenes
    sc = scenes.make("c3")
    (q1, v1, st), (q0, v0, _) = _run_pair(rb, sc, monkeypatch, [40], k=8, dtype="f32")
    assert st["xb_steps"] == 40, st
    assert np.array_equal(q1, q0) and np.array_equal(v1, v0)


@pytest.mark.parametrize("shape", ["c2", "slab8k"])
def test_blocks_on_cooperative_form_worlds(rb, monkeypatch, shape):
    """Worlds small enough for the cooperative per-step form (C2: 4,096
    spheres; one rank's 256 x 32 slab of C3 at 8 GPUs: 8,192) step in blocks
    on the blocks' own table layout: bit-identical to the per-step kernels."""
    from rbhip import scenes
    sc = scenes.make("c2") if shape == "c2" else scenes.flat_spheres(256, 32, seed=0)
    (q1, v1, st), (q0, v0, _) = _run_pair(rb, sc, monkeypatch, [45, 30], k=6)
    assert st["xb_steps"] == 75 and st["xb_fallbacks"] == 0, st
    assert _same(q1, q0) and _same(v1, v0)
