"""One world per host thread (include/rbhip.h, SURVEY §8b "a handle is not
thread-safe; use one world per host thread"): the library keeps no
process-global mutable state besides the thread-local error string (the
bounding radii live in rb_world; the host copy pool serialises its jobs), so
two threads that each create, load, step, read and destroy their own worlds
get exactly the single-threaded results."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(rb, sc, steps):
    with rb.World(sc) as w:
        w.set_state(sc.qpos0, sc.qvel0)
        w.step(steps)
        return w.get_state()


def test_two_threads_each_with_own_worlds(rb_lib=None):
    import rbhip
    from rbhip import scenes
    rbhip.load()
    scs = [scenes.flat_spheres(16, 16, seed=1), scenes.flat_spheres(12, 20, seed=2)]
    steps = 20
    ref = [_run(rbhip, sc, steps) for sc in scs]
    errors = []

    def worker(k):
        try:
            for it in range(100):
                q, v = _run(rbhip, scs[k], steps)
                if not (np.array_equal(q.view(np.uint64), ref[k][0].view(np.uint64)) and
                        np.array_equal(v.view(np.uint64), ref[k][1].view(np.uint64))):
                    errors.append(f"thread {k} iteration {it}: state differs from the single-threaded run")
                    return
        except Exception as e:          # an RbError from the library
            errors.append(f"thread {k}: {e}")

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th), "a worker thread did not finish"
    assert not errors, errors[:3]


def test_unchanged_set_state_is_a_no_op_and_exact(rb_lib=None):
    """rb_set_state with the bytes rb_get_state just returned (the per-frame
    caller) skips the upload; with one byte changed it uploads; results stay
    bit-exact with a world that always uploads."""
    import rbhip
    from rbhip import scenes
    rbhip.load()
    sc = scenes.flat_spheres(32, 32, seed=4)
    with rbhip.World(sc) as w, rbhip.World(sc) as ref:
        q, v = sc.qpos0.copy(), sc.qvel0.copy()
        for frame in range(30):
            w.set_state(q, v)
            w.step(1)
            q, v = w.get_state()
            if frame == 10:
                q[3, 2] += 0.25                     # the caller moves a body between frames
        ref.set_state(sc.qpos0, sc.qvel0)
        ref.step(11)
        q_ref, v_ref = ref.get_state()
        q_ref[3, 2] += 0.25
        ref.set_state(q_ref, v_ref)
        ref.step(19)
        q_ref, v_ref = ref.get_state()
        assert np.array_equal(q.view(np.uint64), q_ref.view(np.uint64))
        assert np.array_equal(v.view(np.uint64), v_ref.view(np.uint64))
        st = w.stats()
        assert st["io_skipped"] >= 25 and st["io_uploads"] >= 2, st
