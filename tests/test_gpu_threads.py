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


def test_threads_on_two_devices_capture_while_the_other_allocates(rb_lib=None):
    """The capture gate serialises per device (rb_capi.hip ApiScope /
    CaptureScope): a thread replaying captured step graphs on device 0 while
    another creates, steps and destroys worlds (hipMalloc, fills, captures)
    on device 1 must see no failed capture and exact results on both.
    Needs two GPUs (skipped on a one-GPU box)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    import rbhip
    from rbhip import scenes
    rbhip.load()
    sc0, sc1 = scenes.flat_spheres(16, 16, seed=1), scenes.flat_spheres(12, 20, seed=2)
    steps = 20
    ref0, ref1 = _run(rbhip, sc0, steps), _run(rbhip, sc1, steps)
    errors = []

    def replayer():
        try:
            with rbhip.World(sc0, device=0) as w:
                for it in range(200):
                    w.set_state(sc0.qpos0, sc0.qvel0)
                    w.step(steps)                      # a cached graph after the first iteration
                    q, v = w.get_state()
                    if not (np.array_equal(q.view(np.uint64), ref0[0].view(np.uint64)) and
                            np.array_equal(v.view(np.uint64), ref0[1].view(np.uint64))):
                        errors.append(f"device 0 iteration {it}: state differs")
                        return
        except Exception as e:
            errors.append(f"device 0: {e}")

    def allocator():
        try:
            for it in range(60):
                with rbhip.World(sc1, device=1) as w:
                    w.set_state(sc1.qpos0, sc1.qvel0)
                    w.step(steps)
                    q, v = w.get_state()
                if not (np.array_equal(q.view(np.uint64), ref1[0].view(np.uint64)) and
                        np.array_equal(v.view(np.uint64), ref1[1].view(np.uint64))):
                    errors.append(f"device 1 iteration {it}: state differs")
                    return
        except Exception as e:
            errors.append(f"device 1: {e}")

    th = [threading.Thread(target=replayer), threading.Thread(target=allocator)]
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


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_get_state_download_forms_agree(monkeypatch, dtype):
    """rb_get_state's three download forms (RBHIP_IO_OUT, read per call:
    0 one DMA, 1 the DMA in four chunks — taken from 16,384 bodies — and 2
    the kernel storing into mapped pinned memory) hand out the same bytes,
    into fresh and into caller-owned arrays, and each leaves the staging a
    mirror of the state (the next unchanged rb_set_state is skipped)."""
    import rbhip
    from rbhip import scenes
    rbhip.load()
    sc = scenes.flat_spheres(160, 128, seed=5)          # 20,480 bodies: the chunked form splits
    with rbhip.World(sc, dtype=dtype) as w:
        w.set_state(sc.qpos0, sc.qvel0)
        w.step(7)
        outs = []
        for mode in ("0", "1", "2"):
            monkeypatch.setenv("RBHIP_IO_OUT", mode)
            q, v = w.get_state()
            qd, vd = np.full((sc.n, 7), -7.0), np.full((sc.n, 6), -7.0)
            w.get_state(qd, vd)
            assert np.array_equal(q.view(np.uint64), qd.view(np.uint64))
            assert np.array_equal(v.view(np.uint64), vd.view(np.uint64))
            before = w.stats()["io_skipped"]
            w.set_state(q, v)
            assert w.stats()["io_skipped"] == before + 1, mode
            outs.append((q, v))
        for q, v in outs[1:]:
            assert np.array_equal(q.view(np.uint64), outs[0][0].view(np.uint64))
            assert np.array_equal(v.view(np.uint64), outs[0][1].view(np.uint64))
        assert np.isfinite(outs[0][0]).all() and (outs[0][0][:, 3:] != 0).any()
