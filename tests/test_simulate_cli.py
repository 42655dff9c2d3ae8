"""Headless runner src/simulate.py: argument handling on
the CPU; the GPU runs are checked in test_gpu_shims.py."""
import os

import numpy as np
import pytest

from src import simulate


def test_unknown_and_unsupported_names(capsys):
    assert simulate.main(["--sim", "nope"]) == 1
    assert simulate.main(["--sim", "compare_builtin"]) == 2
    err = capsys.readouterr().err
    assert "Available" in err and "mj_step" in err


@pytest.mark.parametrize("name", sorted(simulate.SIMS))
def test_builtin_scenes(name):
    sc = simulate.build_scene(name)
    assert sc.n >= 1 and sc.dt > 0


@pytest.mark.skipif(not os.path.isdir("/root/reference/models"), reason="reference checkout not present")
@pytest.mark.parametrize("name,model", [("single_sphere", "sphere"), ("cube_incline", "cube"),
                                        ("multi_sphere", "multi_sphere"), ("ball_collision", "ball_collision")])
def test_mjcf_scenes_equal_builtin(name, model):
    """The reference's model files plus the scripts' initial conditions give
    exactly the built-in scenes."""
    a = simulate.build_scene(name, f"/root/reference/models/{model}.xml")
    b = simulate.build_scene(name)
    for f in ("kind", "mass", "inertia", "size", "planes", "qpos0", "qvel0", "gravity"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert a.dt == b.dt
