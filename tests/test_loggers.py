"""The logger mirrors: the reference's record() surface
and the plot files its save functions write (CPU only; matplotlib Agg)."""
import os

import numpy as np

from src.visualization.logger_base import LoggerBase
from src.visualization.multi_sphere_logger import MultiSphereLogger


def test_multi_sphere_logger_writes_every_reference_plot(tmp_path):
    """multi_sphere_logger.py:24-73: per ball height / 3-D / x-y plots, and
    the combined 3-D and height plots."""
    names = ["ball1", "ball2", "ball3"]
    lg = MultiSphereLogger(names)
    q = np.zeros((3, 7))
    for k in range(5):
        q[:, 0] = [0.1 * k, 0.2 * k, 0.3 * k]
        q[:, 2] = [1.0 - 0.1 * k, 0.8, 0.5 + 0.05 * k]
        lg.record_all(0.01 * k, q)
    lg.record("ball2", 0.05, (1.0, 2.0, 3.0))
    out = str(tmp_path / "plots")
    lg.save_all_plots(out)
    want = {f"{b}_{s}.png" for b in names for s in ("height_vs_time", "trajectory_3d", "trajectory_xy")}
    want |= {"combined_3d_trajectories.png", "combined_height_vs_time.png"}
    got = set(os.listdir(out))
    assert want <= got, want - got
    for f in want:
        assert os.path.getsize(os.path.join(out, f)) > 1000, f
    # the samples themselves (logger_base.py:22-32 record order)
    b2 = lg.loggers["ball2"]
    assert b2.times[-1] == 0.05 and (b2.x_positions[-1], b2.y_positions[-1], b2.z_positions[-1]) == (1.0, 2.0, 3.0)
    assert len(lg.loggers["ball1"].times) == 5


def test_logger_base_record_and_plots(tmp_path):
    lg = LoggerBase()
    for k in range(4):
        lg.record(0.009 * k, np.array([k, -k, 2.0 - 0.1 * k]))
    arr = lg.as_array()
    assert arr.shape == (4, 4) and arr[3, 1] == 3.0 and arr[3, 2] == -3.0
    lg.save_height_vs_time(str(tmp_path / "h.png"))
    lg.save_3d_trajectory(str(tmp_path / "t.png"))
    assert os.path.getsize(tmp_path / "h.png") > 1000 and os.path.getsize(tmp_path / "t.png") > 1000
