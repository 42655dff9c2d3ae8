"""Mirror of src/visualization/multi_sphere_logger.py (one trajectory per
body name)."""
import os

import numpy as np

from src.visualization.logger_base import LoggerBase


class MultiSphereLogger:
    """multi_sphere_logger.py:9-22 — record(ball_name, time, pos)."""

    def __init__(self, ball_names):
        self.ball_names = list(ball_names)
        self.loggers = {ball: LoggerBase() for ball in self.ball_names}

    def record(self, ball_name, time, pos):
        self.loggers[ball_name].record(time, pos)

    def record_all(self, time, qpos):
        """Every body at once from a (N, 7) qpos sample (body k = ball_names[k])."""
        q = np.asarray(qpos).reshape(-1, 7)
        for k, ball in enumerate(self.ball_names):
            self.loggers[ball].record(time, q[k, 0:3])

    def save_npz(self, save_path):
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        np.savez(save_path, **{b: lg.as_array() for b, lg in self.loggers.items()})

    def save_all_plots(self, output_dir="data/multi_sphere/plots"):
        """multi_sphere_logger.py:24-50 (per-ball height and 3-D plots)."""
        os.makedirs(output_dir, exist_ok=True)
        for ball, lg in self.loggers.items():
            lg.save_height_vs_time(os.path.join(output_dir, f"{ball}_height_vs_time.png"))
            lg.save_3d_trajectory(os.path.join(output_dir, f"{ball}_trajectory_3d.png"))
