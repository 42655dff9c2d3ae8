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
        """multi_sphere_logger.py:24-73: per ball its height, 3-D and x-y
        plots; then every ball in one 3-D plot and in one height plot (the
        reference's file names, axis labels and titles)."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        os.makedirs(output_dir, exist_ok=True)
        out = lambda name: os.path.join(output_dir, name)   # noqa: E731
        for ball, lg in self.loggers.items():
            lg.save_height_vs_time(out(f"{ball}_height_vs_time.png"))
            lg.save_3d_trajectory(out(f"{ball}_trajectory_3d.png"))
            _figure_2d(plt, [(lg.x_positions, lg.y_positions, None)], "X", "Y", f"{ball} XY Trajectory",
                       out(f"{ball}_trajectory_xy.png"), marker="o")
        fig = plt.figure()
        ax = fig.add_subplot(111, projection="3d")
        for ball, lg in self.loggers.items():
            ax.plot(lg.x_positions, lg.y_positions, lg.z_positions, label=ball)
        for setter, text in ((ax.set_xlabel, "X"), (ax.set_ylabel, "Y"), (ax.set_zlabel, "Z"),
                             (ax.set_title, "Combined 3D Trajectories")):
            setter(text)
        ax.legend()
        fig.savefig(out("combined_3d_trajectories.png"))
        plt.close(fig)
        _figure_2d(plt, [(lg.times, lg.z_positions, b) for b, lg in self.loggers.items()], "Time (s)", "Height (z)",
                   "Combined Height vs Time", out("combined_height_vs_time.png"), legend=True)
        print(f"All multi-sphere plots saved in {output_dir}")


def _figure_2d(plt, series, xlabel, ylabel, title, path, marker=None, legend=False):
    """One gridded 2-D figure of (x, y, label) series, saved to path."""
    fig = plt.figure()
    for xs, ys, label in series:
        plt.plot(xs, ys, marker=marker, label=label)
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    plt.title(title)
    plt.grid(True)
    if legend:
        plt.legend()
    fig.savefig(path)
    plt.close(fig)
