"""Mirror of src/visualization/logger_base.py: per-body trajectory record
(time, x, y, z) with the reference's plot names.  Plots need matplotlib
(imported when a plot is saved); save_npz writes the raw samples for
headless runs."""
import os

import numpy as np


class LoggerBase:
    """logger_base.py:8-32 — record(time, pos)."""

    def __init__(self):
        self.times = []
        self.x_positions = []
        self.y_positions = []
        self.z_positions = []

    def record(self, time, pos):
        self.times.append(float(time))
        self.x_positions.append(float(pos[0]))
        self.y_positions.append(float(pos[1]))
        self.z_positions.append(float(pos[2]))

    def as_array(self) -> np.ndarray:
        """(n, 4): time, x, y, z."""
        return np.column_stack([self.times, self.x_positions, self.y_positions, self.z_positions]) \
            if self.times else np.zeros((0, 4))

    def save_npz(self, save_path):
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        np.savez(save_path, trajectory=self.as_array())

    def save_height_vs_time(self, save_path):
        """logger_base.py:34-47."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        plt.figure(figsize=(10, 6))
        plt.plot(self.times, self.z_positions, marker="o", linestyle="-")
        plt.xlabel("Time (s)")
        plt.ylabel("Height (z-axis)")
        plt.title("Height vs Time")
        plt.grid(True)
        plt.savefig(save_path)
        plt.close()

    def save_3d_trajectory(self, save_path):
        """logger_base.py:49-64."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        fig = plt.figure(figsize=(10, 7))
        ax = fig.add_subplot(111, projection="3d")
        ax.plot(self.x_positions, self.y_positions, self.z_positions, marker="o")
        ax.set_xlabel("X position")
        ax.set_ylabel("Y position")
        ax.set_zlabel("Height (z)")
        ax.set_title("3D Trajectory")
        plt.savefig(save_path)
        plt.close()
