"""Mirror of src/visualization/data_logger.py (single object, z first)."""
from src.visualization.logger_base import LoggerBase


class DataLogger(LoggerBase):
    """data_logger.py:6-30 — record(time, z, x=None, y=None)."""

    def record(self, time_point, z_position, x_position=None, y_position=None):
        super().record(time_point, [0.0 if x_position is None else x_position,
                                    0.0 if y_position is None else y_position, z_position])

    def save_plot(self, save_path):
        self.save_height_vs_time(save_path)

    def save_trajectory_plot_3d(self, save_path):
        self.save_3d_trajectory(save_path)
