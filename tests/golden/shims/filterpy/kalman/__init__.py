from .kalman_filter import KalmanFilter, update, predict  # noqa: F401
