"""Minimal restatement of filterpy 1.4.5 (third-party, not installed here, not
vendored by the reference). Used ONLY by tests/golden/make_golden.py so the
reference's extrapolation stage (src/extrapolate/extrapolate_merged_states.py:
2,7-8,307-323) can be imported to generate golden vectors. The arithmetic is
filterpy's published KalmanFilter.predict/update (Joseph-form covariance)."""
