import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gnn-track-finding_amd"), ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

# torch before anything loads libgtf: a test process then always holds ONE HIP runtime,
# torch's, which libgtf shares (gtf._native.lib); host helpers that load libgtf lean
# (no torch, as in a drop-in CLI process) find it already bound
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")
