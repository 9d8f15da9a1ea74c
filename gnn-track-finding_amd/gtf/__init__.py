"""gtf -- MI355X-native edge-parallel track-finding pass.

Host side of the drop-in for nishalad95/GNN-track-finding's hot path
(extrapolate -> update -> KL clustering, tag propagation). The compute runs in
``libgtf.so`` (hand-written HIP for gfx950, C-ABI in include/gtf.h); this
package packs the reference's networkx graphs into CSR arrays, moves them to
HBM and calls the C-ABI.
"""
from .params import Params  # noqa: F401
from .graph import TrackGraph, pack, unpack, concat  # noqa: F401

__version__ = "0.1.0"
