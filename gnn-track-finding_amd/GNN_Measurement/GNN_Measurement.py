"""Pickle-compatible hit record stored on every graph node.

Drop-in for the reference's ``GNN_Measurement`` class
(src/GNN_Measurement/GNN_Measurement.py:1-9). Stage gpickles pickle this
class by its module path ``GNN_Measurement.GNN_Measurement``, so the class
name, module path and attribute names must stay exactly as they are.
"""


class GNN_Measurement(object):
    def __init__(self, x, y, z, r, truth_particle=-1, n=None):
        self.x = x
        self.y = y
        self.z = z
        self.r = r
        self.truth_particle = truth_particle
        self.node = n

    def __repr__(self):
        return "GNN_Measurement(x=%r, y=%r, z=%r, r=%r, truth_particle=%r, n=%r)" % (
            self.x, self.y, self.z, self.r, self.truth_particle, self.node)
