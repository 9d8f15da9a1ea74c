"""Golden fixture for the initial track-state estimates (§8 a2), from the REFERENCE.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_tse.py        # writes tests/golden/tse_full.npz

Builds the whole volume-7 network of the committed minCurv_0.3_134 event with the
reference's own load/construct/compute_track_state_estimates (make_golden.
build_network, helper.py:238-452) and stores, per packed slot, every TSE field
(edge_state_vector, the aliased covariance, joint_vector tau, theta, theta2,
variance_theta, var_ms_node, neighbour xyzr, dict order) and, per node,
xy/zr_edge_gradient_mean_var, angle_of_rotation and translation.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (sets up the reference import + shims)


def main():
    with mg._Quiet():
        net = mg.build_network()
    g = mg.pack(net)
    node_xy = np.full((g.n_nodes, 2), np.nan)
    node_zr = np.full((g.n_nodes, 2), np.nan)
    angle = np.full(g.n_nodes, np.nan)
    trans = np.full((g.n_nodes, 2), np.nan)
    i = 0
    for s in net:
        for n, a in s.nodes(data=True):
            node_xy[i] = a["xy_edge_gradient_mean_var"]
            node_zr[i] = a["zr_edge_gradient_mean_var"]
            angle[i] = a["angle_of_rotation"]
            trans[i] = a["translation"]
            i += 1
    assert i == g.n_nodes
    arrs = {"in__" + k: v for k, v in mg.pick(g, mg.IN_FIELDS + ["tse_theta", "tse_var_ms"]).items()}
    arrs.update({"x__xy_mean_var": node_xy, "x__zr_mean_var": node_zr, "x__angle_of_rotation": angle,
                 "x__translation": trans})
    arrs["meta"] = np.array(repr(dict(src="helper.compute_track_state_estimates (vol 7, minCurv_0.3_134)", **mg.P)))
    path = os.path.join(HERE, "tse_full.npz")
    np.savez_compressed(path, **arrs)
    print("wrote tse_full.npz %.1f KB N=%d S=%d" % (os.path.getsize(path) / 1024, g.n_nodes, g.n_slots))


if __name__ == "__main__":
    main()
