"""Reference stage inputs/outputs as gpickle-format object lists, for the
end-to-end drop-in tests (tests/test_dropin.py): the drop-in stages must turn the
input graphs into graphs whose attributes equal the reference's outputs.

Run here only (needs /root/reference); writes tests/golden/dropin_*.pkl.
Reuses the harness of make_golden.py (same shims, same event, same flags).
"""
import os
import pickle
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as M  # noqa: E402


def dump(name, obj):
    path = os.path.join(HERE, "dropin_%s.pkl" % name)
    with open(path, "wb") as f:
        pickle.dump(obj, f, pickle.HIGHEST_PROTOCOL)
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024))


def main():
    with M._Quiet():
        net0 = M.build_network()
    # a few hundred subgraphs of mixed sizes keep the pickles small
    net = [s for s in net0 if len(s) >= 3][:80]
    it1 = M.run_cluster(net, "track_state_estimates", 1.0, 2.0)
    dump("cluster_tse", {"in": net, "out": it1, "args": ("track_state_estimates", 1.0, 2.0)})
    it2 = M.run_extrapolate(it1)
    dump("extrapolate", {"in": it1, "out": it2, "args": M.P})
    rem = M.simulate_extraction(it2)
    dump("update", {"in": rem, "out": M.run_update(rem)})


if __name__ == "__main__":
    main()
