"""Pin config C1's x-y event to the reference's own toy Monte Carlo.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_toymc.py      # writes tests/golden/toymc_c1.npz

It imports the reference's src/toyMC_model/track_simulation_xy.py, seeds numpy's
global stream (np.random.seed(0): the script draws its smearing from it, :75), runs
simulate_event() (:36-188) with matplotlib on the Agg backend, plt.show a no-op and
plt.scatter a no-op (the script's own :177 raises there, see main()),
and records the graphs the script hands to its own plot_network: the last calls are
the weakly connected subgraphs it ends with (:175-178). Stored per subgraph: the node
ids in iteration order, every node's x, y, layer and truth, and the directed edges in
G.edges order. tests/test_toymc.py checks gtf.toymc.subgraphs(0) against them (x, y,
node sets and orders, edge lists exact).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path[:0] = [os.path.join(REF, "src", "toyMC_model"), os.path.join(REF, "src")]
os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True

import matplotlib  # noqa: E402
matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402

SEED = 0


def main():
    import track_simulation_xy as T
    plt.show = lambda *a, **k: None
    # :177 plt.scatter(x, dx) plots the last track's 10 x values against every edge's dx
    # and raises "x and y must be the same size", before the script reaches its connected
    # components (:183); the plot call is replaced by a no-op (no data flows out of it)
    plt.scatter = lambda *a, **k: None
    calls = []
    T.plot_network = lambda GraphList, *a, **k: calls.append([G.copy() for G in GraphList])
    np.random.seed(SEED)
    T.simulate_event()
    plt.close("all")
    subs = [c[0] for c in calls[2:]]      # :175-178, one call per subgraph
    out = {"n_subgraphs": np.array(len(subs))}
    nodes, xs, ys, layers, truth, sub_ptr, e_src, e_dst, e_ptr = [], [], [], [], [], [0], [], [], [0]
    for G in subs:
        for n in G.nodes():
            nodes.append(int(n))
            xs.append(float(G.nodes[n]["xy"][0]))
            ys.append(float(G.nodes[n]["xy"][1]))
            layers.append(int(G.nodes[n]["layer"]))
            truth.append(int(G.nodes[n]["truth"]))
        sub_ptr.append(len(nodes))
        for u, v in G.edges():
            e_src.append(int(u))
            e_dst.append(int(v))
        e_ptr.append(len(e_src))
    out.update(nodes=np.array(nodes, np.int64), x=np.array(xs), y=np.array(ys), layer=np.array(layers, np.int64),
               truth=np.array(truth, np.int64), sub_ptr=np.array(sub_ptr, np.int64),
               edge_src=np.array(e_src, np.int64), edge_dst=np.array(e_dst, np.int64),
               edge_ptr=np.array(e_ptr, np.int64))
    path = os.path.join(HERE, "toymc_c1.npz")
    np.savez_compressed(path, **out)
    print("wrote %s: %d subgraphs, %d nodes, %d directed edges" % (path, len(subs), len(nodes), len(e_src)))


if __name__ == "__main__":
    main()
