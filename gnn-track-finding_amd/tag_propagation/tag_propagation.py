"""Drop-in for tag_propagation/tag_propagation.py (the sweep, without plots).

Run in a directory holding ``0_subgraph.gpickle`` like the reference script
(:64); prints the number of tags flipped per sweep (:166) and writes the final
tags into each node's 'tags' list (appending, :150) to
``0_subgraph_tagged.gpickle``.
"""
import os
import pickle
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf import stages as _st  # noqa: E402


def tag_propagation(graph, threshold=0.1):
    """returns (node -> final tag, tags flipped per sweep) -- :97-164"""
    return _st.tag_propagation(graph, threshold)


def main():
    with open("0_subgraph.gpickle", "rb") as fh:
        G = pickle.load(fh)
    tags, flips = tag_propagation(G)
    print("number of tags flipped per iteration:\n", flips)
    for n, t in tags.items():
        G.nodes[n].setdefault("tags", [n]).append(t)
    with open("0_subgraph_tagged.gpickle", "wb") as fh:
        pickle.dump(G, fh, pickle.HIGHEST_PROTOCOL)


if __name__ == "__main__":
    main()
