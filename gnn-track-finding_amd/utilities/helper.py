"""Drop-in for the hot-path part of src/utilities/helper.py.

Same function names, arguments and mutation semantics as the reference; the
state math runs in libgtf.so (HIP, gfx950) through gtf.stages. Plot helpers and
the pandas graph builders are outside the hot path.
"""
import networkx as nx

from gtf import stages as _st


def get_volume_id(layer_id):                       # helper.py:15-16
    return int(layer_id / 1000)


def get_in_volume_layer_id(layer_id):              # helper.py:18-19
    return int(layer_id % 100)


def initialize_edge_activation(GraphList):         # helper.py:24-25
    for subGraph in GraphList:
        nx.set_edge_attributes(subGraph, 1, "activated")


def compute_track_state_estimates(GraphList, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary):  # helper.py:238-452
    return _st.compute_track_state_estimates(GraphList, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary)


def compute_prior_probabilities(GraphList, track_state_key):       # helper.py:30-63
    _st.compute_prior_probabilities(GraphList, track_state_key)


def query_node_degree_in_edges(subGraph, node_num):                # helper.py:67-73 (scalar accessor)
    return sum(1 for u, _ in subGraph.in_edges(node_num) if subGraph[u][node_num]["activated"] == 1)


def compute_mixture_weights(GraphList, TRACK_STATE_KEY):            # helper.py:76-96
    _st.compute_mixture_weights(GraphList, TRACK_STATE_KEY)


def reweight(subGraphs, track_state_estimates_key):                 # helper.py:143-225
    _st.reweight(subGraphs, track_state_estimates_key)


def save_network(directory, i, subGraph):                           # helper.py:585-587
    _st.save_network(directory, i, subGraph)
