"""ctypes binding of libgtf.so (the C-ABI declared in include/gtf.h).

The library is built in-tree (``__graft_entry__.build()`` / ``make -C
gnn-track-finding_amd/csrc``) and loaded from this directory. There is no CPU
fallback: if the library is missing or fails to load, every call raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GTF_LIB") or os.path.join(HERE, "libgtf.so")   # GTF_LIB: an alternative build

P = ctypes.c_void_p
I32 = ctypes.c_int32
F64 = ctypes.c_double


U32 = ctypes.c_uint32
ABI_VERSION = 7   # GTF_ABI_VERSION of include/gtf.h


class GtfGraph(ctypes.Structure):
    """gtf_graph; keyword construction only -- struct_size / abi_version are filled in,
    and the library refuses a struct of another layout (status -3)"""
    _fields_ = [("struct_size", U32), ("abi_version", U32), ("n_nodes", I32), ("n_slots", I32), ("n_edges", I32), ("n_big", I32),
                ("slot_ptr", P), ("slot_src", P), ("slot_dst", P), ("out_ptr", P), ("out_slot", P),
                ("slot_outpos", P),
                ("is_edge", P), ("rev_edge", P), ("solo", P), ("gnn", P), ("xyzr", P), ("layer", P),
                ("sched", P), ("n_g8", I32), ("n_g16", I32), ("n_g32", I32), ("n_g64", I32), ("out_dst", P),
                ("slot_layer", P), ("n_g4", I32), ("sched_seg", P),
                ("out_sched", P), ("n_o4", I32), ("n_o8", I32), ("n_o16", I32), ("n_g2", I32),
                ("pack_ent", P), ("pack_wave", P), ("n_pack_waves", I32), ("out_lanes", P),
                ("pad_tiles", I32), ("pad_tile_nodes", I32), ("pad_tile_slots", I32), ("pad_count", I32 * 6),
                ("pad_reserved_", I32), ("slot_outidx", P), ("slot_class", P), ("slot_sflags", P),
                ("slot_sxzr", P), ("slot_static", P), ("slot_xclass", P)]

    def __init__(self, **fields):
        super().__init__(**fields)
        self.struct_size = ctypes.sizeof(GtfGraph)
        self.abi_version = ABI_VERSION


class GtfNodes(ctypes.Structure):
    _fields_ = [("has_merged", P), ("merged_state", P), ("merged_cov", P), ("merged_prior", P),
                ("has_tse", P), ("has_uts", P), ("degree", P)]


class GtfStates(ctypes.Structure):
    _fields_ = [("rank", P), ("sv", P), ("tau", P), ("cov", P), ("xyzr", P), ("lik", P), ("mw", P),
                ("prior", P), ("lr", P), ("side", P), ("fresh", P)]


class GtfEdges(ctypes.Structure):
    _fields_ = [("act", P), ("edge_mw", P), ("send_mw", P)]


class GtfParams(ctypes.Structure):
    _fields_ = [("sigma0xy", F64), ("sigma0rz", F64), ("sigma0rz2", F64), ("endcap_boundary", F64),
                ("chi2_cut", F64), ("reweight_threshold", F64), ("cluster_chi2", F64), ("cluster_kl", F64)]


class GtfShard(ctypes.Structure):
    _fields_ = [("senders", P), ("n_senders", I32), ("node_lo", I32), ("node_hi", I32), ("slot_lo", I32),
                ("slot_hi", I32), ("phases", I32), ("slot_list", P), ("n_slot_list", I32), ("pad_", I32)]


class GtfHalo(ctypes.Structure):
    _fields_ = [("node_idx", P), ("node_off", P), ("n_nodes", I32), ("pad_", I32), ("slot_idx", P), ("slot_off", P),
                ("n_slots", I32), ("pad2_", I32)]


HALO_NODE_BYTES = 80   # GTF_HALO_NODE_BYTES


class GtfTseExtra(ctypes.Structure):
    _fields_ = [("theta", P), ("var_ms", P), ("xy_mean_var", P), ("zr_mean_var", P), ("angle", P),
                ("translation", P)]


class GtfExtractParams(ctypes.Structure):
    _fields_ = [("p_accept", F64), ("fragment", I32), ("pad_", I32), ("separation_3d", F64),
                ("merge_distance", F64), ("sigma0xy", F64), ("sigma0rz", F64), ("endcap_boundary", F64)]


class GtfExtractIO(ctypes.Structure):
    _fields_ = [("xyzr", P), ("vivl", P), ("sub_id", P), ("sub_ptr", P), ("n_sub", I32), ("pad_", I32),
                ("order_key", P), ("gnn", P), ("label", P), ("status", P), ("pval_xy", P), ("pval_zr", P),
                ("extracted", P), ("n_candidates", P)]


class GtfEventCsr(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int64), ("n_rows", ctypes.c_int64), ("node_id", P), ("row_a", P),
                ("row_b", P), ("order", P), ("sub_id", P), ("slot_ptr", P), ("slot_src", P), ("tse_rank", P),
                ("out_ptr", P), ("out_slot", P), ("n_edges", ctypes.c_int64), ("n_subgraphs", I32), ("pad_", I32)]


class GtfCandidateGraph(ctypes.Structure):
    _fields_ = [("n_nodes", I32), ("n_slots", I32), ("n_edges", I32), ("pad_", I32), ("slot_ptr", P),
                ("slot_src", P), ("is_edge", P), ("act", P), ("out_ptr", P), ("out_slot", P), ("sub_id", P),
                ("node_id", P)]


class GtfKlGraph(ctypes.Structure):
    _fields_ = [("n_nodes", I32), ("n_slots", I32), ("slot_ptr", P), ("slot_src", P), ("gnn", P), ("truth", P),
                ("pair_ptr", P), ("list", P * 4), ("count", I32 * 4), ("first", I32 * 4), ("n_d1", I32),
                ("gnn_stride", I32), ("slot0", ctypes.c_int64), ("pair0", ctypes.c_int64), ("blk", P),
                ("n_blk", I32), ("deg_runs", I32), ("n_deg", I32 * 6), ("pad_deg_", I32)]


class GtfDiag(ctypes.Structure):
    _fields_ = [("node_err", P), ("edge_chi2", P), ("slot_cluster", P), ("reserved_", P * 5)]


DIAG_OFFSET = 64
COMM_ID_BYTES = 128   # GTF_COMM_ID_BYTES


class GtfPairOut(ctypes.Structure):
    _fields_ = [("chi2", P), ("avg_tau", P), ("avg_theta", P), ("delta_theta", P), ("truth", P), ("err", P)]


class GtfKlOut(ctypes.Structure):
    _fields_ = [("kl", P), ("truth", P), ("emp_var", P), ("emp_mean", P), ("sv", P), ("cov", P), ("err", P)]


GTF_F64, GTF_F32 = 0, 1

ERR_FLAGS = {
    1: "KeyError: sender has no track_state_estimates entry for the receiver (extrapolate_merged_states.py:384)",
    2: "KeyError: last state key has no edge (helper.py:131/138)",
    4: "ValueError: all pairwise distances are zero (clustering.py:120)",
    8: "ValueError: a distance tie removed every state (clustering.py:116)",
    16: "ZeroDivisionError: empty state dict (helper.py:90)",
    32: "ValueError: NaN KL distance (clustering.py:117)",
    64: "KeyError: node has no state dict (remove_state_metadata.py:39)",
    128: "LinAlgError: singular parabola matrix H (learn_KL_parabolic_model utils.py:277)",
    256: "pair_ptr disagrees with the updated_track_states dicts (caller error)",
    512: "KeyError: neighbour not in the subgraph (calculate_distance_between_updated_track_states.py:182-183)",
    1024: "a node holds more than 2048 updated track states (not processed)",
}

# exported symbols (must match include/gtf.h; tests check the .so exports all of them)
SYMBOLS = ["gtf_workspace_bytes", "gtf_workspace_init", "gtf_uts_materialize", "gtf_clear_errors", "gtf_read_errors", "gtf_extrapolate", "gtf_update",
           "gtf_message_passing", "gtf_node_ops",
           "gtf_cluster", "gtf_pass", "gtf_pass_ev", "gtf_tag_prepare", "gtf_tag_sweep", "gtf_tag_sweep_shard", "gtf_tag_workspace_bytes", "gtf_tag_propagate", "gtf_parabolic_kl", "gtf_track_state_estimates", "gtf_pass_shard",
           "gtf_shard_chunk_bytes", "gtf_shard_pack", "gtf_shard_unpack", "gtf_halo_pack", "gtf_halo_unpack",
           "gtf_extract_workspace_bytes",
           "gtf_extract_candidates", "gtf_build_event_csr", "gtf_candidate_order",
           "gtf_build_event_device_workspace_bytes", "gtf_build_event_csr_device",
           "gtf_updated_state_pair_counts", "gtf_updated_state_distances", "gtf_set_diagnostics",
           "gtf_device_init", "gtf_malloc", "gtf_free", "gtf_memcpy_htod", "gtf_memcpy_dtoh", "gtf_memcpy_dtod",
           "gtf_memset", "gtf_stream_synchronize",
           "gtf_comm_unique_id", "gtf_comm_init", "gtf_comm_destroy", "gtf_comm_rank", "gtf_comm_size",
           "gtf_halo_exchange", "gtf_halo_alltoall", "gtf_allreduce_max_i64", "gtf_allgather_bytes",
           "gtf_tag_shard_workspace_bytes",
           "gtf_tag_propagate_shard",
           "gtf_last_error",
           "gtf_version"]

OPS = {"ranks": 1, "priors_tse": 2, "priors_uts": 3, "reweight_uts": 4, "degree": 5, "prune": 6, "mw_tse": 7,
       "mw_uts": 8, "cluster_tse": 9, "cluster_uts": 10, "fresh": 11}

_lib = None
_lean = False   # loaded without torch (lean=True): only gtf.devmem allocations may be used


def lib(lean: bool = False):
    """Load libgtf.so once; raise loudly if it is missing (no fallback path).

    lean=False (default): torch is imported first, so its bundled libamdhip64 (SONAME
    libamdhip64.so.7) satisfies libgtf's NEEDED entry and the process holds ONE HIP
    runtime, which torch tensors and libgtf share. Loaded the other way round, torch
    pulls a second runtime and libgtf's calls see no device.
    lean=True (the drop-in CLIs, gtf.devmem): torch is not imported; libgtf binds the
    system HIP runtime and every allocation comes from gtf_malloc. A process that loaded
    libgtf this way cannot use torch device tensors with it afterwards (lib() raises)."""
    global _lib, _lean
    if _lib is not None:
        if _lean and not lean:
            raise RuntimeError("libgtf was loaded without torch (gtf.devmem, the drop-in CLIs' lean runtime); "
                               "torch device tensors cannot share it in this process")
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libgtf.so not built at %s -- run __graft_entry__.build() "
                           "(hipcc --offload-arch=gfx950); there is no CPU fallback" % LIB_PATH)
    import sys
    if lean and "torch" not in sys.modules:
        _lean = True
    else:
        import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    L.gtf_workspace_bytes.restype = ctypes.c_size_t
    L.gtf_workspace_bytes.argtypes = [I32, I32]
    L.gtf_clear_errors.argtypes = [P, P]
    L.gtf_workspace_init.argtypes = [P, P]
    L.gtf_read_errors.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P]
    L.gtf_set_diagnostics.argtypes = [P, ctypes.POINTER(GtfDiag), P]
    G, N, S, E, PR = (ctypes.POINTER(GtfGraph), ctypes.POINTER(GtfNodes), ctypes.POINTER(GtfStates),
                      ctypes.POINTER(GtfEdges), ctypes.POINTER(GtfParams))
    L.gtf_extrapolate.argtypes = [G, N, S, E, PR, P, P]
    L.gtf_uts_materialize.argtypes = [G, S, P]
    L.gtf_update.argtypes = [G, N, S, S, E, PR, P, P]
    L.gtf_message_passing.argtypes = [G, N, S, E, PR, P, P]
    L.gtf_node_ops.argtypes = [G, N, S, S, E, PR, ctypes.POINTER(ctypes.c_int8), I32, F64, F64, P, P]
    L.gtf_cluster.argtypes = [G, N, S, E, I32, F64, F64, PR, P, P]
    L.gtf_pass.argtypes = [G, N, S, S, E, PR, P, P]
    L.gtf_pass_ev.argtypes = [G, N, S, S, E, PR, P, P, ctypes.POINTER(P)]
    L.gtf_tag_prepare.argtypes = [G, P, P, P, P, P]
    L.gtf_tag_sweep.argtypes = [G, P, P, P, P, P, P]
    L.gtf_tag_workspace_bytes.restype = ctypes.c_size_t
    L.gtf_tag_workspace_bytes.argtypes = [I32, I32]
    L.gtf_tag_propagate.argtypes = [G, P, P, F64, I32, P, ctypes.POINTER(ctypes.c_int32), P, ctypes.c_size_t, P]
    L.gtf_extract_workspace_bytes.restype = ctypes.c_size_t
    L.gtf_extract_workspace_bytes.argtypes = [I32, I32]
    L.gtf_extract_candidates.argtypes = [G, E, ctypes.POINTER(GtfExtractIO), ctypes.POINTER(GtfExtractParams), P, P]
    SH = ctypes.POINTER(GtfShard)
    L.gtf_pass_shard.argtypes = [G, N, S, S, E, PR, SH, P, P, ctypes.POINTER(P)]
    L.gtf_tag_sweep_shard.argtypes = [G, P, P, P, P, SH, I32, I32, P]
    L.gtf_shard_chunk_bytes.restype = ctypes.c_size_t
    L.gtf_shard_chunk_bytes.argtypes = [I32, I32]
    L.gtf_shard_pack.argtypes = [N, E, SH, I32, I32, P, P]
    L.gtf_shard_unpack.argtypes = [N, E, P, I32, I32, P, I32, I32, P]
    HA = ctypes.POINTER(GtfHalo)
    L.gtf_halo_pack.argtypes = [N, E, HA, P, P]
    L.gtf_halo_unpack.argtypes = [N, E, HA, P, P]
    L.gtf_track_state_estimates.argtypes = [G, S, ctypes.POINTER(GtfTseExtra), PR, P]
    L.gtf_parabolic_kl.argtypes = [ctypes.POINTER(GtfKlGraph), I32, ctypes.POINTER(GtfKlOut), P]
    L.gtf_build_event_csr.argtypes = [ctypes.POINTER(GtfEventCsr)]
    L.gtf_build_event_device_workspace_bytes.restype = ctypes.c_size_t
    L.gtf_build_event_device_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    L.gtf_build_event_csr_device.argtypes = [ctypes.POINTER(GtfEventCsr), P, ctypes.c_size_t, P]
    L.gtf_candidate_order.argtypes = [ctypes.POINTER(GtfCandidateGraph), P]
    L.gtf_updated_state_pair_counts.argtypes = [G, N, S, E, P, P]
    L.gtf_updated_state_distances.argtypes = [G, N, S, E, P, P, ctypes.POINTER(GtfPairOut), P]
    L.gtf_device_init.argtypes = [I32]
    L.gtf_malloc.argtypes = [ctypes.POINTER(P), ctypes.c_size_t]
    L.gtf_free.argtypes = [P]
    for fn in ("gtf_memcpy_htod", "gtf_memcpy_dtoh", "gtf_memcpy_dtod"):
        getattr(L, fn).argtypes = [P, P, ctypes.c_size_t, P]
    L.gtf_memset.argtypes = [P, I32, ctypes.c_size_t, P]
    L.gtf_stream_synchronize.argtypes = [P]
    I64 = ctypes.c_int64
    L.gtf_comm_unique_id.argtypes = [P]
    L.gtf_comm_init.argtypes = [ctypes.POINTER(P), I32, I32, P]
    L.gtf_comm_destroy.argtypes = [P]
    L.gtf_comm_rank.argtypes = [P]
    L.gtf_comm_size.argtypes = [P]
    L.gtf_halo_exchange.argtypes = [P, N, E, HA, HA, P, P, P, P, P]
    L.gtf_halo_alltoall.argtypes = [P, P, P, P, P, P]
    L.gtf_allreduce_max_i64.argtypes = [P, P, I64, P]
    L.gtf_allgather_bytes.argtypes = [P, P, P, I64, P]
    L.gtf_tag_shard_workspace_bytes.restype = ctypes.c_size_t
    L.gtf_tag_shard_workspace_bytes.argtypes = [I32, I32, I32]
    L.gtf_tag_propagate_shard.argtypes = [P, G, SH, P, P, F64, I32, P, ctypes.POINTER(ctypes.c_int32), P,
                                          ctypes.c_size_t, P]
    L.gtf_last_error.restype = ctypes.c_char_p
    L.gtf_version.restype = ctypes.c_char_p
    for fn in ("gtf_workspace_init", "gtf_uts_materialize", "gtf_clear_errors", "gtf_read_errors", "gtf_extrapolate", "gtf_update", "gtf_cluster", "gtf_pass",
               "gtf_pass_ev", "gtf_message_passing", "gtf_node_ops",
               "gtf_tag_prepare", "gtf_tag_sweep", "gtf_tag_sweep_shard", "gtf_parabolic_kl", "gtf_track_state_estimates", "gtf_pass_shard", "gtf_shard_pack",
               "gtf_shard_unpack", "gtf_halo_pack", "gtf_halo_unpack", "gtf_extract_candidates", "gtf_build_event_csr",
               "gtf_candidate_order", "gtf_updated_state_pair_counts", "gtf_updated_state_distances",
               "gtf_set_diagnostics", "gtf_build_event_csr_device", "gtf_device_init", "gtf_malloc", "gtf_free",
               "gtf_memcpy_htod", "gtf_memcpy_dtoh", "gtf_memcpy_dtod", "gtf_memset", "gtf_stream_synchronize",
               "gtf_comm_unique_id", "gtf_comm_init", "gtf_comm_destroy", "gtf_comm_rank", "gtf_comm_size",
               "gtf_halo_exchange", "gtf_halo_alltoall", "gtf_allreduce_max_i64", "gtf_allgather_bytes",
               "gtf_tag_propagate_shard"):
        getattr(L, fn).restype = ctypes.c_int
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise RuntimeError("libgtf: %s (rc=%d)" % ((_lib or lib()).gtf_last_error().decode(), rc))
