"""ctypes binding of oracle/cpu_ref.cpp (oracle/build/libcpuref.so, `make -C oracle`).

TEST INFRASTRUCTURE / CPU BASELINE ONLY: the C++ fp64 restatement of the fused pass
(oracle.full_pass, run_gnn_trackml_mod.sh:101,138,112 order) with OpenMP over senders
and receivers -- bench.py's all-cores CPU baseline and a second CPU
check of the fixtures (tests/test_cpu_ref.py). The product path never imports it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from gtf.graph import TrackGraph  # container only

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libcpuref.so")

P = ctypes.c_void_p


class CrGraph(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("n_slots", ctypes.c_int32)] + [
        (n, P) for n in ("slot_ptr", "slot_src", "out_ptr", "out_slot", "is_edge", "rev_edge", "solo", "gnn", "xyzr",
                         "layer", "has_merged", "merged_state", "merged_cov", "merged_prior", "has_tse", "has_uts",
                         "degree", "act", "edge_mw", "send_mw", "tse_rank", "tse_prior", "tse_sv", "tse_tau", "tse_cov",
                         "tse_xyzr", "tse_mw", "uts_rank", "uts_sv",
                         "uts_tau", "uts_cov", "uts_xyzr", "uts_lik", "uts_mw", "uts_prior", "uts_lr", "uts_side",
                         "uts_fresh")]


class CrParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("sigma0xy", "sigma0rz", "sigma0rz2", "endcap_boundary", "chi2_cut",
                                               "reweight_threshold", "cluster_chi2", "cluster_kl")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("%s missing: run `make -C oracle`" % LIB)
        _lib = ctypes.CDLL(LIB)
        _lib.cr_full_pass.restype = ctypes.c_uint32
        _lib.cr_full_pass.argtypes = [ctypes.POINTER(CrGraph), ctypes.POINTER(CrParams), ctypes.c_int]
        _lib.cr_cluster.restype = ctypes.c_uint32
        _lib.cr_cluster.argtypes = [ctypes.POINTER(CrGraph), ctypes.POINTER(CrParams), ctypes.c_int, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int]
    return _lib


class Bound:
    """a TrackGraph's arrays made contiguous with the library's dtypes, and the struct
    pointing at them (the pass then mutates the TrackGraph's own arrays)."""

    DT = {"slot_ptr": np.int32, "out_ptr": np.int32, "out_slot": np.int32}

    def __init__(self, g: TrackGraph):
        self.g = g
        keep = {}

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep[id(a)] = a
            return a.ctypes.data_as(P)

        N, S = g.node, g.slot
        if "solo" not in N:
            sizes = np.bincount(N["sub_id"] - N["sub_id"].min()) if g.n_nodes else np.zeros(0, np.int64)
            solo = (sizes[N["sub_id"] - N["sub_id"].min()] == 1).astype(np.uint8) if g.n_nodes else np.zeros(0, np.uint8)
        else:
            solo = N["solo"]
        for f, dt in (("has_merged", np.uint8), ("merged_state", np.float64), ("merged_cov", np.float64),
                      ("merged_prior", np.float64), ("has_tse", np.uint8), ("has_uts", np.uint8),
                      ("degree", np.int32)):
            N[f] = np.ascontiguousarray(N[f], dtype=dt)
        for f, dt in (("act", np.uint8), ("edge_mw", np.float64), ("tse_rank", np.int32), ("tse_prior", np.float64),
                      ("tse_sv", np.float64), ("tse_tau", np.float64), ("tse_cov", np.float64),
                      ("tse_xyzr", np.float64), ("tse_mw", np.float64),
                      ("uts_rank", np.int32), ("uts_sv", np.float64), ("uts_tau", np.float64),
                      ("uts_cov", np.float64), ("uts_xyzr", np.float64), ("uts_lik", np.float64),
                      ("uts_mw", np.float64), ("uts_prior", np.float64), ("uts_lr", np.float64),
                      ("uts_side", np.int8), ("uts_fresh", np.uint8)):
            S[f] = np.ascontiguousarray(S[f], dtype=dt)
        self.c = CrGraph(
            g.n_nodes, g.n_slots, arr(g.slot_ptr, np.int32), arr(S["slot_src"], np.int32), arr(g.out_ptr, np.int32),
            arr(g.out_slot, np.int32), arr(S["is_edge"], np.uint8), arr(S["rev_edge"], np.uint8),
            arr(solo, np.uint8), arr(N["gnn"], np.float64), arr(N["xyzr"], np.float64), arr(N["layer"], np.float64),
            *[N[f].ctypes.data_as(P) for f in ("has_merged", "merged_state", "merged_cov", "merged_prior", "has_tse",
                                              "has_uts", "degree")],
            S["act"].ctypes.data_as(P), S["edge_mw"].ctypes.data_as(P), arr(S["send_mw"], np.float64),
            *[S[f].ctypes.data_as(P) for f in ("tse_rank", "tse_prior", "tse_sv", "tse_tau", "tse_cov", "tse_xyzr",
                                              "tse_mw", "uts_rank", "uts_sv", "uts_tau", "uts_cov",
                                              "uts_xyzr", "uts_lik", "uts_mw", "uts_prior", "uts_lr", "uts_side",
                                              "uts_fresh")])
        self._keep = keep


def params(p) -> CrParams:
    return CrParams(p.sigma0xy, p.sigma0rz, p.sigma0rz2, p.endcap_boundary, p.chi2_cut, p.reweight_threshold,
                    p.cluster_chi2, p.cluster_kl)


def full_pass(g: TrackGraph, p, threads: int = 0) -> int:
    """the fused pass in place on g; returns the GTF_ERR_* flags (the places where the
    reference raises). threads <= 0: OpenMP's default (all cores)."""
    b = Bound(g)
    cp = params(p)
    return int(lib().cr_full_pass(ctypes.byref(b.c), ctypes.byref(cp), int(threads)))


def cluster(g: TrackGraph, key: str, chi2: float, kl: float, p, threads: int = 0) -> int:
    """clustering.cluster's body on one dict ("tse" / "uts") in place; returns the flags"""
    b = Bound(g)
    cp = params(p)
    return int(lib().cr_cluster(ctypes.byref(b.c), ctypes.byref(cp), 1 if key == "uts" else 0, float(chi2),
                                float(kl), int(threads)))
