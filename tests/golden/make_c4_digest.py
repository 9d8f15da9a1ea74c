"""Full-size parity digest of the benchmark workload C4 (BASELINE configs[3]).

    python tests/golden/make_c4_digest.py        # ~4 min on 4 cores; writes tests/golden/c4_digest.npz

The oracle (oracle/gtf_oracle.py, itself pinned to the reference's own outputs by
tests/test_oracle_golden.py) runs the fused pass -- extrapolate stage, update stage,
clustering on updated_track_states (oracle.full_pass, run_gnn_trackml_mod.sh:101,138,112
order) -- on the seeded C4 event (gtf.synth.workload("c4", seed=0): 179,788 hits,
1,027,548 directed edges), and three more times with the continuous inputs scaled by
(1 + U(-2^-46, 2^-46)) (tests/compare.py noise_envelope). The full outputs are ~100 MB,
so the committed file holds a digest (< 2 MB):

  * the activation mask of every slot, has_merged / has_uts of every node (bit-packed),
    every node's degree and every slot's dense updated_track_states position (dict
    membership and order), all exact;
  * the undetermined positions: decisions that flip under the ulp perturbation, and
    every mask of a node whose decision reads a state whose own perturbation noise
    exceeds 1e-6 (compare.compare_noise's rule);
  * float outputs with their perturbation noise at a seeded 1 % sample of the present
    updated_track_states entries and of the merged nodes;
  * a SHA-256 of the generator's output, so a changed generator fails loudly instead of
    comparing against the wrong event.

tests/test_gpu_c4_digest.py compares the HIP pass with this digest.
"""
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "gnn-track-finding_amd"), os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

OUT = os.path.join(HERE, "c4_digest.npz")
SEED = 0
REL = 2.0 ** -46
N_PERTURB = 3
SAMPLE = 0.01
RTOL = 1e-6

FLOAT_SLOT = ["uts_sv", "uts_cov", "uts_tau", "uts_lik", "uts_mw", "uts_prior", "edge_mw"]
FLOAT_NODE = ["merged_state", "merged_cov", "merged_prior"]
KEEP_SLOT = FLOAT_SLOT + ["act", "uts_rank"]
KEEP_NODE = FLOAT_NODE + ["has_merged", "has_uts", "degree"]


def _run(i):
    import gtf_oracle as O
    from compare import perturbed
    from gtf import synth
    from gtf.params import Params
    g = synth.workload("c4", seed=SEED)
    if i > 0:
        g = perturbed(g, REL, 1000 + i - 1)
    t0 = time.time()
    O.full_pass(g, Params(), tie_policy="stop")
    print("run %d: %.0f s" % (i, time.time() - t0), flush=True)
    return {"node": {k: g.node[k] for k in KEEP_NODE}, "slot": {k: g.slot[k] for k in KEEP_SLOT}}


def main():
    from compare import dense_ranks, input_sha
    from gtf import synth
    g = synth.workload("c4", seed=SEED)
    with mp.get_context("fork").Pool(1 + N_PERTURB) as pool:
        outs = pool.map(_run, range(1 + N_PERTURB))
    ref = outs[0]
    dst = g.slot_dst()
    S, Nn = g.n_slots, g.n_nodes

    def dense(o):
        x = g.copy()
        x.slot["uts_rank"] = o["slot"]["uts_rank"]
        return dense_ranks(x, "uts_rank")

    rank0 = dense(ref)
    noise = {}
    for kind, fields in (("slot", FLOAT_SLOT), ("node", FLOAT_NODE)):
        for f in fields:
            b = ref[kind][f]
            nz = np.zeros_like(b)
            for o in outs[1:]:
                a = o[kind][f]
                d = np.abs(a - b)
                d = np.where(np.isnan(a) & np.isnan(b), 0.0, d)
                d = np.where(np.isnan(d), np.inf, d)
                np.maximum(nz, d, out=nz)
            noise[f] = nz
    flip_act = np.zeros(S, bool)
    flip_rank = np.zeros(S, bool)
    flip_hm = np.zeros(Nn, bool)
    flip_hu = np.zeros(Nn, bool)
    flip_deg = np.zeros(Nn, bool)
    for o in outs[1:]:
        flip_act |= o["slot"]["act"] != ref["slot"]["act"]
        flip_rank |= dense(o) != rank0
        flip_hm |= o["node"]["has_merged"] != ref["node"]["has_merged"]
        flip_hu |= o["node"]["has_uts"] != ref["node"]["has_uts"]
        flip_deg |= o["node"]["degree"] != ref["node"]["degree"]
    present = ref["slot"]["uts_rank"] >= 0
    ill_slot = np.zeros(S, bool)
    for f in ("uts_sv", "uts_cov"):
        ill_slot |= (noise[f] > RTOL * np.abs(ref["slot"][f])).any(axis=1) & present
    ill_node = np.zeros(Nn, bool)
    ill_node[dst[ill_slot]] = True
    und_slot = ill_node[dst]
    und_node = ill_node.copy()
    # a node with any flipping input decision: all its masks are undetermined too
    und_node[dst[flip_act | flip_rank]] = True
    und_node |= flip_hm | flip_hu | flip_deg
    und_slot |= und_node[dst] | flip_act | flip_rank

    rng = np.random.default_rng(12345)
    ps = np.nonzero(present & ~und_slot)[0]
    sidx = np.sort(rng.choice(ps, max(1, int(SAMPLE * ps.size)), replace=False)).astype(np.int32)
    pm = np.nonzero((ref["node"]["has_merged"] == 1) & ~und_node)[0]
    nidx = np.sort(rng.choice(pm, max(1, int(SAMPLE * pm.size)), replace=False)).astype(np.int32)

    out = {
        "input_sha": np.array(input_sha(g)),
        "n_nodes": np.int64(Nn), "n_slots": np.int64(S),
        "act_bits": np.packbits(ref["slot"]["act"].astype(bool)),
        "has_merged_bits": np.packbits(ref["node"]["has_merged"].astype(bool)),
        "has_uts_bits": np.packbits(ref["node"]["has_uts"].astype(bool)),
        "degree": ref["node"]["degree"].astype(np.uint16),
        "uts_dense_rank": rank0.astype(np.int16),
        "und_slot_bits": np.packbits(und_slot),
        "und_node_bits": np.packbits(und_node),
        "sample_slot": sidx, "sample_node": nidx,
        "stats": np.array(str({"undetermined_slots": int(und_slot.sum()), "undetermined_nodes": int(und_node.sum()),
                               "flipping_act": int(flip_act.sum()), "flipping_rank": int(flip_rank.sum()),
                               "flipping_has_merged": int(flip_hm.sum()), "ill_nodes": int(ill_node.sum()),
                               "active_edges": int(ref["slot"]["act"].sum()),
                               "merged_nodes": int(ref["node"]["has_merged"].sum()),
                               "uts_entries": int(present.sum())})),
    }
    for f in FLOAT_SLOT:
        out["slot__" + f] = ref["slot"][f][sidx]
        out["noise__" + f] = noise[f][sidx]
    for f in FLOAT_NODE:
        out["node__" + f] = ref["node"][f][nidx]
        out["noise__" + f] = noise[f][nidx]
    np.savez_compressed(OUT, **out)
    print(str(out["stats"]))
    print("wrote %s (%.2f MB)" % (OUT, os.path.getsize(OUT) / 1e6))


if __name__ == "__main__":
    main()
