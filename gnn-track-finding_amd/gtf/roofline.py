"""Algorithmic bytes per kernel launch (SURVEY.md §8d byte model, fp64 SoA).

Per pass the survey prices B_alg = 183 B per directed edge + 290 B per node:
  * extrapolation side (k_sender_scan + k_extrapolate): 94 B per directed edge
    (read receiver index 4, activation 1, sender TSE mixture weight 8; write
    state 24, covariance 4 x 8 = 32, tau 8, likelihood 8, weight 8, activation 1)
    + 104 B per node (GNN coordinates 32, merged state 24, merged covariance 40,
    write-back of merged_cov[1,1] 8);
  * fused node kernel (priors, side norm, reweight x2, update, KL clustering):
    89 B per directed edge (re-read state 3 + 4 doubles = 56, sender coordinates
    32, deactivation 1) + 186 B per node (xyzr 32, flags/layer 2, merged outputs
    2 x (3 + 6) x 8 = 144, degree 8).
Sums: 183 E + 290 N. DESIGN.md "Roofline" states these figures.

Per kernel of gtf_pass (DESIGN.md "Roofline"):
  * k_sender + k_extrapolate: the extrapolation side above (94 E + 104 N);
  * k_node_multi<reweight/update> (priors, side norm, reweight x2, degree, prune,
    priors, reweight): 100 B per slot -- read rank 4, activation 1, weight 8,
    likelihood 8, prior 8, sender layer 8, stored x 8, TSE rank 4 and prior 8 (= 57,
    +1 reverse-edge flag = 58); write weight 8, prior 8, lr 8, side 1, edge weight 8,
    activation 1, TSE prior 8 (= 42) -- plus 6 B per node (flags, degree);
  * the clustering ops = the KL-distance work: SURVEY §8d's B_KL = 89 B per
    in-edge of an eligible node (3 <= |states| <= 15) + 176 B per eligible node.
  * gtf_pass runs both op sequences in ONE node launch (the fused node kernel, "the
    KL-distance kernel" of the bench line): reweight/update bytes + B_KL.

Parabolic-model KL kernel (gtf_parabolic_kl, §8 a17), minimal unique traffic:
  * 24 B per node of the batch (GNN x, y and truth id, read once: neighbours
    re-read them from cache);
  * 28 B per listed node (d >= 2): list entry 4, slot_ptr 4, pair_ptr 8, emp_var 8
    written, plus its own coordinates counted above;
  * 4 B per in-edge (slot_src);
  * 9 B per pair in fp64 (distance 8 + truth flag 1), 5 B in fp32.
"""

PKL_PER_NODE, PKL_PER_LISTED, PKL_PER_SLOT = 24, 28, 4
PKL_PER_PAIR = {"f64": 9, "f32": 5}

EXTRAP_PER_EDGE, EXTRAP_PER_NODE = 94, 104
REWEIGHT_PER_SLOT, REWEIGHT_PER_NODE = 100, 6
KL_PER_EDGE, KL_PER_NODE = 89, 176
NODE_PER_EDGE, NODE_PER_NODE = 89, 186
PASS_PER_EDGE, PASS_PER_NODE = 183, 290

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def extrap_bytes(n_edges, n_nodes):
    return EXTRAP_PER_EDGE * n_edges + EXTRAP_PER_NODE * n_nodes


def node_bytes(n_edges, n_nodes):
    return NODE_PER_EDGE * n_edges + NODE_PER_NODE * n_nodes


def reweight_bytes(n_slots, n_nodes):
    return REWEIGHT_PER_SLOT * n_slots + REWEIGHT_PER_NODE * n_nodes


def kl_bytes(e_elig, n_elig):
    return KL_PER_EDGE * e_elig + KL_PER_NODE * n_elig


def fused_node_bytes(n_slots, n_nodes, e_elig, n_elig):
    """The fused node kernel (gtf_pass): the reweight/update traffic of every slot plus
    the KL-distance traffic of the eligible nodes' in-edges (each read once)."""
    return reweight_bytes(n_slots, n_nodes) + kl_bytes(e_elig, n_elig)


def pass_bytes(n_edges, n_nodes):
    return PASS_PER_EDGE * n_edges + PASS_PER_NODE * n_nodes


def parabolic_kl_bytes(n_nodes, n_listed, n_slots, n_pairs, dtype="f64"):
    return (PKL_PER_NODE * n_nodes + PKL_PER_LISTED * n_listed + PKL_PER_SLOT * n_slots
            + PKL_PER_PAIR[dtype] * n_pairs)


# VALU issue roofline (the bound of the fp64 node-local work beside HBM): gfx950 has 256
# CUs x 4 SIMDs at ~2.4 GHz; a wave64 VALU instruction issues in 2 cycles on a 32-lane
# SIMD (MI355X_MICROARCH.md), an fp64 add / mul / fma / transcendental in 4 (fp64 runs at
# half the fp32 lane rate: 78.6 TFLOP/s).
SIMDS, CLOCK_HZ = 1024, 2.4e9
VALU_CYC, VALU_F64_CYC = 2, 4
F64_COUNTERS = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                "SQ_INSTS_VALU_TRANS_F64")


def valu_issue_floor_s(counters: dict) -> float:
    """Seconds the launch's VALU instructions need at full issue rate on every SIMD, from
    its SQ counters (per launch): fp64 instructions at 4 cycles, every other at 2."""
    f64 = sum(float(counters.get(k, 0.0)) for k in F64_COUNTERS)
    other = float(counters["SQ_INSTS_VALU"]) - f64
    return (f64 * VALU_F64_CYC + other * VALU_CYC) / (SIMDS * CLOCK_HZ)
