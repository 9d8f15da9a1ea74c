/*
 * gtf.h -- C-ABI of libgtf.so, the MI355X (gfx950) edge-parallel track-finding
 * pass that drops in behind nishalad95/GNN-track-finding's hot path.
 *
 * Every pointer in the structs below is a DEVICE pointer (HBM) owned by the
 * caller; the library keeps no pointer after a call returns and allocates
 * nothing on the hot path (scratch comes from the caller's workspace). All
 * calls are stream-ordered on the hipStream_t passed in (0 = null stream).
 * Return value: 0 = OK, < 0 = error (gtf_last_error() has the message).
 * Reference-semantics exceptions detected on the device (the places where the
 * reference itself raises) are reported as bit flags in the workspace error
 * word; read them with gtf_read_errors().
 *
 * Which reference interface each entry point replaces (file:line in the
 * reference repository):
 *   gtf_extrapolate  -> src/extrapolate/extrapolate_merged_states.py:552-566
 *                       (message_passing :406-451 + extrapolate_validate :26-402,
 *                        compute_prior_probabilities + reweight x2, node degree)
 *   gtf_update       -> src/update/remove_state_metadata.py:29-53
 *   gtf_cluster      -> src/clustering/clustering.py:181-373 (cluster body)
 *   gtf_pass         -> the three above back to back, one fused node kernel
 *                       (run_gnn_trackml_mod.sh:101,138,112 stage order)
 *   gtf_tag_sweep    -> tag_propagation/tag_propagation.py:137-164 (one sweep)
 *   gtf_tag_prepare  -> tag_propagation/tag_propagation.py:97-110
 *   gtf_tag_propagate -> tag_propagation/tag_propagation.py:97-164 (the whole stage)
 *   gtf_tag_sweep_shard -> one sweep (:137-164) on an edge-sharded event
 *   gtf_comm_*, gtf_halo_exchange, gtf_halo_alltoall, gtf_allreduce_max_i64, gtf_allgather_bytes,
 *   gtf_tag_propagate_shard -> no reference counterpart: the collectives of one event
 *                       sharded over the GPUs of a node, in place of the
 *                       serial subgraph loop src/extrapolate/extrapolate_merged_states.py:406-451
 *   gtf_updated_state_distances -> calculate_distance_between_updated_states/
 *                       calculate_distance_between_updated_track_states.py:27-104,134-195
 */
#ifndef GTF_H
#define GTF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* gtf_stream_t; /* a hipStream_t */

/* Version of the struct layouts below. gtf_graph carries it with its own size, and every
 * entry point taking a gtf_graph refuses a caller built against another layout
 * (status -3, gtf_last_error() names both). Bumped on every layout change. */
#define GTF_ABI_VERSION 7u

/* ---- graph structure (read-only on the path) ------------------------------ */
typedef struct gtf_graph {
    uint32_t struct_size;     /* sizeof(gtf_graph) as the caller compiled it */
    uint32_t abi_version;     /* GTF_ABI_VERSION */
    int32_t n_nodes;
    int32_t n_slots;          /* slots = (receiver, sender) pairs, receiver-major */
    int32_t n_edges;          /* directed edges = slots with is_edge == 1 */
    int32_t n_big;            /* schedule entries after the lane-group buckets (> 64 slots) */
    const int32_t* slot_ptr;  /* [N+1] slot segment of each receiver */
    const int32_t* slot_src;  /* [S]   sender node index, -1 = orphan state key */
    const int32_t* slot_dst;  /* [S]   receiver node index */
    const int32_t* out_ptr;   /* [N+1] out-edge segment of each sender */
    const int32_t* out_slot;  /* [E]   slot of each out-edge, successor order */
    const int32_t* slot_outpos; /* [S] position of the slot's edge in its sender's out-list (-1 = none) */
    const uint8_t* is_edge;   /* [S]   edge sender->receiver exists */
    const uint8_t* rev_edge;  /* [S]   edge receiver->sender exists */
    const uint8_t* solo;      /* [N]   node is alone in its subgraph */
    const double*  gnn;       /* [N*4] GNN_Measurement x,y,z,r */
    const double*  xyzr;      /* [N*4] node attribute 'xyzr' */
    const double*  layer;     /* [N]   in_volume_layer_id */
    /* optional node schedule for the node-local stages (NULL = one thread per node):
     * node indices bucketed by slot count -- n_g4 nodes with <= 4 slots (n_g4 is the LAST
     * field of this struct, added after the others), then n_g8 nodes with <= 8 slots,
     * n_g16 with 9..16, n_g32 with 17..32, n_g64 with 33..64 (a group of that many lanes
     * per node), then n_big nodes with more slots (one thread per node). Built once per
     * graph (gtf/device.py); a shard's graph view holds the schedule of its own receivers. */
    const int32_t* sched;     /* [N] */
    int32_t n_g8;
    int32_t n_g16;
    int32_t n_g32;
    int32_t n_g64;
    const int32_t* out_dst;   /* [E] receiver of each out-edge = slot_dst[out_slot] (saves the sender
                                 scan a dependent gather), or NULL */
    const double* slot_layer; /* [S] layer of each slot's sender (NaN for orphans) = layer[slot_src]:
                                 a coalesced read in the node kernels instead of a gather, or NULL */
    int32_t n_g4;             /* schedule entries before the n_g8 bucket: nodes with <= 4 slots
                                 (4 lanes per node; 0 = none, the n_g8 bucket then starts at 0) */
    const int32_t* sched_seg; /* [2*len(sched)] slot segment (slot_ptr[v], slot_ptr[v+1]) of each
                                 schedule entry v, read beside it: the node kernels then reach the
                                 slots without a dependent slot_ptr gather; or NULL */
    /* optional sender schedule for the var_ms scan (NULL = 8 lanes for every node): one
     * (sender, out_ptr[sender], out_ptr[sender+1], 0) int32 quadruple per sender with an
     * out-edge -- n_o4 senders with 1..4 out-edges (4 lanes each), then n_o8 with 5..8
     * (8 lanes), then n_o16 with more (16 lanes). Not used by gtf_pass_shard. */
    const int32_t* out_sched;  /* [4*(n_o4+n_o8+n_o16)] */
    int32_t n_o4;
    int32_t n_o8;
    int32_t n_o16;
    int32_t n_g2;             /* the first n_g2 entries of the n_g4 bucket have <= 2 slots and run on
                                 2 lanes per node in gtf_pass / the node ops (0 = all on 4 lanes) */
    /* optional packed schedule for gtf_pass's node kernel (replaces the lane-group buckets
     * there; the > 64-slot nodes still come from sched): wavefront w takes the entries
     * [pack_wave[w], pack_wave[w+1]) of pack_ent, each (v, slot_ptr[v], slot_ptr[v+1], first
     * lane) as int32 quadruples, one lane per slot (one for a slot-free node), <= 64 lanes. */
    const int32_t* pack_ent;  /* [4*n_entries] */
    const int32_t* pack_wave; /* [n_pack_waves+1] */
    int32_t n_pack_waves;
    /* optional per-lane view of out_sched's 4- and 8-lane buckets (v3): for lane l of entry e
     * of those buckets, (out_slot[o], receiver of o) with o = out_ptr[sender] + l, or (-1, 0)
     * past the sender's last out-edge, as int32 pairs -- the scan then reads each lane's edge
     * beside the schedule entry instead of after it (one dependent round of loads fewer).
     * [2 * (4 * n_o4 + 8 * n_o8)], or NULL. */
    const int32_t* out_lanes;
    /* optional padded tile layout of the node kernel (v3; gtf.graph.padded): the nodes of
     * each lane-group size G = 2, 4, 8, 16, 32, 64 own exactly G slots (their own, then inert
     * padding slots: orphan, no edge, rank -1 in both dicts), and each of pad_tiles tiles
     * holds pad_count[j] nodes of group j, groups in that order: node (t, j, i) is
     * t * pad_tile_nodes + sum(pad_count[:j]) + i, its slots start at t * pad_tile_slots +
     * sum(pad_count[:j] * G[:j]) + i * G[j]. Built with -DGTF_PAD_ARITH=1, gtf_pass's node
     * kernel then finds every node and slot by arithmetic (no schedule loads); the default
     * build reads the schedule (sched must list the nodes either way: the other entry points
     * and the > 64-slot nodes use it). pad_tiles = 0: none. */
    int32_t pad_tiles;
    int32_t pad_tile_nodes;
    int32_t pad_tile_slots;
    int32_t pad_count[6];
    int32_t pad_reserved_;
    /* optional (v4): global out-edge index of each slot's edge, out_ptr[slot_src] + slot_outpos
     * (-1 = no edge), or NULL. With it the sender scan stores the running merged_cov[1,1]
     * each extrapolation sees in out-edge order (contiguous per sender, coalesced stores)
     * and the extrapolation reads it through this index; NULL: stored by slot. [S] */
    const int32_t* slot_outidx;
    /* optional (v5): graph-static partitions of every receiver's slot segment, built once per
     * graph (gtf/device.py) so the node kernel does not rebuild them in every pass. For slot
     * k at position i of a segment of d <= 32 slots: bits 0..31 = the positions j of the
     * segment whose sender has slot k's sender layer (layer[slot_src], compute_prior_
     * probabilities' groups, helper.py:30-63; an orphan or NaN layer: {i}); bits 32..63 = the
     * positions whose sender's GNN_Measurement x equals slot k's sender's (the side norm's
     * distinct-x classes, helper.py:111-139, for entries whose stored x is the sender's live
     * GNN x -- see gtf_states.fresh); for a segment of 33..64 slots (v7) all 64 bits are the
     * same-layer positions and slot_xclass holds the same-x ones; 0 for larger segments. [S], or NULL
     * (the kernel then builds the classes itself). */
    const uint64_t* slot_class;
    /* optional (v5, with slot_class): bit 0 = the sender's GNN x < the receiver's GNN x (the
     * side of a live entry, helper.py:116-121). [S], or NULL. */
    const uint8_t* slot_sflags;
    /* optional (v7): the GNN_Measurement x, z, r of each slot's sender (gnn[4 slot_src + 0, 2, 3],
     * NaN for an orphan key), graph-static like slot_class. The coordinates of a live UTS entry
     * (gtf_states.fresh bit 1, extrapolate_merged_states.py:377) are its sender's GNN ones; the
     * node kernel's clustering stage (the tau geometry of the pairwise chi2, clustering.py:
     * 49-57) and the side norm read them here, contiguously per slot, instead of gathering the
     * sender's 32-byte gnn row per state. A caller that changes g->gnn refreshes it (or passes
     * NULL: the kernel then gathers gnn). [S*3], or NULL. */
    const double* slot_sxzr;
    /* optional (v7): one 32-bit word per slot of a receiver segment of d <= 8 slots, read by the
     * node kernel's lane groups of <= 8 lanes in place of four loads: bits 0..7 = slot_class bits
     * 0..7 (the same-layer positions), bits 8..15 = slot_class bits 32..39 (the same-x
     * positions), bit 16 = is_edge, bit 17 = rev_edge, bit 18 = slot_sflags bit 0; 0 for larger
     * segments. Graph-static, built with slot_class. [S], or NULL. */
    const uint32_t* slot_static;
    /* optional (v7, with slot_class): the same-x positions of the slots of 33..64-slot segments
     * (64 bits; slot_class then holds all 64 same-layer bits there), so the 64-lane groups read
     * their classes too instead of electing leaders per distinct value; 0 elsewhere. [S], or
     * NULL. */
    const uint64_t* slot_xclass;
} gtf_graph;

/* ---- per-node mutable state ------------------------------------------------ */
typedef struct gtf_nodes {
    uint8_t* has_merged;      /* [N] */
    double*  merged_state;    /* [N*3] a, b, c */
    double*  merged_cov;      /* [N*5] c00 c01 c10 c11 c22 (block diagonal) */
    double*  merged_prior;    /* [N] */
    uint8_t* has_tse;         /* [N] node has a 'track_state_estimates' dict */
    uint8_t* has_uts;         /* [N] node has an 'updated_track_states' dict */
    int32_t* degree;          /* [N] */
} gtf_nodes;

/* ---- one state dict (track_state_estimates or updated_track_states) -------- */
typedef struct gtf_states {
    int32_t* rank;            /* [S] dict position, -1 = key absent */
    double*  sv;              /* [S*3] edge_state_vector a, b, c */
    double*  tau;             /* [S]   joint_vector[2] */
    double*  cov;             /* [S*5] c00 c01 c10 c11 c22 */
    double*  xyzr;            /* [S*4] sender coordinates stored in the state */
    double*  lik;             /* [S]   likelihood (UTS only) */
    double*  mw;              /* [S]   mixture_weight */
    double*  prior;           /* [S]   prior */
    double*  lr;              /* [S]   lr_layer_norm (UTS only) */
    int8_t*  side;            /* [S]   0 left, 1 right (UTS only) */
    uint8_t* fresh;           /* [S]   UTS only: bit 0 = entry written by the last message passing;
                                 bit 1 = the entry's xyzr is its sender's live GNN coordinates
                                 gnn[slot_src] (extrapolate_merged_states.py:377 stores exactly
                                 those), so xyzr[k] itself is not written -- gtf_uts_materialize
                                 writes it (before a caller mutates g->gnn or reads uts->xyzr) */
} gtf_states;

/* ---- per-edge attributes (stored per slot) --------------------------------- */
typedef struct gtf_edges {
    uint8_t*      act;        /* [S] 'activated' */
    double*       edge_mw;    /* [S] edge 'mixture_weight' */
    const double* send_mw;    /* [S] sender's track_state_estimates[receiver]['mixture_weight'] */
} gtf_edges;

typedef struct gtf_params {
    double sigma0xy;          /* -e */
    double sigma0rz;          /* -z */
    double sigma0rz2;         /* -m */
    double endcap_boundary;   /* -b */
    double chi2_cut;          /* extrapolation gate -c (extrapolate_merged_states.py:298) */
    double reweight_threshold;/* 0.1 (helper.py:145) */
    double cluster_chi2;      /* clustering -c (clustering.py:228) */
    double cluster_kl;        /* clustering -k (clustering.py:261) */
} gtf_params;

/* Device-detected reference exceptions (bit flags in the error word). */
enum {
    GTF_ERR_SEND_MW_MISSING = 1,   /* KeyError extrapolate_merged_states.py:384 */
    GTF_ERR_STALE_KEY_NO_EDGE = 2, /* KeyError helper.py:131/138 */
    GTF_ERR_ALL_ZERO_DIST = 4,     /* ValueError clustering.py:120 (np.min of empty) */
    GTF_ERR_TIE_EMPTIED = 8,       /* ValueError clustering.py:116 (tie removed every state) */
    GTF_ERR_EMPTY_DICT_MW = 16,    /* ZeroDivisionError helper.py:90 */
    GTF_ERR_NAN_KL = 32,           /* ValueError clustering.py:117 (list.index of NaN) */
    GTF_ERR_NO_STATE_DICT = 64,    /* KeyError remove_state_metadata.py:39 */
    GTF_ERR_SINGULAR_H = 128,      /* LinAlgError learn_KL_parabolic_model/.../utils.py:277 (x_B = 0 or x_B = x_0) */
    GTF_ERR_PAIR_COUNT = 256,      /* pair_ptr disagrees with the state dicts (caller error, a15) */
    GTF_ERR_NEIGHBOUR_MISSING = 512, /* KeyError calculate_distance_between_updated_track_states.py:182-183 */
    GTF_ERR_TOO_MANY_STATES = 1024 /* a15: a node with more than 2048 updated states (not processed) */
};

/* Workspace: caller allocates gtf_workspace_bytes() bytes of device memory and initialises
 * it once with gtf_workspace_init (or allocates it zeroed). Its first 8448 bytes are a
 * header: the error word at offset 0, the gtf_diag record at GTF_DIAG_OFFSET, and from byte
 * 256 the fused node kernel's work-queue counters (the kernel leaves them zero at the end of
 * every launch; only gtf_workspace_init or a zeroed allocation sets them up). One pass at a
 * time per workspace. */
size_t gtf_workspace_bytes(int32_t n_nodes, int32_t n_slots);

/* Zero the whole header (stream-ordered): no error flags, no diagnostics registered.
 * Required once on a workspace that was not allocated zeroed (hipMalloc): the kernels write
 * through every non-NULL gtf_diag pointer they find there. */
int gtf_workspace_init(void* workspace, gtf_stream_t stream);

/* Zero the error word only (stream-ordered); the registered diagnostics stay. */
int gtf_clear_errors(void* workspace, gtf_stream_t stream);

/* ---- Optional diagnostics outputs (SURVEY §5 "Metrics / logging"), off by default ----
 * The reference prints per-edge chi2 values to CSV files (extrapolate_merged_states.py
 * :143-172, the xy-plane chi2 of :134-140 is the one its gate uses) and raises exceptions
 * that abort a whole stage (the GTF_ERR_* places). Registered in the workspace by
 * gtf_set_diagnostics (NULL = all off), the pass kernels of that workspace then write:
 *   node_err[v]  |= the GTF_ERR_* bits of every reference exception node v raised
 *                  (gtf_pass / gtf_extrapolate / gtf_update / gtf_cluster / gtf_node_ops);
 *                  caller-zeroed uint32 [N]: which node (so which subgraph) would raise;
 *   edge_chi2[k]  = chi2 of the extrapolation of slot k's edge (every active out-edge of a
 *                  merged sender, accepted or not; untouched elsewhere), double [S];
 *   slot_cluster  = which states each clustered node merged and which it left (below).
 * The truth-based confusion counts of the reference's printouts (helper.py:186-225,
 * extrapolate_merged_states.py:496-518, clustering.py:342-369) follow on the host from
 * the masks (gtf/diagnostics.py). Nothing here is on the timed path: with no diagnostics
 * registered a kernel reads one uniform pointer. */
#define GTF_DIAG_OFFSET 64
typedef struct gtf_diag {
    uint32_t* node_err;       /* [N] device, or NULL */
    double*   edge_chi2;      /* [S] device, or NULL */
    uint8_t*  slot_cluster;   /* [S] device, or NULL: for every node that clustered (gtf_cluster,
                                 gtf_pass), 1 on the slots of the states merged into its merged
                                 state (clustering.py's edges_to_remain_active), 2 on the states
                                 left over, whose in-edges it deactivates (edges_to_deactivate);
                                 untouched elsewhere (caller-zeroed) */
    void*     reserved_[5];   /* zero */
} gtf_diag;
int gtf_set_diagnostics(void* workspace, const gtf_diag* d, gtf_stream_t stream);
/* Copy the error word to the host (synchronises the stream). */
int gtf_read_errors(void* workspace, uint32_t* flags, gtf_stream_t stream);

int gtf_extrapolate(const gtf_graph* g, gtf_nodes* n, gtf_states* uts, gtf_edges* e,
                    const gtf_params* p, void* workspace, gtf_stream_t stream);
/* message passing alone (extrapolate_merged_states.py:406-451): extrapolation of every
 * merged state along active out-edges, gate, Kalman update, UTS dict insertion
 * (GTF_OP_FRESH then GTF_OP_RANKS in the node kernel). */
int gtf_message_passing(const gtf_graph* g, gtf_nodes* n, gtf_states* uts, gtf_edges* e,
                        const gtf_params* p, void* workspace, gtf_stream_t stream);

/* Node-local helper operations, run in the given order for every node in one launch. */
enum {
    GTF_OP_RANKS = 1,        /* append keys created by message passing to the UTS dict */
    GTF_OP_PRIORS_TSE = 2,   /* helper.compute_prior_probabilities(.., 'track_state_estimates') :30-63 */
    GTF_OP_PRIORS_UTS = 3,   /* helper.compute_prior_probabilities(.., 'updated_track_states') */
    GTF_OP_REWEIGHT_UTS = 4, /* helper.reweight(.., 'updated_track_states') :143-225 */
    GTF_OP_DEGREE = 5,       /* node 'degree' = helper.query_node_degree_in_edges :67-73 */
    GTF_OP_PRUNE = 6,        /* remove_state_metadata.py:31-48 */
    GTF_OP_MW_TSE = 7,       /* helper.compute_mixture_weights(.., 'track_state_estimates') :76-96 */
    GTF_OP_MW_UTS = 8,
    GTF_OP_CLUSTER_TSE = 9,  /* clustering.py:197-321 on track_state_estimates */
    GTF_OP_CLUSTER_UTS = 10,
    GTF_OP_FRESH = 11        /* the entries message passing (re)wrote (uts.fresh): mixture_weight =
                                the sender's TSE weight (extrapolate_merged_states.py:384), prior / lr /
                                side absent; gtf_message_passing / gtf_extrapolate / gtf_pass run it */
};
/* ops: host array of n_ops (<= 24) GTF_OP_* codes; thresholds used by the cluster ops. */
int gtf_node_ops(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                 const gtf_params* p, const int8_t* ops, int32_t n_ops, double chi2_threshold,
                 double kl_threshold, void* workspace, gtf_stream_t stream);
int gtf_update(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
               const gtf_params* p, void* workspace, gtf_stream_t stream);
/* key: 0 = cluster track_state_estimates, 1 = updated_track_states. Where a
 * distance tie empties the state list the reference raises ValueError; here the
 * node keeps the merged state formed so far and GTF_ERR_TIE_EMPTIED is set. */
int gtf_cluster(const gtf_graph* g, gtf_nodes* n, gtf_states* states, gtf_edges* e, int32_t key,
                double chi2_threshold, double kl_threshold, const gtf_params* p, void* workspace,
                gtf_stream_t stream);
/* Write gnn[slot_src] into uts->xyzr of every entry whose xyzr is live (uts->fresh bit 1) and
 * clear that bit: the stored snapshot extrapolate_merged_states.py:377 makes. Call it before
 * mutating g->gnn (extraction's close-proximity merge, extract_track_candidates.py:111-118)
 * and before reading uts->xyzr back. */
int gtf_uts_materialize(const gtf_graph* g, gtf_states* uts, gtf_stream_t stream);

/* extrapolate -> update -> cluster(updated_track_states, p->cluster_chi2, p->cluster_kl) */
int gtf_pass(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
             const gtf_params* p, void* workspace, gtf_stream_t stream);
/* gtf_pass with hipEvent_t events[5] recorded on the stream before the sender scan,
 * after it, after the edge extrapolation kernel, after the fused node kernel (priors,
 * reweights, update and KL clustering in one launch) and at the end of the pass
 * (per-kernel timing for the roofline report; events may be NULL). */
int gtf_pass_ev(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                const gtf_params* p, void* workspace, gtf_stream_t stream, void* const* events);

/* ---- One event sharded across GPUs --------------------------------
 * Rank r owns a contiguous receiver range [node_lo, node_hi) and so the contiguous slot
 * range [slot_lo, slot_hi) (slots are receiver-major); every rank holds the whole graph.
 * gtf_pass_shard runs the pass for the owned receivers: the sender scan over `senders`
 * (every sender with an out-edge into an owned receiver, plus the owned senders whose
 * merged_cov write-back the rank publishes), extrapolation of the owned slots, and the
 * node kernels over the owned receivers (pass `g` with sched, n_g8..n_g64 and n_big describing the
 * owned receivers only; with g->out_sched set, the scan runs on that out-degree-bucketed
 * schedule of the shard's senders). Between passes the ranks exchange what the next pass
 * reads: the halo (gtf_halo_pack -> all-to-all -> gtf_halo_unpack, below), or every owned
 * state (gtf_shard_pack -> an all-gather of equal-size chunks -> gtf_shard_unpack: full
 * replicas, used before reading results back). */
typedef struct gtf_shard {
    const int32_t* senders;   /* [n_senders] device */
    int32_t n_senders;
    int32_t node_lo, node_hi;
    int32_t slot_lo, slot_hi;
    /* ABI v6: the pass in phases, so the halo exchange can overlap the part that does not
     * read it (gtf.shard.ShardedDeviceGraph.step). phases = 0 (or 3): the whole pass; 1: the
     * sender scan over `senders` and the extrapolation only; 2: the node kernels only; 5 (1 |
     * 4): phase 1 fused sender-major -- every out-edge of `senders` into [slot_lo, slot_hi)
     * extrapolated by its scan lane right after the scan (one launch; needs g->out_sched;
     * slot_list unused).
     * slot_list (device, ascending, [n_slot_list]) or NULL: phase 1 extrapolates exactly these
     * owned slots instead of [slot_lo, slot_hi). A rank's pass as two phase-1 calls (the
     * senders whose state and out-edge activations are all its own, with the slots they
     * send to; then the rest, after the exchange) and one phase-2 call equals the one-call
     * pass bit for bit: every sender is scanned once, in its own successor order, and every
     * owned slot extrapolated once. */
    int32_t phases;
    const int32_t* slot_list;
    int32_t n_slot_list;
    int32_t pad_;
} gtf_shard;

int gtf_pass_shard(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                   const gtf_params* p, const gtf_shard* shard, void* workspace, gtf_stream_t stream,
                   void* const* events);
/* bytes of one rank's chunk holding up to cap_nodes node states and cap_slots activations */
size_t gtf_shard_chunk_bytes(int32_t cap_nodes, int32_t cap_slots);
/* write the owned nodes' has_merged / merged_state / merged_cov / merged_prior and the
 * owned slots' activation into chunk (device) */
int gtf_shard_pack(const gtf_nodes* n, const gtf_edges* e, const gtf_shard* shard, int32_t cap_nodes,
                   int32_t cap_slots, void* chunk, gtf_stream_t stream);
/* scatter the chunks of all ranks except `self` (gathered: nranks chunks back to back);
 * ranges: device int32 [4 * nranks] = node_lo, node_hi, slot_lo, slot_hi per rank */
int gtf_shard_unpack(gtf_nodes* n, gtf_edges* e, const void* gathered, int32_t nranks, int32_t self,
                     const int32_t* ranges, int32_t cap_nodes, int32_t cap_slots, gtf_stream_t stream);

/* Halo exchange (the per-pass exchange of gtf/shard.py): only what the other ranks' next
 * pass reads -- the merged state of their halo senders owned here, and the activation
 * of the out-edges of their senders whose receivers are owned here -- instead of every
 * owned state. The lists are built once per plan (host); per pass a rank packs one
 * buffer of per-destination segments, exchanges it with one all-to-all (RCCL over
 * xGMI), and scatters what it received. A node record is GTF_HALO_NODE_BYTES: has_merged
 * as a 64-bit integer, merged_state[3], merged_cov[5], merged_prior (raw fp64 bits);
 * an activation is one byte. Offsets of node records must be multiples of 8. */
#define GTF_HALO_NODE_BYTES 80
typedef struct gtf_halo {
    const int32_t* node_idx;  /* [n_nodes] device: node of each record */
    const int64_t* node_off;  /* [n_nodes] device: byte offset of each record in the buffer */
    int32_t n_nodes;
    int32_t pad_;
    const int32_t* slot_idx;  /* [n_slots] device: slot of each activation byte */
    const int64_t* slot_off;  /* [n_slots] device: byte offset of each activation byte */
    int32_t n_slots;
    int32_t pad2_;
} gtf_halo;
/* gather the listed node states and activations into buf (device) */
int gtf_halo_pack(const gtf_nodes* n, const gtf_edges* e, const gtf_halo* h, void* buf, gtf_stream_t stream);
/* scatter buf (device) into the listed node states and activations */
int gtf_halo_unpack(gtf_nodes* n, gtf_edges* e, const gtf_halo* h, const void* buf, gtf_stream_t stream);

/* Tag propagation. radius: [N] node radius (attr 'zr'[1]); keep: [E] output mask of
 * kept inward neighbours per out-edge (u8, indexed by out-edge position);
 * processed: [N] u8 output; n_processed: device int32 output. With g->out_sched set the
 * prepare runs on its lane groups, so that schedule must list every node with an out-edge
 * (not a shard's restricted one: pass the graph without out_sched then). */
int gtf_tag_prepare(const gtf_graph* g, const double* radius, uint8_t* keep, uint8_t* processed,
                    int32_t* n_processed, gtf_stream_t stream);
/* one Jacobi sweep: tags_out[u] = max(tags_in[u], tags_in[kept neighbours]); *flips = the
 * number of changed tags (zeroed first). With g->out_sched (and out_lanes) the sweep runs
 * on the sender schedule's lane groups, otherwise one thread per node. */
int gtf_tag_sweep(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed,
                  const int64_t* tags_in, int64_t* tags_out, int32_t* flips, gtf_stream_t stream);
/* The whole tag-propagation stage in one call (tag_propagation.py:97-164: prepare, then
 * sweeps while flips / processed > flip_threshold -- the reference's 0.1 -- and fewer than
 * max_sweeps; the first sweep always runs). tags: device int64 [n_nodes], the initial tags
 * in, the final tags out; flips_out: host int32 [max_sweeps] (or NULL), the flip count of
 * every sweep; *sweeps_out: the number of sweeps. workspace: device, at least
 * gtf_tag_workspace_bytes(n_nodes, n_edges) bytes. The prepare launch builds a compact list
 * of every node's kept out-neighbours in the workspace, and the sweeps read those lists with
 * the tags carried as int32 while every tag fits (int64 from the first value that does not;
 * environment GTF_TAG_CSR=0: the keep-mask sweeps of gtf_tag_sweep). The sweeps go out in
 * batches of 4, 8, 16, ... 64 launches with the stop rule evaluated on the device; the host
 * waits once per batch, for a small report (the stop-rule words and the batch's flip totals)
 * the device writes into mapped page-locked memory the host polls (environment
 * GTF_TAG_POLL=0: a device-to-host copy and a stream synchronisation instead). */
size_t gtf_tag_workspace_bytes(int32_t n_nodes, int32_t n_edges);
int gtf_tag_propagate(const gtf_graph* g, const double* radius, int64_t* tags, double flip_threshold,
                      int32_t max_sweeps, int32_t* flips_out, int32_t* sweeps_out, void* workspace,
                      size_t workspace_bytes, gtf_stream_t stream);
/* One rank's sweep of tag propagation on an edge-sharded event (the sweep of
 * tag_propagation.py:137-164 over the rank's owned nodes [shard->node_lo, shard->node_hi)
 * of the replicated graph `g`). tags_in / tags_out: device int64 [n_nodes + nranks].
 * Writes the owned nodes' next tags, INT64_MIN for every other node, this rank's flip count
 * to tags_out[n_nodes + rank] and 0 to the other ranks' count words, so ONE all-reduce(MAX)
 * of the n_nodes + nranks words gives every rank the whole next tag array and every
 * rank's flip count (their sum is the sweep's flips). gtf_tag_prepare runs unsharded on
 * the replica (its n_processed is the whole event's). */
int gtf_tag_sweep_shard(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed,
                        const int64_t* tags_in, int64_t* tags_out, const gtf_shard* shard,
                        int32_t rank, int32_t nranks, gtf_stream_t stream);

/* ---- Native collectives for the sharded event (SURVEY §8b gtf_comm_init, §8e) ----------
 * RCCL over xGMI inside libgtf, one communicator per rank (one process per GPU; create it
 * with the rank's device current), every call stream-ordered on the caller's stream. RCCL is
 * loaded on first use (GTF_RCCL = its path, else an RCCL already loaded in the process, else
 * librccl.so.1). Rank 0 calls gtf_comm_unique_id and hands the GTF_COMM_ID_BYTES to the other
 * ranks (file, socket, MPI, ...); each rank then calls gtf_comm_init. Status -4: an RCCL
 * error (gtf_last_error names it). These replace the role of the reference's serial subgraph
 * loop (src/extrapolate/extrapolate_merged_states.py:406-451) for one event spread over the
 * GPUs of a node. */
#define GTF_COMM_ID_BYTES 128
typedef struct gtf_comm gtf_comm;
int gtf_comm_unique_id(void* id);
int gtf_comm_init(gtf_comm** comm, int32_t rank, int32_t nranks, const void* rccl_uid);
int gtf_comm_destroy(gtf_comm* comm);
int gtf_comm_rank(const gtf_comm* comm);
int gtf_comm_size(const gtf_comm* comm);
/* The per-pass halo exchange: gtf_halo_pack into send_buf, one all-to-all of the
 * per-destination segments (send_bytes[p] / recv_bytes[p]: host int64 [nranks], segments back
 * to back in rank order, a rank's own segment empty), gtf_halo_unpack from recv_buf. */
int gtf_halo_exchange(gtf_comm* comm, gtf_nodes* n, gtf_edges* e, const gtf_halo* send, const gtf_halo* recv,
                      void* send_buf, void* recv_buf, const int64_t* send_bytes, const int64_t* recv_bytes,
                      gtf_stream_t stream);
/* the all-to-all of gtf_halo_exchange alone (no pack / unpack), for a caller that runs it on
 * a stream of its own beside the pass's phase 1 (gtf_shard.phases) */
int gtf_halo_alltoall(gtf_comm* comm, const void* send_buf, void* recv_buf, const int64_t* send_bytes,
                      const int64_t* recv_bytes, gtf_stream_t stream);
/* in-place all-reduce(MAX) of int64 words (the sharded tag sweep's exchange) */
int gtf_allreduce_max_i64(gtf_comm* comm, int64_t* words, int64_t count, gtf_stream_t stream);
/* all-gather of one equal-size chunk per rank into gathered (nranks chunks, rank order):
 * gtf_shard_pack -> this -> gtf_shard_unpack completes every replica */
int gtf_allgather_bytes(gtf_comm* comm, const void* chunk, void* gathered, int64_t bytes, gtf_stream_t stream);
/* The whole tag-propagation stage on an edge-sharded event (tag_propagation.py:97-164): prepare
 * on the replica, per sweep gtf_tag_sweep_shard over the owned nodes + one all-reduce(MAX),
 * stop when flips / processed <= flip_threshold (one synchronisation per sweep). tags: device
 * int64 [n_nodes] in / out (every rank ends with the whole array). */
size_t gtf_tag_shard_workspace_bytes(int32_t n_nodes, int32_t n_edges, int32_t nranks);
int gtf_tag_propagate_shard(gtf_comm* comm, const gtf_graph* g, const gtf_shard* shard, const double* radius,
                            int64_t* tags, double flip_threshold, int32_t max_sweeps, int32_t* flips_out,
                            int32_t* sweeps_out, void* workspace, size_t workspace_bytes, gtf_stream_t stream);

/* ---- Distances between updated track states --------------------
 * calculate_distance_between_updated_states/calculate_distance_between_updated_track_states.py:
 * mahalanobis_distance (:27-104) over the pair loop of :134-195. For every node with an
 * updated_track_states dict (n->has_uts, :143) and more than one active in-edge (:139-140),
 * every pair i > j of its dict entries in dict order (:174-176): the [a, b] Mahalanobis term
 * plus the delta-tau term with the hard-coded sigma_z = 0.5 / sigma_r = 0.1, swapped where
 * |x| >= 600 (:62-74); <tau>, <theta>, delta theta (:89-99); and the truth flag (:190-193).
 * Coordinates: g->xyzr of the node and of each neighbour (:162-163, :182-183).
 * Pairs of node v are written at [pair_ptr[v] + t], t = i (i - 1) / 2 + j (the reference's
 * loop order). gtf_updated_state_pair_counts writes each node's pair count (0 or d(d-1)/2)
 * for the caller's exclusive scan into pair_ptr [N+1]; a node whose pair_ptr range has
 * another size is skipped with GTF_ERR_PAIR_COUNT. Uses g->sched when present. */
typedef struct gtf_pair_out {
    double* chi2;         /* [P] */
    double* avg_tau;      /* [P] or NULL */
    double* avg_theta;    /* [P] or NULL */
    double* delta_theta;  /* [P] or NULL */
    int8_t* truth;        /* [P] or NULL (needs node truth) */
    uint32_t* err;        /* device error word (GTF_ERR_PAIR_COUNT / _NEIGHBOUR_MISSING / _TOO_MANY_STATES) or NULL */
} gtf_pair_out;

int gtf_updated_state_pair_counts(const gtf_graph* g, const gtf_nodes* n, const gtf_states* uts, const gtf_edges* e,
                                  int64_t* counts, gtf_stream_t stream);
/* truth: [N] truth_particle per node (device), or NULL */
int gtf_updated_state_distances(const gtf_graph* g, const gtf_nodes* n, const gtf_states* uts, const gtf_edges* e,
                                const int64_t* truth, const int64_t* pair_ptr, const gtf_pair_out* out,
                                gtf_stream_t stream);

/* ---- Initial track-state estimates -----------------------------
 * helper.compute_track_state_estimates (helper.py:238-452): for every key of every
 * node's track_state_estimates dict (slots with tse->rank >= 0; the dict order is an
 * input, the reference's reversed(set(nx.all_neighbors)) order) writes tse->sv
 * (edge_state_vector), tse->cov (the aliased edge/joint covariance, :417-425),
 * tse->tau (joint_vector[2]) and tse->xyzr (neighbour coordinates), plus the optional
 * per-slot / per-node extras below. Needs g->sched (the slot-count node schedule).
 * The reference reads its set-ordered tau / del_tau / theta lists with dict positions
 * (:384, :419-431); that pairing is reproduced. */
typedef struct gtf_tse_extra {
    double* theta;        /* [S*3] theta, theta2, variance_theta, or NULL */
    double* var_ms;       /* [S]   var_ms_node, or NULL */
    double* xy_mean_var;  /* [N*2] xy_edge_gradient_mean_var, or NULL */
    double* zr_mean_var;  /* [N*2] zr_edge_gradient_mean_var, or NULL */
    double* angle;        /* [N]   angle_of_rotation, or NULL */
    double* translation;  /* [N*2] translation, or NULL */
} gtf_tse_extra;

int gtf_track_state_estimates(const gtf_graph* g, gtf_states* tse, const gtf_tse_extra* extra,
                              const gtf_params* p, gtf_stream_t stream);

/* ---- Track-candidate extraction ---------------------------
 * src/extract/extract_track_candidates.py main (:349-467) on the pass's output: CCA
 * over the activated edges of each subgraph (a subgraph with no deactivated edge stays
 * one candidate), then per candidate the fragment check, close-proximity merging (the
 * reference mutates the merged node's GNN_Measurement in place, :111-114: io->gnn is
 * updated the same way), the one-hit-per-layer check, rotate_track and the xy / rz
 * Kalman fits with their chi-square p-values; a candidate is extracted when both
 * p-values reach p_accept. Candidates are identified by their first node (min index). */
typedef struct gtf_extract_params {
    double p_accept;          /* -p */
    int32_t fragment;         /* -n minimum hits (>= 3) */
    int32_t pad_;
    double separation_3d;     /* -s (rotate_track) */
    double merge_distance;    /* -t (close-proximity merging) */
    double sigma0xy, sigma0rz, endcap_boundary;   /* -e -z -b */
} gtf_extract_params;

typedef struct gtf_extract_io {
    const double* xyzr;       /* [N*4] node attribute xyzr */
    const double* vivl;       /* [N*2] volume_id, in_volume_layer_id */
    const int32_t* sub_id;    /* [N]   subgraph of each node (nodes grouped by subgraph) */
    const int32_t* sub_ptr;   /* [n_sub+1] first node of each subgraph */
    int32_t n_sub;
    int32_t pad_;
    const int32_t* order_key; /* [N] member order inside a candidate (distinct values), or NULL = node order */
    double* gnn;              /* [N*4] GNN_Measurement x,y,z,r: merged nodes get the midpoint */
    int32_t* label;           /* [N] out: candidate id of each node */
    int8_t* status;           /* [N] out per candidate id: 0 fragment, 1 bad layers, 2 rejected, 3 extracted */
    double* pval_xy;          /* [N] out per candidate id (NaN when not fitted) */
    double* pval_zr;
    uint8_t* extracted;       /* [N] out per node */
    int32_t* n_candidates;    /* device scalar out */
} gtf_extract_io;

size_t gtf_extract_workspace_bytes(int32_t n_nodes, int32_t n_sub);
/* synchronises the stream once per connected-components round (a few rounds) */
int gtf_extract_candidates(const gtf_graph* g, const gtf_edges* e, const gtf_extract_io* io,
                           const gtf_extract_params* p, void* workspace, gtf_stream_t stream);

/* ---- Parabolic-model KL training data -------------------------
 * learn_KL_parabolic_model/src/generate_training_data: the per-edge parabolic
 * state of compute_track_state_estimates (utils.py:221-289; S = diag(16, 0.01,
 * 0.01), H rows [x^2, x, 1]) for every in-edge of a node, and the pairwise KL
 * distance KLDistance / calc_pairwise_distances (extract_metadata_trackml_parabolic_
 * model.py:15-25) of every pair i > j of a node with >= 2 in-edges (:61-62), with the
 * node's gradient variance (utils.py:240-254, :286) and the pair truth flag (:82-95).
 *
 * Pairs of node v are written at out->kl[pair_ptr[v] + t], t = i (i - 1) / 2 + j
 * (row-major lower triangle over the node's in-slots, slot order); pair_ptr[v + 1] -
 * pair_ptr[v] must be d (d - 1) / 2 for d = slot_ptr[v + 1] - slot_ptr[v] >= 2, else 0.
 * emp_var is the variance over in-neighbours, which is the reference's variance
 * over nx.all_neighbors when the edge set is symmetric (helper.py:512-518 adds both
 * directions). */
typedef struct gtf_kl_graph {
    int32_t n_nodes, n_slots;
    const int32_t* slot_ptr;  /* [N+1] in-edge CSR (every slot an edge) */
    const int32_t* slot_src;  /* [S] neighbour of each in-edge */
    const double* gnn;        /* [N*gnn_stride] GNN_Measurement x, y(, z, r) */
    const int64_t* truth;     /* [N] truth_particle, or NULL */
    const int64_t* pair_ptr;  /* [N+1] */
    const int32_t* list[4];   /* nodes to process by in-degree bucket, any order within a bucket:
                                 d in [1, 2], [3, 4] (one thread each), [5, 8] (8-lane groups) and d > 8
                                 (one 64-lane wavefront each); d = 1 nodes yield states and
                                 gradient moments but no pairs */
    int32_t count[4];
    /* ordered layout (v3; gtf.parabolic.ParabolicKL(ordered=True)): when every list[i] is
     * NULL, bucket i is the node range [first[i], first[i] + count[i]), and bucket 0 holds
     * n_d1 one-edge nodes, then its two-edge nodes, with consecutive slots from slot0 (in
     * node order) and one pair each from pair0: the kernel then reaches bucket 0's slots,
     * neighbours and pairs by arithmetic, and every bucket's nodes without a list load. */
    int32_t first[4];
    int32_t n_d1;
    int32_t gnn_stride;       /* doubles per gnn row: 0 or 4 (x, y, z, r), or 2 (a compact x, y copy:
                                 the kernel reads only x and y, so half the gathered bytes) */
    int64_t slot0;
    int64_t pair0;
    /* tiled layout (gtf.parabolic.ParabolicKL(tile=T)): the nodes azimuth-sorted per event and
     * cut into tiles of <= 256 one- / two-edge (bucket-0) nodes and the nodes between them, bucket
     * 0 first inside a tile (one-edge, then two-edge nodes, consecutive slots and one pair each).
     * One 256-thread block per tile record of 12 int32: (first node, bucket-0 count n0, its
     * one-edge count, the in-tile three-edge count n3, the in-tile four-edge count n4, 0, bucket
     * 0's first slot, its first pair low / high 32 bits, window [lo, hi) of at most 1024
     * consecutive nodes holding the tile's neighbours, 0); the n3 three-edge and then n4
     * four-edge nodes follow the tile's bucket-0 nodes (slots and pairs consecutive) and run in
     * the tile's block, one thread per node, so n0 + n3 + n4 <= 256 (the block skips nodes past
     * 256 without an error; gtf.parabolic.ParabolicKL._block_table refuses such tiles). n3 and
     * n4 must be 0 when list[1] is given (bucket 1 then runs by list). The block loads its
     * sender lists and the window's x, y and truth ids in one round and reads the neighbours from
     * LDS. Buckets 1..3 come from list[1..3] / count[1..3] (count[0] and list[0] are ignored). The
     * library clamps each window to its LDS size but does not check the records' node, slot and
     * pair ranges against the arrays (they live in device memory): build them with
     * gtf.parabolic.ParabolicKL(tile=T), or keep every range inside n_nodes / n_slots. */
    const int32_t* blk;       /* [12 * n_blk] or NULL */
    int32_t n_blk;
    /* ordered layout, degree runs (round 4): deg_runs = 1 when buckets 1 and 2 hold their nodes
     * sorted by in-degree, n_deg[k] nodes of in-degree 3 + k (k = 0..5) one run after another
     * (sum n_deg[0..1] = count[1], sum n_deg[2..5] = count[2]), with consecutive slots and pairs
     * after bucket 0's: the kernel then finds their slots and pairs by arithmetic as well (one
     * dependent round of loads fewer). 0: slot_ptr / pair_ptr are read per node. */
    int32_t deg_runs;
    int32_t n_deg[6];
    int32_t pad_deg_;
} gtf_kl_graph;

enum { GTF_F64 = 0, GTF_F32 = 1 };

typedef struct gtf_kl_out {
    void* kl;          /* [P] double (GTF_F64) or float (GTF_F32) */
    int8_t* truth;     /* [P] or NULL (needs graph truth) */
    double* emp_var;   /* [N] or NULL; np.var of the gradients, written for the listed nodes */
    double* emp_mean;  /* [N] or NULL; np.mean of the gradients (xy_edge_gradient_mean_var[0]) */
    double* sv;        /* [S*3] edge_state_vector or NULL */
    double* cov;       /* [S*9] edge_covariance (row-major) or NULL */
    uint32_t* err;     /* device error word (GTF_ERR_SINGULAR_H) or NULL */
} gtf_kl_out;

/* dtype: GTF_F64 computes states and distances in fp64 (the reference's precision);
 * GTF_F32 rotates/translates in fp64 and forms states and distances in fp32 (the
 * config-5 tolerance sweep). sv/cov outputs are fp64 in both modes. */
int gtf_parabolic_kl(const gtf_kl_graph* g, int32_t dtype, const gtf_kl_out* out, gtf_stream_t stream);

/* ---- event conversion: CSV rows -> packed CSR in the reference's orders -------------
 * Replaces helper.construct_graph + nx.DiGraph + the weakly-connected-component
 * subgraph copies of event_conversion.py:63-84 (helper.py:465-521) and the key order of
 * helper.compute_track_state_estimates' dicts (helper.py:277, 350-351). Host function
 * (no device work): the packed graph then goes to the GPU, where
 * gtf_track_state_estimates and gtf_node_ops compute the states, priors, mixture
 * weights and degrees. Orders are CPython 3.10 set orders, reproduced exactly. */
typedef struct gtf_event_csr {
    int64_t n_nodes;          /* in: nodes kept by the volume window, CSV order */
    int64_t n_rows;           /* in: edges.csv rows */
    const int64_t* node_id;   /* in: [n_nodes] node_idx, unique, in [0, 2^61 - 1) */
    const int64_t* row_a;     /* in: [n_rows] second column (node1): add_edge(a, b) first */
    const int64_t* row_b;     /* in: [n_rows] first column (node2) */
    int32_t* order;           /* out: [n_nodes] CSV index of packed node i */
    int32_t* sub_id;          /* out: [n_nodes] subgraph (weakly connected component) */
    int32_t* slot_ptr;        /* out: [n_nodes + 1] */
    int32_t* slot_src;        /* out: [2 * n_rows] packed sender per slot (ascending per receiver) */
    int32_t* tse_rank;        /* out: [2 * n_rows] track_state_estimates dict position */
    int32_t* out_ptr;         /* out: [n_nodes + 1] */
    int32_t* out_slot;        /* out: [2 * n_rows] successor order */
    int64_t n_edges;          /* out: directed edges (= slots) */
    int32_t n_subgraphs;      /* out */
    int32_t pad_;
} gtf_event_csr;

int gtf_build_event_csr(gtf_event_csr* ev);

/* The same build on the GPU (SURVEY §8f #2 "graph build on device"; gtf_build_dev.hip):
 * every pointer of `ev` a DEVICE array of the sizes above, the outputs equal to
 * gtf_build_event_csr's bit for bit (radix sorts for the id lookup and networkx's
 * successor insertion order, hook + pointer jumping for the weakly connected components,
 * CPython 3.10 set tables in the workspace for the set orders). Synchronises `stream`
 * (n_edges / n_subgraphs are returned in `ev`). Replaces helper.construct_graph
 * (helper.py:465-521) and event_conversion.py:63-84 like the host builder. */
size_t gtf_build_event_device_workspace_bytes(int64_t n_nodes, int64_t n_rows);
int gtf_build_event_csr_device(gtf_event_csr* ev, void* workspace, size_t workspace_bytes, gtf_stream_t stream);

/* Member order of every extraction candidate as the reference builds it: CCA over the
 * active edges of each subgraph (extract_track_candidates.py:332-346) -- networkx
 * weakly connected components, each copied as subGraph.subgraph(component) (set order
 * when the component is under half the subgraph) -- or the whole subgraph when none of
 * its edges is inactive. order_key[v] = v's position in its candidate: the order
 * rotate_track's stable r-sort and the efficiency's particle vote break ties in.
 * Host arrays of the packed graph; sub_id grouped (pack order). */
typedef struct gtf_candidate_graph {
    int32_t n_nodes, n_slots, n_edges, pad_;
    const int32_t* slot_ptr;
    const int32_t* slot_src;
    const uint8_t* is_edge;
    const uint8_t* act;
    const int32_t* out_ptr;
    const int32_t* out_slot;
    const int32_t* sub_id;
    const int64_t* node_id;
} gtf_candidate_graph;

int gtf_candidate_order(const gtf_candidate_graph* cg, int32_t* order_key);

/* Device memory for a host without a framework allocator (csrc/gtf_mem.hip): the drop-in
 * stage CLIs (extrapolate_merged_states.py:521-572, clustering.py:380-415,
 * remove_state_metadata.py:11-57 -- one process per stage and iteration) allocate and
 * copy through the HIP runtime libgtf is linked against instead of loading a framework
 * (gtf/devmem.py). Copies are stream-ordered; gtf_memcpy_dtoh synchronises the stream.
 * gtf_malloc(…, 0) returns a valid 256-byte allocation (never a null pointer). */
int gtf_device_init(int32_t device);
int gtf_malloc(void** ptr, size_t bytes);
int gtf_free(void* ptr);
int gtf_memcpy_htod(void* dst, const void* src, size_t bytes, gtf_stream_t stream);
int gtf_memcpy_dtoh(void* dst, const void* src, size_t bytes, gtf_stream_t stream);
int gtf_memcpy_dtod(void* dst, const void* src, size_t bytes, gtf_stream_t stream);
int gtf_memset(void* dst, int32_t value, size_t bytes, gtf_stream_t stream);
int gtf_stream_synchronize(gtf_stream_t stream);

const char* gtf_last_error(void);
const char* gtf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GTF_H */
