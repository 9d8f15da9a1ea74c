// gtf_comm.hip -- the sharded pass's collectives inside libgtf (SURVEY §8b gtf_comm_init, §8e):
// RCCL over xGMI, one communicator per rank (one process per GPU), every call stream-ordered
// on the caller's HIP stream. A native or torch-free host drives the edge-sharded event with
// these alone: the per-pass halo exchange (pack -> one all-to-all of per-destination
// segments -> unpack), the all-gather of owned states before read-back, and the sharded tag
// propagation's all-reduce(MAX) per sweep.
//
// RCCL is loaded on first use (dlopen), not linked: the library is ~0.5 GB of device code
// whose load would sit in every drop-in CLI's start-up, and a process that already holds
// PyTorch's RCCL can point GTF_RCCL at that copy so one RCCL serves both. The reference has
// no counterpart (its scaling is the serial subgraph loop of
// src/extrapolate/extrapolate_merged_states.py:406-451); this replaces that loop's role for
// one event spread over the GPUs of a node.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    const char* (*error_string)(ncclResult_t);
    ncclResult_t (*group_start)();
    ncclResult_t (*group_end)();
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
};

Rccl g_rccl;

int fail(const char* what) {
    gtf::set_error(what);
    return -1;
}

int nccl_fail(const char* what, ncclResult_t r) {
    char m[256];
    snprintf(m, sizeof(m), "%s: %s", what, g_rccl.error_string ? g_rccl.error_string(r) : "RCCL error");
    gtf::set_error(m);
    return -4;
}

template <typename F>
bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(g_rccl.h, name));
    return f != nullptr;
}

// GTF_RCCL (a path) first, then an RCCL already loaded in the process, then the ROCm one
int load_rccl() {
    if (g_rccl.h) return 0;
    const char* env = getenv("GTF_RCCL");
    void* h = nullptr;
    if (env && *env) h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return fail("gtf_comm: cannot load RCCL (librccl.so.1; set GTF_RCCL to its path)");
    g_rccl.h = h;
    bool ok = sym(g_rccl.get_unique_id, "ncclGetUniqueId") && sym(g_rccl.comm_init_rank, "ncclCommInitRank") &&
              sym(g_rccl.comm_destroy, "ncclCommDestroy") && sym(g_rccl.error_string, "ncclGetErrorString") &&
              sym(g_rccl.group_start, "ncclGroupStart") && sym(g_rccl.group_end, "ncclGroupEnd") &&
              sym(g_rccl.send, "ncclSend") && sym(g_rccl.recv, "ncclRecv") &&
              sym(g_rccl.all_reduce, "ncclAllReduce") && sym(g_rccl.all_gather, "ncclAllGather");
    if (!ok) {
        g_rccl.h = nullptr;
        return fail("gtf_comm: RCCL lacks a symbol");
    }
    return 0;
}

}  // namespace

struct gtf_comm {
    ncclComm_t c;
    int32_t rank, nranks;
};

extern "C" {

int gtf_comm_unique_id(void* id) {
    if (!id) return fail("gtf_comm_unique_id: null id");
    if (int rc = load_rccl()) return rc;
    ncclUniqueId u;
    const ncclResult_t r = g_rccl.get_unique_id(&u);
    if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
    memcpy(id, &u, sizeof(u));
    return 0;
}

int gtf_comm_init(gtf_comm** comm, int32_t rank, int32_t nranks, const void* rccl_uid) {
    if (!comm || !rccl_uid || nranks < 1 || rank < 0 || rank >= nranks)
        return fail("gtf_comm_init: bad arguments");
    *comm = nullptr;
    if (int rc = load_rccl()) return rc;
    ncclUniqueId u;
    memcpy(&u, rccl_uid, sizeof(u));
    ncclComm_t c = nullptr;
    const ncclResult_t r = g_rccl.comm_init_rank(&c, nranks, u, rank);   // on the current HIP device
    if (r != ncclSuccess) return nccl_fail("ncclCommInitRank", r);
    *comm = new gtf_comm{c, rank, nranks};
    return 0;
}

int gtf_comm_destroy(gtf_comm* comm) {
    if (!comm) return 0;
    const ncclResult_t r = g_rccl.comm_destroy(comm->c);
    delete comm;
    return r == ncclSuccess ? 0 : nccl_fail("ncclCommDestroy", r);
}

int gtf_comm_rank(const gtf_comm* comm) { return comm ? comm->rank : -1; }
int gtf_comm_size(const gtf_comm* comm) { return comm ? comm->nranks : -1; }

// the all-to-all of the halo segments: per-destination segments back to back, in rank
// order, on both sides (grouped ncclSend / ncclRecv on `stream`)
int gtf_halo_alltoall(gtf_comm* comm, const void* send_buf, void* recv_buf, const int64_t* send_bytes,
                      const int64_t* recv_bytes, gtf_stream_t stream) {
    if (!comm || !send_bytes || !recv_bytes) return fail("gtf_halo_alltoall: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    int64_t so = 0, ro = 0;
    ncclResult_t r = g_rccl.group_start();
    for (int p = 0; p < comm->nranks && r == ncclSuccess; p++) {
        if (p != comm->rank && send_bytes[p] > 0)
            r = g_rccl.send((const char*)send_buf + so, (size_t)send_bytes[p], ncclUint8, p, comm->c, st);
        if (r == ncclSuccess && p != comm->rank && recv_bytes[p] > 0)
            r = g_rccl.recv((char*)recv_buf + ro, (size_t)recv_bytes[p], ncclUint8, p, comm->c, st);
        so += send_bytes[p];
        ro += recv_bytes[p];
    }
    const ncclResult_t r2 = g_rccl.group_end();
    if (r != ncclSuccess) return nccl_fail("gtf_halo_alltoall send/recv", r);
    if (r2 != ncclSuccess) return nccl_fail("gtf_halo_alltoall group", r2);
    return 0;
}

int gtf_halo_exchange(gtf_comm* comm, gtf_nodes* n, gtf_edges* e, const gtf_halo* send, const gtf_halo* recv,
                      void* send_buf, void* recv_buf, const int64_t* send_bytes, const int64_t* recv_bytes,
                      gtf_stream_t stream) {
    if (!comm || !send_bytes || !recv_bytes) return fail("gtf_halo_exchange: bad arguments");
    if (int rc = gtf_halo_pack(n, e, send, send_buf, stream)) return rc;
    if (int rc = gtf_halo_alltoall(comm, send_buf, recv_buf, send_bytes, recv_bytes, stream)) return rc;
    return gtf_halo_unpack(n, e, recv, recv_buf, stream);
}

int gtf_allreduce_max_i64(gtf_comm* comm, int64_t* words, int64_t count, gtf_stream_t stream) {
    if (!comm || count < 0 || (count > 0 && !words)) return fail("gtf_allreduce_max_i64: bad arguments");
    if (count == 0) return 0;
    const ncclResult_t r =
        g_rccl.all_reduce(words, words, (size_t)count, ncclInt64, ncclMax, comm->c, (hipStream_t)stream);
    return r == ncclSuccess ? 0 : nccl_fail("ncclAllReduce", r);
}

int gtf_allgather_bytes(gtf_comm* comm, const void* chunk, void* gathered, int64_t bytes, gtf_stream_t stream) {
    if (!comm || bytes < 0 || (bytes > 0 && (!chunk || !gathered))) return fail("gtf_allgather_bytes: bad arguments");
    if (bytes == 0) return 0;
    const ncclResult_t r = g_rccl.all_gather(chunk, gathered, (size_t)bytes, ncclUint8, comm->c, (hipStream_t)stream);
    return r == ncclSuccess ? 0 : nccl_fail("ncclAllGather", r);
}

// The sharded tag-propagation stage (tag_propagation.py:97-164 over an edge-sharded event):
// gtf_tag_prepare on the replica, then per sweep gtf_tag_sweep_shard over the owned nodes and
// one all-reduce(MAX) of the n_nodes + nranks words (next tags + every rank's flip count);
// the stop rule reads the summed count (one synchronisation per sweep).
size_t gtf_tag_shard_workspace_bytes(int32_t n_nodes, int32_t n_edges, int32_t nranks) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t n = n_nodes > 0 ? (size_t)n_nodes : 1, e = n_edges > 0 ? (size_t)n_edges : 1;
    const size_t w = (size_t)(n_nodes > 0 ? n_nodes : 0) + (size_t)(nranks > 0 ? nranks : 1);
    return al(2 * sizeof(int32_t)) + al(e) + al(n) + 2 * al(sizeof(int64_t) * w);
}

int gtf_tag_propagate_shard(gtf_comm* comm, const gtf_graph* g, const gtf_shard* shard, const double* radius,
                            int64_t* tags, double flip_threshold, int32_t max_sweeps, int32_t* flips_out,
                            int32_t* sweeps_out, void* workspace, size_t workspace_bytes, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_propagate_shard")) return rc;
    if (!comm || !shard || !sweeps_out || max_sweeps < 0 || (g->n_nodes > 0 && (!tags || !radius)))
        return fail("gtf_tag_propagate_shard: bad arguments");
    const int32_t N = g->n_nodes, R = comm->nranks;
    if (!workspace || workspace_bytes < gtf_tag_shard_workspace_bytes(N, g->n_edges, R))
        return fail("gtf_tag_propagate_shard: workspace smaller than gtf_tag_shard_workspace_bytes()");
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    hipStream_t st = (hipStream_t)stream;
    const size_t n = N > 0 ? (size_t)N : 1, e = g->n_edges > 0 ? (size_t)g->n_edges : 1, w = (size_t)N + R;
    char* p = static_cast<char*>(workspace);
    int32_t* cnt = reinterpret_cast<int32_t*>(p);
    p += al(2 * sizeof(int32_t));
    uint8_t* keep = reinterpret_cast<uint8_t*>(p);
    p += al(e);
    uint8_t* proc = reinterpret_cast<uint8_t*>(p);
    p += al(n);
    int64_t* buf[2] = {reinterpret_cast<int64_t*>(p), reinterpret_cast<int64_t*>(p + al(sizeof(int64_t) * w))};
    *sweeps_out = 0;
    // prepare covers the whole replica: a rank's graph view carries only its own senders'
    // schedule, so the thread-per-node form (no out_sched) runs here
    gtf_graph whole = *g;
    whole.out_sched = nullptr;
    whole.out_lanes = nullptr;
    if (int rc = gtf_tag_prepare(&whole, radius, keep, proc, cnt, stream)) return rc;
    int32_t total = 0;
    if (N > 0 && hipMemcpyAsync(buf[0], tags, sizeof(int64_t) * (size_t)N, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail("gtf_tag_propagate_shard: copying the tags");
    if (hipMemcpyAsync(&total, cnt, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail("gtf_tag_propagate_shard: reading the processed count");
    std::vector<int64_t> words((size_t)R);
    double frac = 1.0;
    int32_t s = 0, cur = 0;
    while (frac > flip_threshold && s < max_sweeps) {
        if (int rc = gtf_tag_sweep_shard(g, keep, proc, buf[cur], buf[cur ^ 1], shard, comm->rank, R, stream)) return rc;
        if (int rc = gtf_allreduce_max_i64(comm, buf[cur ^ 1], (int64_t)w, stream)) return rc;
        if (hipMemcpyAsync(words.data(), buf[cur ^ 1] + N, sizeof(int64_t) * (size_t)R, hipMemcpyDeviceToHost, st) !=
                hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail("gtf_tag_propagate_shard: reading the flip counts");
        int64_t f = 0;
        for (int64_t x : words) f += x;
        if (flips_out) flips_out[s] = (int32_t)f;
        s++;
        frac = total ? (double)f / (double)total : 0.0;
        cur ^= 1;
    }
    *sweeps_out = s;
    if (N > 0 && hipMemcpyAsync(tags, buf[cur], sizeof(int64_t) * (size_t)N, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail("gtf_tag_propagate_shard: copying the tags back");
    return 0;
}

}  // extern "C"
