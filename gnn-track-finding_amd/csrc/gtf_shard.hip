// gtf_shard.hip -- the per-pass exchange of one event sharded across GPUs.
//
// Rank r owns receivers [node_lo, node_hi) and their slots [slot_lo, slot_hi). After a
// pass, the only data another rank's next pass reads is (a) the owned senders' merged
// state (has_merged, state, covariance incl. the cumulative var_ms write-back, prior)
// and (b) the owned slots' activation, which other ranks' sender scans read for the
// out-edges of their halo senders. Each rank packs (a) and (b) into one chunk of a
// fixed layout; an all-gather of equal-size chunks over RCCL puts every chunk on every
// GPU; one unpack launch scatters the other ranks' chunks into the replicated arrays.
// Values travel as bytes, so the replicas are bit-identical to the owner's arrays.
// The halo exchange (gtf_halo_pack / gtf_halo_unpack) moves only the records another
// rank's next pass reads, through per-destination segments of one all-to-all.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

constexpr int BLOCK = 256;

inline __host__ __device__ size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct ChunkLayout {
    size_t hm, ms, mc, mp, act, bytes;
};

__host__ __device__ inline ChunkLayout layout(int cap_n, int cap_s) {
    ChunkLayout L;
    size_t o = 0;
    L.hm = o;  o += al256((size_t)cap_n);
    L.ms = o;  o += al256(sizeof(double) * 3 * (size_t)cap_n);
    L.mc = o;  o += al256(sizeof(double) * 5 * (size_t)cap_n);
    L.mp = o;  o += al256(sizeof(double) * (size_t)cap_n);
    L.act = o; o += al256((size_t)cap_s);
    L.bytes = o;
    return L;
}

// one thread per node field element / slot of the owned ranges
__global__ void __launch_bounds__(BLOCK) k_pack(gtf_nodes n, gtf_edges e, int node_lo, int nn, int slot_lo, int ns,
                                                char* chunk, ChunkLayout L) {
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < nn) {
        const int64_t v = node_lo + t;
        chunk[L.hm + t] = (char)n.has_merged[v];
        double* ms = (double*)(chunk + L.ms);
        double* mc = (double*)(chunk + L.mc);
        double* mp = (double*)(chunk + L.mp);
        for (int i = 0; i < 3; i++) ms[3 * (int64_t)t + i] = n.merged_state[3 * v + i];
        for (int i = 0; i < 5; i++) mc[5 * (int64_t)t + i] = n.merged_cov[5 * v + i];
        mp[t] = n.merged_prior[v];
    }
    if (t < ns) chunk[L.act + t] = (char)e.act[slot_lo + t];
}

// blockIdx.y = source rank; threads over max(cap_nodes, cap_slots)
__global__ void __launch_bounds__(BLOCK) k_unpack(gtf_nodes n, gtf_edges e, const char* gathered, int self,
                                                  const int32_t* ranges, ChunkLayout L) {
    const int r = blockIdx.y;
    if (r == self) return;
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    const int node_lo = ranges[4 * r], node_hi = ranges[4 * r + 1];
    const int slot_lo = ranges[4 * r + 2], slot_hi = ranges[4 * r + 3];
    const char* chunk = gathered + (size_t)r * L.bytes;
    if (t < node_hi - node_lo) {
        const int64_t v = node_lo + t;
        n.has_merged[v] = (uint8_t)chunk[L.hm + t];
        const double* ms = (const double*)(chunk + L.ms);
        const double* mc = (const double*)(chunk + L.mc);
        const double* mp = (const double*)(chunk + L.mp);
        for (int i = 0; i < 3; i++) n.merged_state[3 * v + i] = ms[3 * (int64_t)t + i];
        for (int i = 0; i < 5; i++) n.merged_cov[5 * v + i] = mc[5 * (int64_t)t + i];
        n.merged_prior[v] = mp[t];
    }
    if (t < slot_hi - slot_lo) e.act[slot_lo + t] = (uint8_t)chunk[L.act + t];
}

// halo records: thread t < n_nodes packs / unpacks node record t, the others activation
// bytes (one launch covers both lists)
__global__ void __launch_bounds__(BLOCK) k_halo_pack(gtf_nodes n, gtf_edges e, gtf_halo h, char* buf) {
    const int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t < h.n_nodes) {
        const int64_t v = h.node_idx[t];
        uint64_t* rec = (uint64_t*)(buf + h.node_off[t]);
        rec[0] = n.has_merged[v];
        const uint64_t* ms = (const uint64_t*)(n.merged_state + 3 * v);
        const uint64_t* mc = (const uint64_t*)(n.merged_cov + 5 * v);
        for (int i = 0; i < 3; i++) rec[1 + i] = ms[i];
        for (int i = 0; i < 5; i++) rec[4 + i] = mc[i];
        rec[9] = *(const uint64_t*)(n.merged_prior + v);
    } else if (t < (int64_t)h.n_nodes + h.n_slots) {
        const int64_t j = t - h.n_nodes;
        buf[h.slot_off[j]] = (char)e.act[h.slot_idx[j]];
    }
}

__global__ void __launch_bounds__(BLOCK) k_halo_unpack(gtf_nodes n, gtf_edges e, gtf_halo h, const char* buf) {
    const int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t < h.n_nodes) {
        const int64_t v = h.node_idx[t];
        const uint64_t* rec = (const uint64_t*)(buf + h.node_off[t]);
        n.has_merged[v] = (uint8_t)rec[0];
        uint64_t* ms = (uint64_t*)(n.merged_state + 3 * v);
        uint64_t* mc = (uint64_t*)(n.merged_cov + 5 * v);
        for (int i = 0; i < 3; i++) ms[i] = rec[1 + i];
        for (int i = 0; i < 5; i++) mc[i] = rec[4 + i];
        *(uint64_t*)(n.merged_prior + v) = rec[9];
    } else if (t < (int64_t)h.n_nodes + h.n_slots) {
        const int64_t j = t - h.n_nodes;
        e.act[h.slot_idx[j]] = (uint8_t)buf[h.slot_off[j]];
    }
}

bool halo_ok(const gtf_halo* h) {
    return h && h->n_nodes >= 0 && h->n_slots >= 0 && (h->n_nodes == 0 || (h->node_idx && h->node_off)) &&
           (h->n_slots == 0 || (h->slot_idx && h->slot_off));
}

}  // namespace

extern "C" {

int gtf_halo_pack(const gtf_nodes* n, const gtf_edges* e, const gtf_halo* h, void* buf, gtf_stream_t stream) {
    if (!n || !e || !halo_ok(h) || (!buf && h->n_nodes + h->n_slots > 0)) {
        gtf::set_error("gtf_halo_pack: bad arguments");
        return -2;
    }
    const int64_t m = (int64_t)h->n_nodes + h->n_slots;
    if (m > 0)
        hipLaunchKernelGGL(k_halo_pack, dim3((unsigned)((m + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, (hipStream_t)stream,
                           *n, *e, *h, (char*)buf);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { gtf::set_error(hipGetErrorString(err)); return -1; }
    return 0;
}

int gtf_halo_unpack(gtf_nodes* n, gtf_edges* e, const gtf_halo* h, const void* buf, gtf_stream_t stream) {
    if (!n || !e || !halo_ok(h) || (!buf && h->n_nodes + h->n_slots > 0)) {
        gtf::set_error("gtf_halo_unpack: bad arguments");
        return -2;
    }
    const int64_t m = (int64_t)h->n_nodes + h->n_slots;
    if (m > 0)
        hipLaunchKernelGGL(k_halo_unpack, dim3((unsigned)((m + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                           (hipStream_t)stream, *n, *e, *h, (const char*)buf);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { gtf::set_error(hipGetErrorString(err)); return -1; }
    return 0;
}


size_t gtf_shard_chunk_bytes(int32_t cap_nodes, int32_t cap_slots) {
    return layout(cap_nodes > 0 ? cap_nodes : 0, cap_slots > 0 ? cap_slots : 0).bytes;
}

int gtf_shard_pack(const gtf_nodes* n, const gtf_edges* e, const gtf_shard* sh, int32_t cap_nodes,
                   int32_t cap_slots, void* chunk, gtf_stream_t stream) {
    if (!n || !e || !sh || !chunk) { gtf::set_error("gtf_shard_pack: null argument"); return -2; }
    const int nn = sh->node_hi - sh->node_lo, ns = sh->slot_hi - sh->slot_lo;
    if (nn < 0 || ns < 0 || nn > cap_nodes || ns > cap_slots) {
        gtf::set_error("gtf_shard_pack: owned range exceeds the chunk capacity");
        return -2;
    }
    const int m = nn > ns ? nn : ns;
    if (m > 0)
        hipLaunchKernelGGL(k_pack, dim3((m + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, (hipStream_t)stream, *n, *e,
                           sh->node_lo, nn, sh->slot_lo, ns, (char*)chunk, layout(cap_nodes, cap_slots));
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { gtf::set_error(hipGetErrorString(err)); return -1; }
    return 0;
}

int gtf_shard_unpack(gtf_nodes* n, gtf_edges* e, const void* gathered, int32_t nranks, int32_t self,
                     const int32_t* ranges, int32_t cap_nodes, int32_t cap_slots, gtf_stream_t stream) {
    if (!n || !e || !gathered || !ranges || nranks < 1 || self < 0 || self >= nranks) {
        gtf::set_error("gtf_shard_unpack: bad arguments");
        return -2;
    }
    const int m = cap_nodes > cap_slots ? cap_nodes : cap_slots;
    if (m > 0 && nranks > 1)
        hipLaunchKernelGGL(k_unpack, dim3((m + BLOCK - 1) / BLOCK, nranks), dim3(BLOCK), 0, (hipStream_t)stream, *n,
                           *e, (const char*)gathered, self, ranges, layout(cap_nodes, cap_slots));
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { gtf::set_error(hipGetErrorString(err)); return -1; }
    return 0;
}

}  // extern "C"
