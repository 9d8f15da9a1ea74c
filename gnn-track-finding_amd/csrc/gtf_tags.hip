// gtf_tags.hip -- tag propagation ("custom CCA") as CSR kernels for gfx950.
// Reference: tag_propagation/tag_propagation.py:97-164. The reference walks a
// dict-of-dicts adjacency and deep-copies the whole graph every sweep; here one
// sweep is one launch over the out-CSR, reading the previous tag array and
// writing the next (Jacobi). Counts never go through one hot word: a device-scope atomic
// on one address saturates near 88 per microsecond on MI355X (MI355X_MICROARCH.md,
// dequeue), so a wave-per-atomic count over the ~20k waves of a C4 launch costs ~200 us.
// The processed count is a separate reduction of the processed bytes (a few dozen block
// atomics), and a sweep's flips are summed per block in LDS and added to one of
// TAG_SHARDS counter words, each on its own 128-byte line (block % TAG_SHARDS).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace {
constexpr int BLOCK = 256;
constexpr int TAG_SHARDS = 32;    // counter words of one sweep's flip count
constexpr int TAG_STRIDE = 32;    // int32 words between two shards (one 128-byte line each)

// the block's count of `mine` lanes added to ctr: one atomic per block, to shard
// blockIdx % nsh (nsh = 1: ctr is a single word). Every thread of the block calls it.
template <typename T>
__device__ __forceinline__ void block_count_add(int mine, T* ctr, int nsh) {
    __shared__ int s_cnt[BLOCK / 64];
    const unsigned long long b = __ballot(mine);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = (int)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) t += s_cnt[w];
        if (t) atomicAdd(ctr + (nsh > 1 ? (int)(blockIdx.x % nsh) * TAG_STRIDE : 0), (T)t);
    }
}

// two counts of one block in one reduction: `a` lanes added to ctr_a (shard blockIdx % nsh_a)
// and, when ctr_b is not NULL (block-uniform), `b` lanes to ctr_b (shard blockIdx % TAG_SHARDS)
__device__ __forceinline__ void block_count_add2(int a, int32_t* ctr_a, int nsh_a, int b, int32_t* ctr_b) {
    __shared__ int s_cnt2[2][BLOCK / 64];
    const unsigned long long ba = __ballot(a), bb = __ballot(b);
    if ((threadIdx.x & 63) == 0) {
        s_cnt2[0][threadIdx.x >> 6] = (int)__popcll(ba);
        s_cnt2[1][threadIdx.x >> 6] = (int)__popcll(bb);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int ta = 0, tb = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) { ta += s_cnt2[0][w]; tb += s_cnt2[1][w]; }
        if (ta) atomicAdd(ctr_a + (nsh_a > 1 ? (int)(blockIdx.x % nsh_a) * TAG_STRIDE : 0), ta);
        if (ctr_b && tb) atomicAdd(ctr_b + (int)(blockIdx.x % TAG_SHARDS) * TAG_STRIDE, tb);
    }
}

// the total of a sharded counter (wave-uniform: every lane gets it)
__device__ __forceinline__ int32_t shard_total(const int32_t* ctr, int nsh) {
    const int lane = threadIdx.x & 63;
    int v = lane < nsh ? ctr[lane * TAG_STRIDE] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// n_processed = the number of nonzero (= 1) bytes of processed[0, n): 16 bytes per thread
// per step over the 16-byte aligned body (block 0 also takes the head and tail bytes), a
// block sum, one atomic per block (a few dozen blocks)
__global__ void __launch_bounds__(BLOCK) k_count_flags(const uint8_t* f, int n, int32_t* out) {
    const int head0 = (int)((16 - ((uintptr_t)f & 15)) & 15);
    const int head = head0 < n ? head0 : n;
    const int nv = (n - head) / 16;
    const int tail = head + 16 * nv;
    int cnt = 0;
    const uint4* v = reinterpret_cast<const uint4*>(f + head);
    for (int i = blockIdx.x * BLOCK + threadIdx.x; i < nv; i += gridDim.x * BLOCK) {
        const uint4 x = v[i];   // bytes are 0 or 1: one bit each
        cnt += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
    }
    if (blockIdx.x == 0) {
        const int t = (int)threadIdx.x;
        if (t < head) cnt += f[t] != 0;
        if (t < n - tail) cnt += f[tail + t] != 0;
    }
    __shared__ int s_cnt[BLOCK / 64];
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < BLOCK / 64; w++) t += s_cnt[w];
        if (t) atomicAdd(out, t);
    }
}

// keep[e] = neighbour radius <= node radius (:99-110); processed[u] = any kept (:109-110)
// zero (may be NULL): nzero int32 words zeroed by block 0 (the stop-rule words the count
// kernel and the sweeps that follow add to)
__device__ __forceinline__ void zero_words(int32_t* zero, int nzero) {
    if (zero && blockIdx.x == 0)
        for (int i = (int)threadIdx.x; i < nzero; i += BLOCK) zero[i] = 0;
}

// the kept inward neighbours as a compact list per node (gtf_tag_propagate's sweeps): kcnt[u]
// of them, their node indices at kidx[out_ptr[u] ...] (the front of u's own out-edge range).
// With `kword` (graphs of < 2^23 edges) the node's list is one 4-byte word, out_ptr[u] << 9 |
// min(count, 511), and kcnt[u] is written only where the count saturates: the sweep reads one
// word per node instead of the count and the offset.
constexpr uint32_t KW_BITS = 9, KW_SAT = (1u << KW_BITS) - 1u;
struct TagCsr {
    int32_t* kcnt;    // [N] or NULL: no lists
    int32_t* kidx;    // [E]
    uint32_t* kword;  // [N] or NULL: kcnt for every node
};
__device__ __forceinline__ void csr_node(const TagCsr& csr, int u, int base, int nk) {
    if (csr.kword) {
        csr.kword[u] = ((uint32_t)base << KW_BITS) | (nk < (int)KW_SAT ? (uint32_t)nk : KW_SAT);
        if (nk >= (int)KW_SAT) csr.kcnt[u] = nk;
    } else {
        csr.kcnt[u] = nk;
    }
}

__global__ void __launch_bounds__(BLOCK) k_tag_prepare(gtf_graph g, const double* radius, uint8_t* keep,
                                                       uint8_t* processed, int32_t* zero, int nzero, TagCsr csr) {
    zero_words(zero, nzero);
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    if (u < g.n_nodes) {
        const double ru = radius[u];
        int any = 0, nk = 0;
        const int o0 = g.out_ptr[u];
        for (int i = o0; i < g.out_ptr[u + 1]; i++) {
            const int w = g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]];
            const uint8_t k = !(radius[w] > ru);
            if (keep) keep[i] = k;
            any |= k;
            if (k && csr.kcnt) csr.kidx[o0 + nk++] = w;
        }
        if (processed) processed[u] = (uint8_t)any;
        if (csr.kcnt) csr_node(csr, u, o0, nk);
    }
}

// The same on the sender schedule's lane groups (gtf_graph.out_sched + out_lanes): every lane
// reads its out-edge's neighbour radius in one round beside the node's own, a group ballot
// gives processed[u]; nodes without an out-edge are not processed (the launch's last blocks)
template <int G>
__device__ __forceinline__ unsigned long long group_bits(bool pred) {   // this lane's G-lane group's ballot
    const unsigned long long m = __ballot(pred);
    if constexpr (G == 64) return m;
    else return (m >> ((int)threadIdx.x & 63 & ~(G - 1))) & ((1ull << G) - 1ull);
}

template <int G>
__device__ __forceinline__ void prep_group(const gtf_graph& g, const double* radius, uint8_t* keep, uint8_t* processed,
                                          const int4* list, const int2* lanes, int count, int b, const TagCsr& csr) {
    const int t = b * BLOCK + (int)threadIdx.x;
    const int gi = t / G, gl = t & (G - 1);
    if (gi >= count) return;   // group-uniform
    const int4 en = list[gi];
    const int u = en.x;
    const double ru = radius[u];
    int nk = 0;   // kept out-edges (group-uniform)
    if (lanes) {   // one out-edge per lane (<= G of them)
        const int2 kv = lanes[t];
        const bool edge = kv.x >= 0;
        const double rw = radius[edge ? kv.y : u];
        const bool k = edge && !(rw > ru);
        if (edge && keep) keep[en.y + gl] = (uint8_t)k;
        const unsigned long long km = group_bits<G>(k);
        if (csr.kcnt && k) csr.kidx[en.y + __popcll(km & ((1ull << gl) - 1ull))] = kv.y;   // (in out-list order)
        nk = __popcll(km);
    } else {       // chunks of G out-edges (a group-uniform trip count: the ballots see every lane)
        for (int c0 = en.y; c0 < en.z; c0 += G) {
            const int i = c0 + gl;
            const bool in = i < en.z;
            const int w = in ? (g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]) : u;
            const bool k = in && !(radius[w] > ru);
            if (in && keep) keep[i] = (uint8_t)k;
            const unsigned long long km = group_bits<G>(k);
            if (csr.kcnt && k) csr.kidx[en.y + nk + __popcll(km & ((1ull << gl) - 1ull))] = w;
            nk += __popcll(km);
        }
    }
    if (gl == 0) {
        if (processed) processed[u] = (uint8_t)(nk > 0);
        if (csr.kcnt) csr_node(csr, u, en.y, nk);
    }
}

// exclusive prefix of v over the block's threads in thread order (every thread of the block calls it)
__device__ __forceinline__ int block_excl_scan(int v) {
    __shared__ int s_tot[BLOCK / 64];
    const int lane = (int)threadIdx.x & 63, wid = (int)threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tot[wid] = x;
    __syncthreads();
    int add = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; w++) add += w < wid ? s_tot[w] : 0;
    __syncthreads();   // (s_tot is reused by the next call)
    return add + x - v;
}

// gtf_tag_propagate's prepare in the compact-list form (no keep mask, no processed flags: its
// sweeps read neither), NPT nodes per thread BLOCK apart with their loads interleaved as in
// sweep_csr_nodes: the out-list bounds and own radius of each, its first four out-neighbours,
// their radii (longer lists in steps of four); the kept ones in out-list order. Where they go:
// - pack = 0: the front of the node's own out-range (kidx[out_ptr[u] ...]);
// - pack = 1 (packed words only: the word carries the offset): back to back in node order from
//   the start of the out-range of the node's run of BLOCK nodes (a block scan of the counts; a
//   run's kept lists never outgrow its out-edges), so the lists a sweep wave reads are dense --
//   half the kidx lines of the out-range fronts on C3, where about half the out-edges are kept.
template <int NPT>
__global__ void __launch_bounds__(BLOCK) k_tag_prepare_csr(gtf_graph g, const double* radius, TagCsr csr,
                                                           int32_t* zero, int nzero, int pack) {
    zero_words(zero, nzero);
    const int blk = gtf::xcd_local(blockIdx.x, gridDim.x);
    const int u0 = blk * BLOCK * NPT + (int)threadIdx.x;
    int o0[NPT], o1[NPT];
    double ru[NPT];
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        const int u = u0 + j * BLOCK;
        o0[j] = o1[j] = 0;
        ru[j] = 0.0;
        if (u < g.n_nodes) {
            o0[j] = g.out_ptr[u];
            o1[j] = g.out_ptr[u + 1];
            ru[j] = radius[u];
        }
    }
    constexpr int R = 4;   // out-neighbours per node in the second round (then chunks of R)
    auto dst = [&](int i) { return g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]; };
    int w[NPT][R];
#pragma unroll
    for (int j = 0; j < NPT; j++)
#pragma unroll
        for (int r = 0; r < R; r++) w[j][r] = o0[j] + r < o1[j] ? dst(o0[j] + r) : 0;
    double rw[NPT][R];
#pragma unroll
    for (int j = 0; j < NPT; j++)
#pragma unroll
        for (int r = 0; r < R; r++) rw[j][r] = o0[j] + r < o1[j] ? radius[w[j][r]] : 0.0;
    // the kept out-neighbours past the first R of node j: counted, or (write) stored from kidx[at]
    auto rest = [&](int j, bool write, int at) {
        int nk = 0;
        for (int i = o0[j] + R; i < o1[j]; i += R) {   // longer lists: R independent loads per step
            int x[R];
            double rx[R];
#pragma unroll
            for (int r = 0; r < R; r++) x[r] = i + r < o1[j] ? dst(i + r) : 0;
#pragma unroll
            for (int r = 0; r < R; r++) rx[r] = i + r < o1[j] ? radius[x[r]] : 0.0;
#pragma unroll
            for (int r = 0; r < R; r++)
                if (i + r < o1[j] && !(rx[r] > ru[j])) {
                    if (write) csr.kidx[at + nk] = x[r];
                    nk++;
                }
        }
        return nk;
    };
#ifndef GTF_TAG_PACK_MASK
#define GTF_TAG_PACK_MASK 1   // 1: the count pass keeps the kept bits of out-edges R .. R + 31, so the write pass
                              // reloads only their neighbour indices (no second radius gather)
#endif
    // (pack) the count pass of the out-edges past the first R: the kept bits of the next 32
    auto rest_count = [&](int j, uint32_t& km) {
        int nk = 0;
        km = 0u;
        for (int i = o0[j] + R; i < o1[j]; i += R) {
            int x[R];
            double rx[R];
#pragma unroll
            for (int r = 0; r < R; r++) x[r] = i + r < o1[j] ? dst(i + r) : 0;
#pragma unroll
            for (int r = 0; r < R; r++) rx[r] = i + r < o1[j] ? radius[x[r]] : 0.0;
#pragma unroll
            for (int r = 0; r < R; r++)
                if (i + r < o1[j] && !(rx[r] > ru[j])) {
                    const int off = i + r - o0[j] - R;
                    if (off < 32) km |= 1u << off;
                    nk++;
                }
        }
        return nk;
    };
    // ... and its write pass: the bits' neighbours reloaded, anything past them recomputed
    auto rest_write = [&](int j, uint32_t km, int at) {
        int nk = 0;
        while (km) {
            const int off = __builtin_ctz(km);
            km &= km - 1u;
            csr.kidx[at + nk++] = dst(o0[j] + R + off);
        }
        for (int i = o0[j] + R + 32; i < o1[j]; i++) {
            const int x = dst(i);
            if (!(radius[x] > ru[j])) csr.kidx[at + nk++] = x;
        }
        return nk;
    };
    int base[NPT];
    uint32_t kmask[NPT];
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        base[j] = o0[j];
        kmask[j] = 0u;
    }
    if (pack) {   // (uniform) the counts first, then every node's place in its run
        int nk[NPT];
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            nk[j] = 0;
#pragma unroll
            for (int r = 0; r < R; r++) nk[j] += o0[j] + r < o1[j] && !(rw[j][r] > ru[j]);
            if (o1[j] - o0[j] > R) nk[j] += GTF_TAG_PACK_MASK ? rest_count(j, kmask[j]) : rest(j, false, 0);
        }
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            const int first = blk * BLOCK * NPT + j * BLOCK;   // the run's first node
            const int run0 = first < g.n_nodes ? g.out_ptr[first] : 0;
            base[j] = run0 + block_excl_scan(nk[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        const int u = u0 + j * BLOCK;
        if (u >= g.n_nodes) continue;
        int nk = 0;
#pragma unroll
        for (int r = 0; r < R; r++)
            if (o0[j] + r < o1[j] && !(rw[j][r] > ru[j])) csr.kidx[base[j] + nk++] = w[j][r];
        if (o1[j] - o0[j] > R)
            nk += pack && GTF_TAG_PACK_MASK ? rest_write(j, kmask[j], base[j] + nk) : rest(j, true, base[j] + nk);
        csr_node(csr, u, base[j], nk);
    }
}

struct PrepBuckets {
    const int4* list[3];
    const int2* lanes[2];
    int32_t count[3];
    int32_t blocks[3];
};

__global__ void __launch_bounds__(BLOCK) k_tag_prepare_sched(gtf_graph g, const double* radius, uint8_t* keep,
                                                             uint8_t* processed, PrepBuckets pb, int32_t* zero,
                                                             int nzero, TagCsr csr) {
    zero_words(zero, nzero);
    // (XCD-contiguous block ranges: a run of one bucket's senders -- neighbours of each other --
    // shares one XCD's L2 for the radius gathers)
    int b = gtf::xcd_local(blockIdx.x, gridDim.x);
    if (b < pb.blocks[0]) {
        prep_group<4>(g, radius, keep, processed, pb.list[0], pb.lanes[0], pb.count[0], b, csr);
    } else if ((b -= pb.blocks[0]) < pb.blocks[1]) {
        prep_group<8>(g, radius, keep, processed, pb.list[1], pb.lanes[1], pb.count[1], b, csr);
    } else if ((b -= pb.blocks[1]) < pb.blocks[2]) {
        prep_group<16>(g, radius, keep, processed, pb.list[2], nullptr, pb.count[2], b, csr);
    } else {
        const int u = (b - pb.blocks[2]) * BLOCK + (int)threadIdx.x;
        if (u < g.n_nodes && g.out_ptr[u + 1] == g.out_ptr[u]) {
            if (processed) processed[u] = 0;
            if (csr.kcnt) csr_node(csr, u, g.out_ptr[u], 0);
        }
    }
}

// The stop rule of the sweep loop on the device (tag_propagation.py:130-164): sweep s runs
// only while the previous sweep flipped more than flip_threshold of the processed nodes
// (frac = 0 when none are processed, where the reference divides by zero), so a batch of
// sweeps is enqueued without a host read between them and the sweeps past the stop return
// at once. Every block takes the same decision from the finished previous sweep's count.
struct TagCtl {
    const int32_t* total;   // processed count, TAG_SHARDS shards (counted by the first sweep)
    const int32_t* prev;    // flips of the previous sweep (TAG_SHARDS shards), NULL for the first
    int32_t* stop;          // set once the rule stops the loop
    int32_t* nexec;         // sweeps executed
    double thr;
    int32_t* next;          // the next sweep's counter shards, zeroed by block 0 (NULL: the caller zeroes)
    int32_t* count_processed;   // (the first sweep) where its blocks add the processed nodes, else NULL
};

__device__ __forceinline__ bool tag_skip(const TagCtl& c) {
    if (!c.stop) return false;
    if (*c.stop) return true;
    if (c.prev) {
        const int32_t tot = shard_total(c.total, TAG_SHARDS), f = shard_total(c.prev, TAG_SHARDS);
        const double frac = tot ? (double)f / (double)tot : 0.0;
        if (!(frac > c.thr)) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(c.stop, 1);
            return true;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(c.nexec, 1);
    if (c.next && blockIdx.x == 0 && threadIdx.x < TAG_SHARDS) c.next[threadIdx.x * TAG_STRIDE] = 0;
    return false;
}

// the batch's stop-rule words and per-sweep flip totals into the caller's page-locked report
// (mapped, coherent): rep[1..3] = processed, stop, executed; rep[4 + i] = flips of sweep s + i;
// rep[0] = seq last, after a system-scope fence, so the host that sees seq sees the rest
__global__ void __launch_bounds__(64) k_tag_report(const int32_t* hdr, const int32_t* pshards, const int32_t* ring,
                                                   int s, int nb, int ring_n, int32_t* rep, int32_t seq) {
    const int t = (int)threadIdx.x;
    const int32_t processed = shard_total(pshards, TAG_SHARDS);
    if (t < nb) {
        const int32_t* c = ring + (size_t)((s + t) % ring_n) * TAG_SHARDS * TAG_STRIDE;
        int f = 0;
        for (int k = 0; k < TAG_SHARDS; k++) f += c[k * TAG_STRIDE];
        rep[4 + t] = f;
    }
    if (t == 0) rep[1] = processed;
    if (t == 1 || t == 2) rep[1 + t] = hdr[t];
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(rep, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the final tags into the caller's array: after an odd number of executed sweeps they sit
// in the workspace copy (sweep s reads buffer s % 2 and writes the other)
__global__ void __launch_bounds__(BLOCK) k_tag_final(int64_t* tags, const int64_t* other, const int32_t* nexec, int n) {
    const int u = blockIdx.x * BLOCK + threadIdx.x;
    if (u < n && (*nexec & 1)) tags[u] = other[u];
}

// tags_out[u] = max(tags_in[u], tags_in[kept successors]) (:141-150 -- max, not min)
__global__ void __launch_bounds__(BLOCK) k_tag_sweep(gtf_graph g, const uint8_t* keep, const uint8_t* processed,
                                                     const int64_t* tin, int64_t* tout, int32_t* flips, int nsh,
                                                     TagCtl ctl) {
    if (tag_skip(ctl)) return;
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    int flipped = 0, pr = 0;
    if (u < g.n_nodes) {
        const int64_t t0 = tin[u];
        int64_t t = t0;
        pr = processed[u] != 0;
        if (pr) {
            for (int i = g.out_ptr[u]; i < g.out_ptr[u + 1]; i++)
                if (keep[i]) {
                    const int64_t tw = tin[g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]];
                    t = tw > t ? tw : t;
                }
            flipped = (t != t0);
        }
        tout[u] = t;
    }
    block_count_add2(flipped, flips, nsh, pr, ctl.count_processed);
}
// With the sender schedule (gtf_graph.out_sched + out_lanes): G lanes per node over its
// out-edges, every lane's loads in one round (its keep flag, its neighbour's tag, the
// node's own tag) and a group max, instead of a thread walking the out-list one dependent
// gather at a time. Nodes without an out-edge keep their tag (one thread per node in the
// launch's last blocks copies it).
template <int G>
__device__ __forceinline__ int tag_group_lanes(const gtf_graph& g, const uint8_t* keep, const uint8_t* processed,
                                               const int64_t* tin, int64_t* tout, const int4* list, const int2* lanes,
                                               int count, int b) {
    const int t = b * BLOCK + (int)threadIdx.x;
    const int gi = t / G, gl = t & (G - 1);
    if (gi >= count) return 0;   // group-uniform
    const int4 en = list[gi];
    const int2 kv = lanes[t];
    const int u = en.x, i = en.y + gl;
    const bool edge = kv.x >= 0;
    const uint8_t kp = edge ? keep[i] : 0;
    const int64_t tw = tin[edge ? kv.y : u];
    const int64_t t0 = tin[u];
    const uint8_t pr = processed[u];
    int64_t m = (edge && kp) ? (tw > t0 ? tw : t0) : t0;
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(m, o, G);
        m = x > m ? x : m;
    }
    if (!pr) m = t0;
    if (gl == 0) tout[u] = m;
    return (gl == 0 && m != t0) | ((gl == 0 && pr) ? 2 : 0);   // bit 0 flipped, bit 1 processed
}

template <int G>
__device__ __forceinline__ int tag_group(const gtf_graph& g, const uint8_t* keep, const uint8_t* processed,
                                         const int64_t* tin, int64_t* tout, const int4* list, int count, int b) {
    const int gi = (b * BLOCK + (int)threadIdx.x) / G, gl = threadIdx.x & (G - 1);
    if (gi >= count) return 0;
    const int4 en = list[gi];
    const int u = en.x;
    const int64_t t0 = tin[u];
    int64_t m = t0;
    for (int i = en.y + gl; i < en.z; i += G)
        if (keep[i]) {
            const int64_t tw = tin[g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]];
            m = tw > m ? tw : m;
        }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(m, o, G);
        m = x > m ? x : m;
    }
    const bool pr = processed[u] != 0;
    if (!pr) m = t0;
    if (gl == 0) tout[u] = m;
    return (gl == 0 && m != t0) | ((gl == 0 && pr) ? 2 : 0);   // bit 0 flipped, bit 1 processed
}

struct TagBuckets {
    const int4* list[3];
    const int2* lanes[2];
    int32_t count[3];
    int32_t blocks[3];
    int32_t copy_blocks;   // one thread per node: out-degree 0 -> tag kept
};

__global__ void __launch_bounds__(BLOCK) k_tag_sweep_sched(gtf_graph g, const uint8_t* keep, const uint8_t* processed,
                                                           const int64_t* tin, int64_t* tout, int32_t* flips,
                                                           int nsh, TagBuckets tb, TagCtl ctl) {
    if (tag_skip(ctl)) return;
    int b = gtf::xcd_local(blockIdx.x, gridDim.x), flipped = 0;   // (bit 0 flipped, bit 1 processed: tag_group*)
    if (b < tb.blocks[0]) {
        flipped = tb.lanes[0] ? tag_group_lanes<4>(g, keep, processed, tin, tout, tb.list[0], tb.lanes[0], tb.count[0], b)
                              : tag_group<4>(g, keep, processed, tin, tout, tb.list[0], tb.count[0], b);
    } else if ((b -= tb.blocks[0]) < tb.blocks[1]) {
        flipped = tb.lanes[1] ? tag_group_lanes<8>(g, keep, processed, tin, tout, tb.list[1], tb.lanes[1], tb.count[1], b)
                              : tag_group<8>(g, keep, processed, tin, tout, tb.list[1], tb.count[1], b);
    } else if ((b -= tb.blocks[1]) < tb.blocks[2]) {
        flipped = tag_group<16>(g, keep, processed, tin, tout, tb.list[2], tb.count[2], b);
    } else {
        const int u = (b - tb.blocks[2]) * BLOCK + (int)threadIdx.x;
        if (u < g.n_nodes && g.out_ptr[u + 1] == g.out_ptr[u]) tout[u] = tin[u];
        return;   // (block-uniform: these blocks count no flips)
    }
    block_count_add2(flipped & 1, flips, nsh, (flipped >> 1) & 1, ctl.count_processed);
}

// gtf_tag_propagate's sweep over the compact kept lists (TagCsr), one thread per node: the
// node's count and list offset and its own tag in one round, its kept neighbours' indices in
// the next, their tags in the third -- instead of the sender schedule's 16-byte entry plus an
// 8-byte lane record per out-edge (24+ bytes per sender on C3's small out-degrees) and the keep
// mask. The tags travel as int32 when every value fits: the first sweep reads the caller's
// int64 tags, writes its output in both widths and raises `ovf` if any output does not fit;
// the later sweeps run on the int32 pair unless `ovf` is set (then on the int64 pair, as the
// scheduled sweep does). The maximum of values that fit fits, so one check suffices.
// NPT nodes per thread (BLOCK apart, so every round of loads stays coalesced), their loads
// interleaved: the words and own tags of all of them, then the first four kept indices of each,
// then those neighbours' tags -- three dependent rounds for NPT nodes instead of for one.
// Longer lists finish in steps of four independent loads.
// `t32` (the first sweep only): the int32 copy of the output, with `ovf` raised where a value
// does not fit.
template <int NPT, int R, typename T>
__device__ __forceinline__ void sweep_csr_nodes(const gtf_graph& g, const TagCsr& csr, const T* tin, T* tout,
                                                int32_t* t32, int32_t* ovf, int u0, int& nflip, int& nproc) {
    int c[NPT], b[NPT];
    T t[NPT];
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        const int u = u0 + j * BLOCK;
        c[j] = 0;
        b[j] = 0;
        t[j] = 0;
        if (u < g.n_nodes) {
            if (csr.kword) {   // (uniform)
                const uint32_t w = csr.kword[u];
                b[j] = (int)(w >> KW_BITS);
                c[j] = (int)(w & KW_SAT);
            } else {
                c[j] = csr.kcnt[u];
                b[j] = g.out_ptr[u];
            }
            t[j] = tin[u];
        }
    }
    int a[NPT][R];   // R kept indices per node in the second round (then chunks of R)
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        if (csr.kword && c[j] == (int)KW_SAT) c[j] = csr.kcnt[u0 + j * BLOCK];   // (a saturated count)
#pragma unroll
        for (int r = 0; r < R; r++) a[j][r] = c[j] > r ? csr.kidx[b[j] + r] : 0;
    }
    T m[NPT];
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        m[j] = t[j];
#pragma unroll
        for (int r = 0; r < R; r++)
            if (c[j] > r) {
                const T v = tin[a[j][r]];
                m[j] = v > m[j] ? v : m[j];
            }
    }
#pragma unroll
    for (int j = 0; j < NPT; j++)
        for (int k = R; k < c[j]; k += R) {   // longer lists: R independent loads per step
            int x[R];
#pragma unroll
            for (int r = 0; r < R; r++) x[r] = k + r < c[j] ? csr.kidx[b[j] + k + r] : -1;
#pragma unroll
            for (int r = 0; r < R; r++)
                if (x[r] >= 0) {
                    const T v = tin[x[r]];
                    m[j] = v > m[j] ? v : m[j];
                }
        }
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        const int u = u0 + j * BLOCK;
        const bool in = u < g.n_nodes;
        if (in) {
            tout[u] = m[j];
            if (t32) {
                t32[u] = (int32_t)m[j];
                if ((int64_t)m[j] != (int64_t)(int32_t)m[j]) atomicOr(ovf, 1);   // (only where a value does not fit)
            }
        }
        // wave-level counts by ballot (every lane of the wave holds them): a cross-lane sum would
        // add a dependent chain of LDS permutes to the end of every wave, exposed on a launch of
        // one round of waves like C4's
        nflip += (int)__popcll(__ballot(in && m[j] != t[j]));
        nproc += (int)__popcll(__ballot(in && c[j] > 0));
    }
}

// the block's totals of two wave-level counts into sharded counters (block_count_add2 with counts)
__device__ __forceinline__ void block_sum_add2(int a, int32_t* ctr_a, int nsh_a, int b, int32_t* ctr_b) {
    __shared__ int s_sum2[2][BLOCK / 64];
    if ((threadIdx.x & 63) == 0) {
        s_sum2[0][threadIdx.x >> 6] = a;
        s_sum2[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int ta = 0, tb = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) { ta += s_sum2[0][w]; tb += s_sum2[1][w]; }
        if (ta) atomicAdd(ctr_a + (nsh_a > 1 ? (int)(blockIdx.x % nsh_a) * TAG_STRIDE : 0), ta);
        if (ctr_b && tb) atomicAdd(ctr_b + (int)(blockIdx.x % TAG_SHARDS) * TAG_STRIDE, tb);
    }
}

// one node per thread (the launches of under ~262 k nodes, C4's): the count and offset, then the
// list in steps of four independent loads -- measured 6.2 against 9.4 us per C4 sweep for
// sweep_csr_nodes<1, 4> (round 6)
template <typename T>
__device__ __forceinline__ T tag_max_csr(const T* tin, const int32_t* kidx, int base, int c, T t) {
    int j = 0;
    for (; j + 4 <= c; j += 4) {   // four gathers in flight
        const int a0 = kidx[base + j], a1 = kidx[base + j + 1], a2 = kidx[base + j + 2], a3 = kidx[base + j + 3];
        const T v0 = tin[a0], v1 = tin[a1], v2 = tin[a2], v3 = tin[a3];
        t = v0 > t ? v0 : t;
        t = v1 > t ? v1 : t;
        t = v2 > t ? v2 : t;
        t = v3 > t ? v3 : t;
    }
    for (; j < c; j++) {
        const T v = tin[kidx[base + j]];
        t = v > t ? v : t;
    }
    return t;
}

__global__ void __launch_bounds__(BLOCK) k_tag_sweep_csr1(gtf_graph g, TagCsr csr, const int64_t* tin64, int64_t* tout64,
                                                          const int32_t* tin32, int32_t* tout32, int first,
                                                          int32_t* ovf, int32_t* flips, int nsh, TagCtl ctl) {
    if (tag_skip(ctl)) return;
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    int flipped = 0, pr = 0;
    if (u < g.n_nodes) {
        int c, base;
        if (csr.kword) {   // (uniform)
            const uint32_t w = csr.kword[u];
            base = (int)(w >> KW_BITS);
            c = (int)(w & KW_SAT);
            if (c == (int)KW_SAT) c = csr.kcnt[u];
        } else {
            c = csr.kcnt[u];
            base = g.out_ptr[u];
        }
        pr = c > 0;
        if (first || *ovf) {   // (uniform)
            const int64_t t0 = tin64[u];
            const int64_t t = c > 0 ? tag_max_csr<int64_t>(tin64, csr.kidx, base, c, t0) : t0;
            tout64[u] = t;
            if (first) {
                tout32[u] = (int32_t)t;
                if (t != (int64_t)(int32_t)t) atomicOr(ovf, 1);   // (only where a value does not fit)
            }
            flipped = t != t0;
        } else {
            const int32_t t0 = tin32[u];
            const int32_t t = c > 0 ? tag_max_csr<int32_t>(tin32, csr.kidx, base, c, t0) : t0;
            tout32[u] = t;
            flipped = t != t0;
        }
    }
    block_count_add2(flipped, flips, nsh, pr, ctl.count_processed);
}

template <int NPT, int R>
__global__ void __launch_bounds__(BLOCK) k_tag_sweep_csr(gtf_graph g, TagCsr csr, const int64_t* tin64, int64_t* tout64,
                                                         const int32_t* tin32, int32_t* tout32, int first,
                                                         int32_t* ovf, int32_t* flips, int nsh, TagCtl ctl) {
    if (tag_skip(ctl)) return;
    const int u0 = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK * NPT + (int)threadIdx.x;
    int nflip = 0, nproc = 0;
    if (first || *ovf)   // (uniform)
        sweep_csr_nodes<NPT, R, int64_t>(g, csr, tin64, tout64, first ? tout32 : nullptr, ovf, u0, nflip, nproc);
    else
        sweep_csr_nodes<NPT, R, int32_t>(g, csr, tin32, tout32, nullptr, nullptr, u0, nflip, nproc);
    block_sum_add2(nflip, flips, nsh, nproc, ctl.count_processed);
}

// The wave-cooperative sweep over block-packed lists (k_tag_prepare_csr with pack: a 64-node
// group's kept lists are back to back, from its first node's offset on). A wave takes NG groups
// of 64 consecutive nodes: the packed words and own tags (one node per lane), then the group's
// whole list range in coalesced loads (lane l: entries l, l + 64, ...), each entry's neighbour tag
// gathered by the lane that loaded it and staged in LDS, and every lane's maximum over its own
// entries from there. Against sweep_csr_nodes (each lane loading its own node's entries, R at a
// time, predicated on its count), the index loads are whole-wave and dense and every gather lane
// is a kept edge: about half the vector memory instructions per node. A group whose lists hold
// more than COOP_CAP entries takes the per-lane loop (wave-uniform).
constexpr int COOP_CAP = 256;
template <int NG, typename T>
__device__ __forceinline__ void sweep_coop_nodes(const gtf_graph& g, const TagCsr& csr, const T* tin, T* tout,
                                                 int32_t* t32, int32_t* ovf, int n0, T* buf, int& nflip, int& nproc) {
    const int lane = (int)threadIdx.x & 63;
    int c[NG], b[NG];
    T t[NG];
#pragma unroll
    for (int j = 0; j < NG; j++) {
        const int u = n0 + j * 64 + lane;
        c[j] = 0;
        b[j] = 0;
        t[j] = 0;
        if (u < g.n_nodes) {
            const uint32_t w = csr.kword[u];
            b[j] = (int)(w >> KW_BITS);
            c[j] = (int)(w & KW_SAT);
            t[j] = tin[u];
        }
    }
    int w0[NG], tot[NG];
    bool fits = true;
#pragma unroll
    for (int j = 0; j < NG; j++) {
        const int g0 = n0 + j * 64;   // (wave-uniform)
        if (c[j] == (int)KW_SAT) c[j] = csr.kcnt[g0 + lane];   // (a saturated count)
        const int last = g.n_nodes - 1 - g0 < 63 ? g.n_nodes - 1 - g0 : 63;   // the group's last node's lane
        w0[j] = __builtin_amdgcn_readfirstlane(b[j]);
        tot[j] = last >= 0 ? __shfl(b[j] + c[j], last) - w0[j] : 0;
        fits = fits && tot[j] <= COOP_CAP;
    }
    T m[NG];
    if (fits) {   // (uniform)
        constexpr int NI = COOP_CAP / 64;
        int x[NG][NI];
#pragma unroll
        for (int j = 0; j < NG; j++)
#pragma unroll
            for (int i = 0; i < NI; i++)
                x[j][i] = i * 64 < tot[j] && i * 64 + lane < tot[j] ? csr.kidx[w0[j] + i * 64 + lane] : -1;
        T v[NG][NI];
#pragma unroll
        for (int j = 0; j < NG; j++)
#pragma unroll
            for (int i = 0; i < NI; i++) v[j][i] = x[j][i] >= 0 ? tin[x[j][i]] : (T)0;
#pragma unroll
        for (int j = 0; j < NG; j++)
#pragma unroll
            for (int i = 0; i < NI; i++)
                if (i * 64 < tot[j]) buf[j * COOP_CAP + i * 64 + lane] = v[j][i];
        gtf::wave_lds_sync();
#pragma unroll
        for (int j = 0; j < NG; j++) {
            m[j] = t[j];
            const T* s = buf + j * COOP_CAP + (b[j] - w0[j]);
            for (int k = 0; k < c[j]; k++) {
                const T y = s[k];
                m[j] = y > m[j] ? y : m[j];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NG; j++) m[j] = c[j] > 0 ? tag_max_csr<T>(tin, csr.kidx, b[j], c[j], t[j]) : t[j];
    }
#pragma unroll
    for (int j = 0; j < NG; j++) {
        const int u = n0 + j * 64 + lane;
        const bool in = u < g.n_nodes;
        if (in) {
            tout[u] = m[j];
            if (t32) {
                t32[u] = (int32_t)m[j];
                if ((int64_t)m[j] != (int64_t)(int32_t)m[j]) atomicOr(ovf, 1);   // (only where a value does not fit)
            }
        }
        nflip += (int)__popcll(__ballot(in && m[j] != t[j]));
        nproc += (int)__popcll(__ballot(in && c[j] > 0));
    }
}

template <int NG>
__global__ void __launch_bounds__(BLOCK) k_tag_sweep_coop(gtf_graph g, TagCsr csr, const int64_t* tin64, int64_t* tout64,
                                                          const int32_t* tin32, int32_t* tout32, int first,
                                                          int32_t* ovf, int32_t* flips, int nsh, TagCtl ctl) {
    if (tag_skip(ctl)) return;
    __shared__ int64_t s_buf[BLOCK / 64][NG * COOP_CAP];   // (the int32 sweeps use half of it)
    const int wv = (int)threadIdx.x >> 6;
    const int n0 = (gtf::xcd_local(blockIdx.x, gridDim.x) * (BLOCK / 64) + wv) * 64 * NG;
    int nflip = 0, nproc = 0;
    if (first || *ovf)   // (uniform)
        sweep_coop_nodes<NG, int64_t>(g, csr, tin64, tout64, first ? tout32 : nullptr, ovf, n0, s_buf[wv], nflip,
                                      nproc);
    else
        sweep_coop_nodes<NG, int32_t>(g, csr, tin32, tout32, nullptr, nullptr, n0,
                                      reinterpret_cast<int32_t*>(s_buf[wv]), nflip, nproc);
    block_sum_add2(nflip, flips, nsh, nproc, ctl.count_processed);
}

// the final tags into the caller's int64 array after a run of CSR sweeps: from the int32 pair
// (sweep q wrote buffer (q + 1) % 2, so nexec sweeps end in buffer nexec % 2), or -- when a
// value did not fit -- from the int64 pair as k_tag_final does
__global__ void __launch_bounds__(BLOCK) k_tag_final_csr(int64_t* tags, const int64_t* other, const int32_t* t32,
                                                         const int32_t* nexec, const int32_t* ovf, int n) {
    const int u = blockIdx.x * BLOCK + threadIdx.x;
    const int ne = *nexec;
    if (u >= n || ne == 0) return;
    if (*ovf) {
        if (ne & 1) tags[u] = other[u];
    } else {
        tags[u] = (int64_t)t32[(size_t)(ne & 1) * (size_t)n + u];
    }
}

// One rank's sweep of the sharded tag propagation: the owned nodes
// [lo, hi) as k_tag_sweep computes them; every other node's word is INT64_MIN and this
// rank's flip count goes to word n_nodes + rank (the other ranks' words stay 0), so an
// all-reduce(MAX) of the n_nodes + nranks words is the whole next tag array on every rank
// plus every rank's flip count: one collective per sweep, bit-exact (integer max).
__global__ void __launch_bounds__(BLOCK) k_tag_sweep_owned(gtf_graph g, const uint8_t* keep, const uint8_t* processed,
                                                           const int64_t* tin, int64_t* tout, int lo, int hi,
                                                           unsigned long long* flips) {
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    int flipped = 0;
    if (u < g.n_nodes) {
        int64_t t = INT64_MIN;
        if (u >= lo && u < hi) {
            const int64_t t0 = tin[u];
            t = t0;
            if (processed[u]) {
                for (int i = g.out_ptr[u]; i < g.out_ptr[u + 1]; i++)
                    if (keep[i]) {
                        const int64_t tw = tin[g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]];
                        t = tw > t ? tw : t;
                    }
                flipped = (t != t0);
            }
        }
        tout[u] = t;
    }
    block_count_add(flipped, flips, 1);
}
}  // namespace

extern "C" {

static int hip_fail(const char* what) {
    char m[256];
    snprintf(m, sizeof(m), "%s: %s", what, hipGetErrorString(hipGetLastError()));
    gtf::set_error(m);
    return -1;
}

// nodes per thread of the compact-list prepare (GTF_TAG_PREP_NPT 1 / 2 / 4; 0: the lane-group or
// thread-per-node prepare with the keep mask skipped). Measured (round 6): on C3 (2.0 M nodes)
// one node per thread 40 us against 48-49 us for the lane groups or two per thread; on C4
// (180 k nodes) the lane groups' wider launch is ahead.
static int tag_prep_npt(int n) {
    const char* e = getenv("GTF_TAG_PREP_NPT");
    if (e && e[0]) {
        const int v = atoi(e);
        if (v == 0 || v == 1 || v == 2 || v == 4) return v;
    }
    return n >= 2 * BLOCK * 512 ? 1 : 0;
}

static bool tag_pack_enabled() {   // (read per call: a test switches it in-process)
    const char* e = getenv("GTF_TAG_PACK");   // 0: each kept list at the front of its node's out-range
    return !(e && e[0] == '0');
}

// zero_count: n_processed zeroed here (else the caller has, or the prepare launch zeroes the
// nzero words at `zero`, n_processed among them)
static int tag_prepare(const gtf_graph* g, const double* radius, uint8_t* keep, uint8_t* processed,
                       int32_t* n_processed, bool zero_count, hipStream_t st, int32_t* zero = nullptr,
                       int nzero = 0, TagCsr csr = TagCsr{nullptr, nullptr, nullptr}) {
    // n_processed NULL: no count here (gtf_tag_propagate's first sweep counts the processed nodes)
    if (zero_count && hipMemsetAsync(n_processed, 0, sizeof(int32_t), st) != hipSuccess)
        return hip_fail("gtf_tag_prepare");
    if (g->n_nodes <= 0 && zero && hipMemsetAsync(zero, 0, nzero * sizeof(int32_t), st) != hipSuccess)
        return hip_fail("gtf_tag_prepare");
    if (g->n_nodes > 0 && !keep && csr.kcnt && tag_prep_npt(g->n_nodes) > 0) {   // the compact lists alone
        const int npt = tag_prep_npt(g->n_nodes);
        auto kern = npt == 4 ? k_tag_prepare_csr<4> : npt == 2 ? k_tag_prepare_csr<2> : k_tag_prepare_csr<1>;
        hipLaunchKernelGGL(kern, dim3((g->n_nodes + BLOCK * npt - 1) / (BLOCK * npt)), dim3(BLOCK), 0, st, *g,
                           radius, csr, zero, nzero, csr.kword && tag_pack_enabled() ? 1 : 0);
    } else if (g->n_nodes > 0 && g->out_sched) {   // lane groups over the sender schedule
        PrepBuckets pb;
        const int cnt[3] = {g->n_o4, g->n_o8, g->n_o16}, gs[3] = {4, 8, 16};
        const int4* l = reinterpret_cast<const int4*>(g->out_sched);
        const int2* ln = reinterpret_cast<const int2*>(g->out_lanes);
        pb.lanes[0] = ln;
        pb.lanes[1] = ln ? ln + 4 * g->n_o4 : nullptr;
        int total = 0;
        for (int q = 0; q < 3; q++) {
            pb.list[q] = l;
            l += cnt[q];
            pb.count[q] = cnt[q];
            pb.blocks[q] = (cnt[q] + BLOCK / gs[q] - 1) / (BLOCK / gs[q]);
            total += pb.blocks[q];
        }
        total += (g->n_nodes + BLOCK - 1) / BLOCK;   // nodes without an out-edge
        hipLaunchKernelGGL(k_tag_prepare_sched, dim3(total), dim3(BLOCK), 0, st, *g, radius, keep, processed, pb,
                           zero, nzero, csr);
    } else if (g->n_nodes > 0) {
        hipLaunchKernelGGL(k_tag_prepare, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, *g, radius,
                           keep, processed, zero, nzero, csr);
    }
    if (g->n_nodes > 0 && n_processed) {   // the processed count: a reduction of the processed bytes
        int blocks = (g->n_nodes / 16 + BLOCK * 4 - 1) / (BLOCK * 4);   // ~4 steps per thread
        blocks = blocks < 1 ? 1 : (blocks > 128 ? 128 : blocks);
        hipLaunchKernelGGL(k_count_flags, dim3(blocks), dim3(BLOCK), 0, st, processed, g->n_nodes, n_processed);
    }
    return hipGetLastError() == hipSuccess ? 0 : hip_fail("gtf_tag_prepare launch");
}

int gtf_tag_prepare(const gtf_graph* g, const double* radius, uint8_t* keep, uint8_t* processed,
                    int32_t* n_processed, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_prepare")) return rc;
    return tag_prepare(g, radius, keep, processed, n_processed, true, (hipStream_t)stream);
}

// flips: TAG_SHARDS counter words TAG_STRIDE apart (nsh = TAG_SHARDS, zeroed by the caller)
// or one word (nsh = 1, zeroed here)
static int tag_sweep(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed, const int64_t* tags_in,
                     int64_t* tags_out, int32_t* flips, int nsh, const TagCtl& ctl, hipStream_t st) {
    if (nsh == 1 && hipMemsetAsync(flips, 0, sizeof(int32_t), st) != hipSuccess) return hip_fail("gtf_tag_sweep");
    if (g->n_nodes > 0 && g->out_sched) {   // lane groups over the sender schedule
        TagBuckets tb;
        const int cnt[3] = {g->n_o4, g->n_o8, g->n_o16}, gs[3] = {4, 8, 16};
        const int4* l = reinterpret_cast<const int4*>(g->out_sched);
        const int2* ln = reinterpret_cast<const int2*>(g->out_lanes);
        tb.lanes[0] = ln;
        tb.lanes[1] = ln ? ln + 4 * g->n_o4 : nullptr;
        int total = 0;
        for (int q = 0; q < 3; q++) {
            tb.list[q] = l;
            l += cnt[q];
            tb.count[q] = cnt[q];
            tb.blocks[q] = (cnt[q] + BLOCK / gs[q] - 1) / (BLOCK / gs[q]);
            total += tb.blocks[q];
        }
        tb.copy_blocks = (g->n_nodes + BLOCK - 1) / BLOCK;   // nodes without an out-edge are not scheduled
        total += tb.copy_blocks;
        if (total > 0)
            hipLaunchKernelGGL(k_tag_sweep_sched, dim3(total), dim3(BLOCK), 0, st, *g, keep, processed, tags_in,
                               tags_out, flips, nsh, tb, ctl);
    } else if (g->n_nodes > 0) {
        hipLaunchKernelGGL(k_tag_sweep, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, *g, keep,
                           processed, tags_in, tags_out, flips, nsh, ctl);
    }
    return hipGetLastError() == hipSuccess ? 0 : hip_fail("gtf_tag_sweep launch");
}

int gtf_tag_sweep(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed, const int64_t* tags_in,
                  int64_t* tags_out, int32_t* flips, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_sweep")) return rc;
    const TagCtl none{nullptr, nullptr, nullptr, nullptr, 0.0, nullptr, nullptr};
    return tag_sweep(g, keep, processed, tags_in, tags_out, flips, 1, none, (hipStream_t)stream);
}

static size_t tag_align(size_t x) { return (x + 255) & ~size_t(255); }

// the stop-rule words of gtf_tag_propagate: processed count, stop flag, executed sweeps; then
// a ring of per-sweep flip counters, TAG_SHARDS words each (TAG_STRIDE apart)
constexpr int TAG_RING = 128;
constexpr size_t TAG_CTR = (size_t)TAG_SHARDS * TAG_STRIDE;   // int32 words per sweep
// the stop-rule words, the processed count's shards, then the ring of flip counters
constexpr size_t TAG_HDR = 64 * sizeof(int32_t) + TAG_CTR * sizeof(int32_t) + TAG_RING * TAG_CTR * sizeof(int32_t);

size_t gtf_tag_workspace_bytes(int32_t n_nodes, int32_t n_edges) {
    const size_t n = n_nodes > 0 ? (size_t)n_nodes : 1, e = n_edges > 0 ? (size_t)n_edges : 1;
    // header, keep mask, processed flags, the int64 ping-pong copy; then the compact kept lists
    // (count and packed word per node, neighbour indices per out-edge) and the int32 tag pair
    return tag_align(TAG_HDR) + tag_align(e) + tag_align(n) + tag_align(sizeof(int64_t) * n) +
           2 * tag_align(sizeof(int32_t) * n) + tag_align(sizeof(int32_t) * e) + tag_align(sizeof(int32_t) * 2 * n);
}

// batches of sweeps between two reads of the stop-rule words: at most the report's 64 totals
constexpr int32_t TAG_MAX_BATCH = 64;

// the mapped report of gtf_tag_propagate (one per host thread, kept): 4 header words + the
// flip totals of one batch. Coherent page-locked memory: the report kernel's system-scope
// stores reach the host while the stream runs.
struct TagReport {
    int32_t* host = nullptr;
    int32_t* dev = nullptr;
    int32_t seq = 0;
};
static TagReport& tag_report() {
    static thread_local TagReport r;
    static thread_local bool tried = false;
    if (!tried) {
        tried = true;
        void* h = nullptr;
        if (hipHostMalloc(&h, (4 + TAG_MAX_BATCH) * sizeof(int32_t),
                          hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) == hipSuccess) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
                r.host = static_cast<int32_t*>(h);
                r.dev = static_cast<int32_t*>(d);
                __atomic_store_n(r.host, 0, __ATOMIC_RELAXED);
            } else {
                (void)hipHostFree(h);
            }
        }
        (void)hipGetLastError();
    }
    return r;
}
static int32_t* tag_report_buffer() { return tag_report().host; }
static int32_t* tag_report_dev() { return tag_report().dev; }
static int32_t tag_next_seq() {
    TagReport& r = tag_report();
    r.seq = r.seq == INT32_MAX ? 1 : r.seq + 1;
    return r.seq;
}
static bool tag_poll_enabled() {   // (read per call: a test switches it in-process)
    const char* e = getenv("GTF_TAG_POLL");   // 0: the copy-and-synchronise read-back
    return !(e && e[0] == '0');
}
// the host waits for the report's sequence word; a stream that finished (or failed) without it
// showing ends the wait -- then the words are re-read once after the stream's completion
static int tag_wait_report(int32_t* rep, int32_t seq, hipStream_t st) {
    for (uint64_t spin = 1;; spin++) {
        if (__atomic_load_n(rep, __ATOMIC_ACQUIRE) == seq) break;
        if ((spin & 255) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                if (__atomic_load_n(rep, __ATOMIC_ACQUIRE) == seq) break;
                (void)hipGetLastError();
                gtf::set_error("gtf_tag_propagate: the report did not reach the host");
                return -1;
            }
            if (q != hipErrorNotReady) return hip_fail("gtf_tag_propagate: waiting for the report");
        }
        __builtin_ia32_pause();
    }
    (void)hipGetLastError();   // (a not-ready query leaves its status behind)
    return 0;
}

static bool tag_csr_enabled() {   // (read per call: a test switches it in-process)
    const char* e = getenv("GTF_TAG_CSR");   // 0: the scheduled sweep over the keep mask
    return !(e && e[0] == '0');
}
// nodes per thread of the compact-list sweep: 2 where that keeps >= 2 blocks per CU (256 CUs);
// 4 measured no faster on C3 (round 6)
static int tag_nodes_per_thread(int n) {
    const char* e = getenv("GTF_TAG_NPT");
    if (e && e[0]) {   // 1 / 2 / 4 (A/B)
        const int v = atoi(e);
        if (v == 1 || v == 2 || v == 4) return v;
    }
    return n >= 2 * BLOCK * 512 ? 2 : 1;
}
static int tag_sweep_r() {   // kept indices per node in the second round of a 2- / 4-node sweep
    const char* e = getenv("GTF_TAG_R");   // (GTF_TAG_R 2 / 4; C3: 2 at least as fast)
    return e && e[0] == '4' ? 4 : 2;
}
// sweeps in the first batch (then doubling): 4 -- a sweep enqueued past the stop returns at once
// (~1 us), a batch boundary costs a report and a host round trip (~10-15 us), and the stage
// runs 1 sweep (+1 that sees the stop) on ascending tags, 7-10 on the descending ones
static int32_t tag_first_batch() {
    const char* e = getenv("GTF_TAG_BATCH0");   // (A/B: 1, 2, 4, 8 ...)
    const int v = e && e[0] ? atoi(e) : 4;
    return v < 1 ? 1 : (v > TAG_MAX_BATCH ? TAG_MAX_BATCH : v);
}
static int tag_coop_groups() {   // the wave-cooperative sweep on packed lists: 64-node groups per wave (0: off)
    const char* e = getenv("GTF_TAG_COOP");
    if (e && e[0]) {
        const int v = atoi(e);
        return v == 1 || v == 2 || v == 4 ? v : 0;
    }
    return 2;
}
static bool tag_kword_enabled() {
    const char* e = getenv("GTF_TAG_KWORD");   // 0: the count and the offset per node
    return !(e && e[0] == '0');
}

static int32_t* tag_readback_buffer() {
    static thread_local int32_t* buf = nullptr;
    if (!buf && hipHostMalloc((void**)&buf, (64 + (1 + TAG_RING) * TAG_CTR) * sizeof(int32_t), hipHostMallocPortable) !=
                    hipSuccess)
        buf = nullptr;
    return buf;
}

// The whole stage behind one call: prepare, then the sweeps (the loop of
// tag_propagation.py:130-164, first sweep unconditional) in batches of 4, 8, 16, ... launches
// whose stop test runs on the device (TagCtl), over the compact kept lists with the tags
// ping-ponging between two int32 arrays (or `tags` and the workspace's int64 copy); the host
// reads the batch's flip counters once per batch and stops as soon as the rule has. The final
// tags land in `tags` by a device copy.
int gtf_tag_propagate(const gtf_graph* g, const double* radius, int64_t* tags, double flip_threshold,
                      int32_t max_sweeps, int32_t* flips_out, int32_t* sweeps_out, void* workspace,
                      size_t workspace_bytes, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_propagate")) return rc;
    if (!sweeps_out || (g->n_nodes > 0 && (!tags || !radius)) || max_sweeps < 0) {
        gtf::set_error("gtf_tag_propagate: null argument or negative max_sweeps");
        return -2;
    }
    const int32_t n_edges = g->n_nodes > 0 ? g->n_edges : 0;
    if (!workspace || workspace_bytes < gtf_tag_workspace_bytes(g->n_nodes, n_edges)) {
        gtf::set_error("gtf_tag_propagate: workspace smaller than gtf_tag_workspace_bytes()");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t n = g->n_nodes > 0 ? (size_t)g->n_nodes : 1, e = n_edges > 0 ? (size_t)n_edges : 1;
    char* w = static_cast<char*>(workspace);
    int32_t* hdr = reinterpret_cast<int32_t*>(w);   // [1] stop [2] executed
    int32_t* pshards = hdr + 64;                    // the processed count, TAG_SHARDS shards
    int32_t* ring = pshards + TAG_CTR;
    w += tag_align(TAG_HDR);
    uint8_t* keep = reinterpret_cast<uint8_t*>(w);
    w += tag_align(e);
    uint8_t* proc = reinterpret_cast<uint8_t*>(w);
    w += tag_align(n);
    int64_t* other = reinterpret_cast<int64_t*>(w);
    w += tag_align(sizeof(int64_t) * n);
    int32_t* kcnt = reinterpret_cast<int32_t*>(w);
    w += tag_align(sizeof(int32_t) * n);
    int32_t* kidx = reinterpret_cast<int32_t*>(w);
    w += tag_align(sizeof(int32_t) * e);
    int32_t* t32 = reinterpret_cast<int32_t*>(w);   // [2n]: the int32 ping-pong pair
    w += tag_align(sizeof(int32_t) * 2 * n);
    uint32_t* kword = reinterpret_cast<uint32_t*>(w);
    // the sweeps over compact kept lists with int32 tags (k_tag_sweep_csr; GTF_TAG_CSR=0: the
    // scheduled sweep of gtf_tag_sweep over the keep mask and processed flags, which only it
    // reads); one packed word per node where every list offset fits its 23 bits
    const bool csr = tag_csr_enabled();
    const bool packed = csr && (size_t)n_edges < ((size_t)1 << (32 - KW_BITS)) && tag_kword_enabled();
    const TagCsr lists{csr ? kcnt : nullptr, kidx, packed ? kword : nullptr};
    const int npt = tag_nodes_per_thread(g->n_nodes);
    // the wave-cooperative sweep where the thread prepare packs the lists (graphs the 2- / 4-node
    // sweeps take)
    const int coop = packed && npt > 1 && tag_prep_npt(g->n_nodes) > 0 && tag_pack_enabled() ? tag_coop_groups() : 0;
    int32_t* ovf = hdr + 3;   // (zeroed with the header by the prepare launch)
    *sweeps_out = 0;
    // the header words and the first sweep's counter shards zeroed by the prepare launch; every
    // executed sweep zeroes the next one's (TagCtl.next)
    int32_t* hostrep = tag_report_buffer();   // mapped page-locked report (NULL: read back by copy)
    const bool poll = hostrep && tag_poll_enabled();
    if (int rc = tag_prepare(g, radius, csr ? nullptr : keep, csr ? nullptr : proc, nullptr, false, st, hdr,
                             64 + 2 * (int)TAG_CTR, lists))
        return rc;
    int32_t s = 0, batch = tag_first_batch(), executed = 0;
    int32_t* host = poll ? nullptr : tag_readback_buffer();   // the header words, then the ring
    if (!poll && !host) return hip_fail("gtf_tag_propagate: page-locked read-back buffer");
    bool stopped = false;
    // the final tags into `tags` (k_tag_final: a copy when the executed count is odd), enqueued
    // after every batch -- before the host has read whether the batch stopped the loop -- so the
    // last one is already queued when it has: no launch on the stage's tail. An early copy is
    // harmless: the next batch's first sweep rewrites every tag of `tags` or reads it as copied.
    auto final_copy = [&]() -> int {
        if (g->n_nodes <= 0) return 0;
        if (csr)
            hipLaunchKernelGGL(k_tag_final_csr, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, tags, other,
                               t32, hdr + 2, ovf, g->n_nodes);
        else
            hipLaunchKernelGGL(k_tag_final, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, tags, other,
                               hdr + 2, g->n_nodes);
        return hipGetLastError() == hipSuccess ? 0 : hip_fail("gtf_tag_propagate: final copy");
    };
    bool copied = false;
    while (!stopped && s < max_sweeps) {
        const int32_t at = s % TAG_RING;
        int32_t nb = batch < max_sweeps - s ? batch : max_sweeps - s;
        if (nb > TAG_RING - at) nb = TAG_RING - at;   // the batch's counters stay contiguous in the ring
        for (int32_t i = 0; i < nb; i++) {
            const int32_t q = s + i;
            const TagCtl ctl{pshards, q > 0 ? ring + ((q - 1) % TAG_RING) * TAG_CTR : nullptr, hdr + 1, hdr + 2,
                             flip_threshold, ring + ((q + 1) % TAG_RING) * TAG_CTR, q == 0 ? pshards : nullptr};
            int64_t* tin = (q & 1) ? other : tags;
            int64_t* tout = (q & 1) ? tags : other;
            if (csr) {
                if (g->n_nodes > 0) {
                    int32_t* b0 = t32 + (size_t)(q & 1) * n;         // sweep q reads buffer q % 2 ...
                    int32_t* b1 = t32 + (size_t)((q + 1) & 1) * n;   // ... and writes the other
                    auto kern = npt == 1   ? k_tag_sweep_csr1
                                : npt == 4 ? (tag_sweep_r() == 4 ? k_tag_sweep_csr<4, 4> : k_tag_sweep_csr<4, 2>)
                                           : (tag_sweep_r() == 4 ? k_tag_sweep_csr<2, 4> : k_tag_sweep_csr<2, 2>);
                    int per_block = BLOCK * npt;
                    if (coop) {
                        kern = coop == 1 ? k_tag_sweep_coop<1> : coop == 4 ? k_tag_sweep_coop<4> : k_tag_sweep_coop<2>;
                        per_block = BLOCK * coop;
                    }
                    hipLaunchKernelGGL(kern, dim3((g->n_nodes + per_block - 1) / per_block), dim3(BLOCK), 0,
                                       st, *g, lists, tin, tout, b0, b1, q == 0 ? 1 : 0, ovf,
                                       ring + (q % TAG_RING) * TAG_CTR, TAG_SHARDS, ctl);
                    if (hipGetLastError() != hipSuccess) return hip_fail("gtf_tag_propagate: sweep launch");
                }
            } else if (int rc = tag_sweep(g, keep, proc, tin, tout, ring + (q % TAG_RING) * TAG_CTR, TAG_SHARDS, ctl,
                                          st)) {
                return rc;
            }
        }
        int32_t words[3];   // processed, stop, executed
        const int32_t* fl;  // flips of sweeps s, s + 1, ...
        std::vector<int32_t> tot;
        if (poll) {
            // one small launch writes the words and the batch's flip totals into the mapped report;
            // the host waits for its sequence word instead of a copy and a stream synchronisation
            const int32_t seq = tag_next_seq();
            hipLaunchKernelGGL(k_tag_report, dim3(1), dim3(64), 0, st, hdr, pshards, ring, s, nb, TAG_RING,
                               tag_report_dev(), seq);
            if (hipGetLastError() != hipSuccess) return hip_fail("gtf_tag_propagate: report launch");
            if (int rc = final_copy()) return rc;
            copied = true;
            if (int rc = tag_wait_report(hostrep, seq, st)) return rc;
            for (int k = 0; k < 3; k++) words[k] = hostrep[1 + k];
            fl = hostrep + 4;
        } else {
            // one read-back: the header words through the batch's last counter
            if (int rc = final_copy()) return rc;
            copied = true;
            if (hipMemcpyAsync(host, hdr, (64 + (1 + at + nb) * TAG_CTR) * sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
                    hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return hip_fail("gtf_tag_propagate: reading the flip counts");
            words[0] = 0;
            for (int k = 0; k < TAG_SHARDS; k++) words[0] += host[64 + k * TAG_STRIDE];
            for (int k = 1; k < 3; k++) words[k] = host[k];
            tot.resize(nb);
            for (int32_t i = 0; i < nb; i++) {
                const int32_t* c = host + 64 + (1 + at + i) * TAG_CTR;
                int32_t f = 0;
                for (int k = 0; k < TAG_SHARDS; k++) f += c[k * TAG_STRIDE];
                tot[i] = f;
            }
            fl = tot.data();
        }
        executed = words[2];
        for (int32_t q = s; q < executed; q++) {
            const int32_t f = fl[q - s];
            if (flips_out) flips_out[q] = f;
            // the rule on the host too: the batch's last executed sweep may already stop it
            const double frac = words[0] ? (double)f / (double)words[0] : 0.0;
            if (q == executed - 1 && !(frac > flip_threshold)) stopped = true;
        }
        stopped = stopped || words[1] != 0 || executed < s + nb;
        s = executed;
        if (batch < TAG_MAX_BATCH) batch *= 2;
    }
    *sweeps_out = executed;
    if (!copied) return final_copy();   // (no sweep at all)
    return 0;
}

int gtf_tag_sweep_shard(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed, const int64_t* tags_in,
                        int64_t* tags_out, const gtf_shard* shard, int32_t rank, int32_t nranks,
                        gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_sweep_shard")) return rc;
    if (!shard || rank < 0 || rank >= nranks || shard->node_lo < 0 || shard->node_hi < shard->node_lo ||
        shard->node_hi > g->n_nodes) {
        gtf::set_error("gtf_tag_sweep_shard: owned node range or rank out of bounds");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    int64_t* words = tags_out + g->n_nodes;   // the nranks flip-count words
    if (hipMemsetAsync(words, 0, sizeof(int64_t) * (size_t)nranks, st) != hipSuccess)
        return hip_fail("gtf_tag_sweep_shard");
    if (g->n_nodes > 0)
        hipLaunchKernelGGL(k_tag_sweep_owned, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, *g, keep,
                           processed, tags_in, tags_out, shard->node_lo, shard->node_hi,
                           reinterpret_cast<unsigned long long*>(words + rank));
    return hipGetLastError() == hipSuccess ? 0 : hip_fail("gtf_tag_sweep_shard launch");
}

}  // extern "C"
