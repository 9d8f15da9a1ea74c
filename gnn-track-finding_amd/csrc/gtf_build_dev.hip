// gtf_build_dev.hip -- event conversion's graph build on the GPU ("CSV ->
// CSR directly" on the device): the same packed CSR, in the same networkx orders, as the
// host builder gtf_build_event_csr (gtf_build.cpp), from device arrays of the CSV columns.
//
// The reference (helper.construct_graph, helper.py:465-521; event_conversion.py:63-84)
// adds both directions of every edges.csv row to a networkx DiGraph, splits it into
// weakly connected components and copies each one; the orders that come out of that are
// what every later stage depends on. Here, as sorts, scans and per-segment threads:
//
//   1. node ids -> CSV index: radix sort of (id, index), binary search per row end;
//   2. G's successor lists in insertion order: both directions of row r at times 2r and
//      2r + 1, a stable radix sort by (u, v) keeps each pair's first time (networkx keeps
//      a repeated edge's first position), a second one by (u, time) gives succ[u] in
//      insertion order;
//   3. weakly connected components by hook + pointer jumping to the minimum CSV index
//      (= the node networkx's component loop starts from, so components come out in
//      root order);
//   4. node order of each component's copy: CSV-index order when 2|c| >= |G| (FilterAtlas
//      iterates G), else CPython 3.10 set order -- one thread per such component runs the
//      BFS (successors in insertion order; the graph is symmetric, so the predecessor
//      loop adds nothing) into a set table and copies it into a second one
//      (show_nodes(set(c))), exactly as gtf_build.cpp's PySet does, in global scratch;
//   5. slots: (packed receiver, packed sender) sorted, so each receiver's predecessors
//      come in copy node order; out-lists keep G's successor order; the
//      track_state_estimates key order reversed(set(chain(pred, succ))) (helper.py:277,
//      350-351) from one set table per node.
//
// Integer and byte work only: sorts and scans are hipCUB, the rest one thread per row /
// edge / node / component. Not on the timed path (once per event).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "../../include/gtf.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

constexpr int BLOCK = 256;
inline int grid(int64_t n) { return (int)((n + BLOCK - 1) / BLOCK); }
inline size_t al(size_t x) { return (x + 255) & ~size_t(255); }

constexpr uint64_t NONE = ~uint64_t(0);
constexpr int32_t ERR_DUP = 1, ERR_RANGE = 2, ERR_ASYM = 4, ERR_OVER = 8;

// final table size of a CPython 3.10 set after n distinct insertions (start 8, resize when
// fill * 5 >= mask * 3 to the next power of two above 4 * fill, 2 * fill past 50000)
__host__ __device__ inline int64_t set_capacity(int64_t n) {
    int64_t mask = 7;
    for (int64_t fill = 1; fill <= n; fill++) {
        if (fill * 5 >= mask * 3) {
            const int64_t minused = fill > 50000 ? fill * 2 : fill * 4;
            int64_t ns = 8;
            while (ns <= minused) ns <<= 1;
            mask = ns - 1;
        }
    }
    return mask + 1;
}

// CPython 3.10 set of non-negative ints in caller memory: `a` the live table, `b` a spare
// of the same capacity (set_capacity of the distinct keys to come), swapped on resize
struct DevSet {
    int64_t* a;
    int64_t* b;
    int64_t mask;
    int64_t fill;
    int64_t cap;        // entries of each table (a resize beyond it sets `over` and stops)
    bool over;

    __device__ void init(int64_t* t0, int64_t* t1, int64_t capacity) {
        a = t0;
        b = t1;
        mask = 7;
        fill = 0;
        cap = capacity;
        over = capacity < 8;
        if (!over)
            for (int i = 0; i < 8; i++) a[i] = -1;
    }
    __device__ void insert_clean(int64_t key) {
        uint64_t perturb = (uint64_t)key;
        int64_t i = key & mask;
        for (;;) {
            if (a[i] < 0) { a[i] = key; return; }
            if (i + 9 <= mask)
                for (int64_t j = 1; j <= 9; j++)
                    if (a[i + j] < 0) { a[i + j] = key; return; }
            perturb >>= 5;
            i = (int64_t)(((uint64_t)i * 5 + 1 + perturb) & (uint64_t)mask);
        }
    }
    __device__ void resize(int64_t minused) {
        int64_t ns = 8;
        while (ns <= minused) ns <<= 1;
        if (ns > cap) { over = true; return; }   // more distinct keys than the table was sized for
        int64_t* old = a;
        const int64_t om = mask;
        a = b;
        b = old;
        mask = ns - 1;
        for (int64_t i = 0; i <= mask; i++) a[i] = -1;
        for (int64_t i = 0; i <= om; i++)
            if (old[i] >= 0) insert_clean(old[i]);
    }
    __device__ void add(int64_t key) {
        if (over) return;
        uint64_t perturb = (uint64_t)key;
        int64_t i = key & mask;
        for (;;) {
            int64_t probes = (i + 9 <= mask) ? 9 : 0;
            int64_t j = i;
            for (;;) {
                if (a[j] < 0) {
                    a[j] = key;
                    fill++;
                    if (fill * 5 >= mask * 3) resize(fill > 50000 ? fill * 2 : fill * 4);
                    return;
                }
                if (a[j] == key) return;
                if (probes-- == 0) break;
                j++;
            }
            perturb >>= 5;
            i = (int64_t)(((uint64_t)i * 5 + 1 + perturb) & (uint64_t)mask);
        }
    }
};

// CSV index of node id `key` (ids sorted ascending), -1 if absent
__device__ inline int32_t find_id(const uint64_t* ids, const int32_t* idx, int32_t n, int64_t key) {
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (ids[m] < (uint64_t)key) lo = m + 1;
        else hi = m;
    }
    return (lo < n && ids[lo] == (uint64_t)key) ? idx[lo] : -1;
}

// first position in [b, e) of slot_src holding >= x
__device__ inline int32_t lower(const int32_t* s, int32_t b, int32_t e, int32_t x) {
    while (b < e) {
        const int32_t m = (b + e) >> 1;
        if (s[m] < x) b = m + 1;
        else e = m;
    }
    return b;
}

__global__ void k_iota(int32_t* a, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}

__global__ void k_check_ids(const uint64_t* ids, int64_t n, int32_t* err) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    if (ids[i] >= ((uint64_t)1 << 61) - 1) atomicOr(err, ERR_RANGE);   // also catches negatives
    if (i > 0 && ids[i] == ids[i - 1]) atomicOr(err, ERR_DUP);
}

// both directions of row r at times 2r (a -> b) and 2r + 1 (b -> a); rows naming a node
// outside the window are dropped (helper.py:512-518 adds edges between kept nodes only)
__global__ void k_rows(const int64_t* ra, const int64_t* rb, int64_t R, const uint64_t* ids, const int32_t* idx,
                       int32_t n, uint64_t* key, int32_t* t) {
    const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= R) return;
    const int32_t ia = find_id(ids, idx, n, ra[r]), ib = find_id(ids, idx, n, rb[r]);
    const bool ok = ia >= 0 && ib >= 0;
    key[2 * r] = ok ? ((uint64_t)ia << 32) | (uint32_t)ib : NONE;
    key[2 * r + 1] = ok ? ((uint64_t)ib << 32) | (uint32_t)ia : NONE;
    t[2 * r] = (int32_t)(2 * r);
    t[2 * r + 1] = (int32_t)(2 * r + 1);
}

// sorted by (u, v) with times ascending inside a pair: keep each pair's first insertion,
// re-keyed by (u, time) with v as the value
__global__ void k_first(const uint64_t* key, const int32_t* t, int64_t n, uint64_t* k2, int32_t* v2) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    const bool keep = k != NONE && (i == 0 || key[i - 1] != k);
    k2[i] = keep ? ((k >> 32) << 33) | (uint32_t)t[i] : NONE;
    v2[i] = (int32_t)(k & 0xffffffffu);
}

__global__ void k_count_valid(const uint64_t* k, int64_t n, int32_t* m) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    // sorted: the valid keys form a prefix; its end is where NONE starts
    if (k[i] != NONE && (i + 1 == n || k[i + 1] == NONE)) *m = (int32_t)(i + 1);
}

__global__ void k_gdeg(const uint64_t* k, int32_t m, int32_t* deg) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < m) atomicAdd(&deg[k[i] >> 33], 1);
}

__global__ void k_lab_init(int32_t* lab, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) lab[i] = (int32_t)i;
}

// hook the larger root under the smaller one (labels only decrease, so every component
// ends labelled by its minimum CSV index)
__global__ void k_hook(const uint64_t* k, const int32_t* v, int32_t m, int32_t* lab, int32_t* changed) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    const int32_t a = lab[(int32_t)(k[i] >> 33)], b = lab[v[i]];
    if (a == b) return;
    atomicMin(&lab[a > b ? a : b], a < b ? a : b);
    *changed = 1;
}

__global__ void k_compress(int32_t* lab, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    int32_t l = lab[i];
    while (lab[l] != l) l = lab[l];
    lab[i] = l;
}

__global__ void k_isroot(const int32_t* lab, int64_t n, int32_t* isroot) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i <= n) isroot[i] = (i < n && lab[i] == i) ? 1 : 0;
}

__global__ void k_comp_of(const int32_t* lab, const int32_t* rank, int64_t n, int32_t* comp, int32_t* size,
                          uint64_t* key) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int32_t c = rank[lab[i]];
    comp[i] = c;
    key[i] = (uint64_t)c;
    atomicAdd(&size[c], 1);
}

// members of every component in CSV-index order (the stable sort by component): the
// copy's node order when 2|c| >= |G|
__global__ void k_order_sorted(const int32_t* memb, const int32_t* comp, const int32_t* size, int64_t n,
                               int32_t* order) {
    const int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const int32_t g = memb[p];
    if (2 * (int64_t)size[comp[g]] >= n) order[p] = g;
}

__global__ void k_comp_words(const int32_t* size, int32_t n_sub, int64_t n, int64_t* words) {
    const int32_t c = blockIdx.x * BLOCK + threadIdx.x;
    if (c > n_sub) return;
    words[c] = (c < n_sub && 2 * (int64_t)size[c] < n) ? 3 * set_capacity(size[c]) : 0;
}

// one thread per component smaller than half the graph: BFS from its root in successor
// order into set(...) (nx.weakly_connected_components: set(_plain_bfs(G, root))), then the
// copy's node order = the order of a second set filled from the first (show_nodes)
__global__ void k_comp_order(const int32_t* memb, const int32_t* coff, const int32_t* size, int32_t n_sub, int64_t n,
                             const int32_t* gptr, const uint64_t* gkey, const int32_t* gdst, const int64_t* node_id,
                             const uint64_t* ids, const int32_t* idx, const int64_t* toff, int64_t* tbl,
                             int32_t* queue, uint8_t* seen, int32_t* order, int32_t* err) {
    const int32_t c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= n_sub || 2 * (int64_t)size[c] >= n) return;
    const int32_t lo = coff[c], sz = size[c];
    const int64_t cap = set_capacity(sz);
    int64_t* t = tbl + toff[c];
    DevSet s;
    s.init(t, t + cap, cap);
    const int32_t root = memb[lo];
    int32_t head = lo, tail = lo;
    seen[root] = 1;
    s.add(node_id[root]);
    queue[tail++] = root;
    while (head < tail) {
        const int32_t v = queue[head++];
        for (int32_t j = gptr[v]; j < gptr[v + 1]; j++) {
            const int32_t w = gdst[j];
            if (!seen[w]) {
                seen[w] = 1;
                s.add(node_id[w]);
                queue[tail++] = w;
            }
        }
    }
    (void)gkey;
    DevSet shown;
    int64_t* spare = (s.a == t) ? t + cap : t;   // the first set's spare table
    shown.init(spare, t + 2 * cap, cap);
    for (int64_t i = 0; i <= s.mask; i++)
        if (s.a[i] >= 0) shown.add(s.a[i]);
    if (s.over || shown.over) { atomicOr(err, ERR_OVER); return; }
    int32_t r = lo;
    for (int64_t i = 0; i <= shown.mask; i++)
        if (shown.a[i] >= 0) order[r++] = find_id(ids, idx, (int32_t)n, shown.a[i]);
}

__global__ void k_pos(const int32_t* order, const int32_t* comp, int64_t n, int32_t* pos, int32_t* sub_id) {
    const int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    pos[order[p]] = (int32_t)p;
    sub_id[p] = comp[order[p]];
}

// every kept edge u -> v as (packed receiver, packed sender): sorted, each receiver's
// predecessors come in copy node order (the copy adds edges in its node order)
__global__ void k_slot_keys(const uint64_t* gkey, const int32_t* gdst, int32_t m, const int32_t* pos, uint64_t* sk,
                            int32_t* rdeg) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    const int32_t q = pos[gdst[i]], p = pos[(int32_t)(gkey[i] >> 33)];
    sk[i] = ((uint64_t)q << 32) | (uint32_t)p;
    atomicAdd(&rdeg[q], 1);
}

__global__ void k_slot_src(const uint64_t* sk, int32_t m, int32_t* slot_src) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < m) slot_src[i] = (int32_t)(sk[i] & 0xffffffffu);
}

__global__ void k_outdeg(const int32_t* order, const int32_t* gdeg, int64_t n, int32_t* od) {
    const int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p <= n) od[p] = p < n ? gdeg[order[p]] : 0;
}

// out-list of packed sender p in G's successor order: the slot of p in each receiver
__global__ void k_out_slot(const uint64_t* gkey, const int32_t* gdst, const int32_t* gptr, int32_t m,
                           const int32_t* pos, const int32_t* slot_ptr, const int32_t* slot_src,
                           const int32_t* out_ptr, int32_t* out_slot) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    const int32_t u = (int32_t)(gkey[i] >> 33), p = pos[u], q = pos[gdst[i]];
    out_slot[out_ptr[p] + (i - gptr[u])] = lower(slot_src, slot_ptr[q], slot_ptr[q + 1], p);
}

__global__ void k_tse_words(const int32_t* slot_ptr, int64_t n, int64_t* words) {
    const int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p <= n) words[p] = p < n ? 2 * set_capacity(slot_ptr[p + 1] - slot_ptr[p]) : 0;
}

// track_state_estimates key order of packed node p: reversed(set(chain(pred, succ)))
// with the copy's predecessors (slot order) then G's successors
__global__ void k_tse_rank(const int32_t* order, int64_t n, const int32_t* slot_ptr, const int32_t* slot_src,
                           const int32_t* gptr, const int32_t* gdst, const int32_t* pos, const int64_t* node_id,
                           const uint64_t* ids, const int32_t* idx, const int64_t* toff, int64_t* tbl,
                           int32_t* tse_rank, int32_t* err) {
    const int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n) return;
    const int32_t b = slot_ptr[p], e = slot_ptr[p + 1], u = order[p];
    const int64_t cap = set_capacity(e - b);
    DevSet s;
    s.init(tbl + toff[p], tbl + toff[p] + cap, cap);
    for (int32_t k = b; k < e; k++) {
        s.add(node_id[order[slot_src[k]]]);
        tse_rank[k] = -1;
    }
    for (int32_t j = gptr[u]; j < gptr[u + 1]; j++) s.add(node_id[gdst[j]]);
    if (s.over) { atomicOr(err, ERR_OVER); return; }
    int32_t r = 0;
    for (int64_t i = s.mask; i >= 0; i--) {   // reversed iteration order
        if (s.a[i] < 0) continue;
        const int32_t q = pos[find_id(ids, idx, (int32_t)n, s.a[i])];
        const int32_t f = lower(slot_src, b, e, q);
        if (f == e || slot_src[f] != q) { atomicOr(err, ERR_ASYM); return; }
        tse_rank[f] = r++;
    }
}

struct BuildWs {
    uint64_t *ids, *ka, *kb, *gk;
    int32_t *idx, *iota, *va, *vb, *gv;
    int32_t *gdeg, *gptr, *lab, *isroot, *rank, *comp, *size, *coff, *memb, *pos, *queue, *rdeg, *od;
    uint8_t* seen;
    int64_t *words, *toff, *tbl;
    int32_t* scal;   // [0] error bits, [1] changed, [2] valid edges
    void* cub;
    size_t cub_bytes, tbl_words;
};

size_t cub_need(int64_t n) {
    size_t a = 0, b = 0, c = 0, d = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (int)n);
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int32_t*)nullptr, (int32_t*)nullptr, (int)n + 1);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, d, (int64_t*)nullptr, (int64_t*)nullptr, (int)n + 1);
    size_t m = a > b ? a : b;
    m = m > c ? m : c;
    return m > d ? m : d;
}

// capacity bound: a set of k distinct keys has a table of <= 8 max(k, 1) entries, so the
// component tables (3 per component) take <= 24 N words and the key-order tables (2 per
// node) <= 16 (S + N)
BuildWs carve(void* base, int64_t N, int64_t R, bool with_ptrs) {
    const int64_t E2 = 2 * R, M = N > E2 ? N : E2, n1 = N + 1;
    char* p = (char*)base;
    BuildWs w;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes ? bytes : 1); return (void*)q; };
    w.ids = (uint64_t*)take(8 * N);
    w.ka = (uint64_t*)take(8 * M);
    w.kb = (uint64_t*)take(8 * M);
    w.idx = (int32_t*)take(4 * N);
    w.iota = (int32_t*)take(4 * M);
    w.va = (int32_t*)take(4 * M);
    w.vb = (int32_t*)take(4 * M);
    w.gk = (uint64_t*)take(8 * (E2 > 0 ? E2 : 1));
    w.gv = (int32_t*)take(4 * (E2 > 0 ? E2 : 1));
    w.gdeg = (int32_t*)take(4 * n1);
    w.gptr = (int32_t*)take(4 * n1);
    w.lab = (int32_t*)take(4 * n1);
    w.isroot = (int32_t*)take(4 * n1);
    w.rank = (int32_t*)take(4 * n1);
    w.comp = (int32_t*)take(4 * n1);
    w.size = (int32_t*)take(4 * n1);
    w.coff = (int32_t*)take(4 * n1);
    w.memb = (int32_t*)take(4 * n1);
    w.pos = (int32_t*)take(4 * n1);
    w.queue = (int32_t*)take(4 * n1);
    w.rdeg = (int32_t*)take(4 * n1);
    w.od = (int32_t*)take(4 * n1);
    w.seen = (uint8_t*)take(n1);
    w.words = (int64_t*)take(8 * n1);
    w.toff = (int64_t*)take(8 * n1);
    w.scal = (int32_t*)take(64);
    w.cub_bytes = cub_need(M > n1 ? M : n1);
    w.cub = take(w.cub_bytes);
    const int64_t t1 = 24 * (N > 0 ? N : 1), t2 = 16 * (E2 + N + 1);
    w.tbl_words = (size_t)(t1 > t2 ? t1 : t2);
    w.tbl = (int64_t*)take(8 * w.tbl_words);
    (void)with_ptrs;
    return w;
}

size_t carve_bytes(int64_t N, int64_t R) {
    BuildWs w = carve((void*)(uintptr_t)0, N, R, false);
    return (size_t)((char*)w.tbl - (char*)0) + al(8 * w.tbl_words) + 256;
}

}  // namespace

extern "C" {

size_t gtf_build_event_device_workspace_bytes(int64_t n_nodes, int64_t n_rows) {
    return carve_bytes(n_nodes > 0 ? n_nodes : 0, n_rows > 0 ? n_rows : 0);
}

int gtf_build_event_csr_device(gtf_event_csr* ev, void* workspace, size_t workspace_bytes, gtf_stream_t stream) {
    if (!ev || ev->n_nodes < 0 || ev->n_rows < 0 || (ev->n_nodes && !ev->node_id) ||
        (ev->n_rows && (!ev->row_a || !ev->row_b)) || !ev->order || !ev->sub_id || !ev->slot_ptr || !ev->out_ptr ||
        (ev->n_rows && (!ev->slot_src || !ev->tse_rank || !ev->out_slot)) || !workspace) {
        gtf::set_error("gtf_build_event_csr_device: bad arguments");
        return -2;
    }
    const int64_t N = ev->n_nodes, R = ev->n_rows, E2 = 2 * R;
    if (N > INT32_MAX / 2 || E2 > INT32_MAX / 2) {
        gtf::set_error("gtf_build_event_csr_device: graph too large for int32 indices");
        return -2;
    }
    if (workspace_bytes < carve_bytes(N, R)) {
        gtf::set_error("gtf_build_event_csr_device: workspace smaller than gtf_build_event_device_workspace_bytes");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    BuildWs w = carve(workspace, N, R, true);
    auto fail = [&](const char* what) {
        gtf::set_error(what);
        return -1;
    };
#define GTF_CK(x, what) \
    if ((x) != hipSuccess) return fail(what)
    const int32_t zero4[3] = {0, 0, 0};
    GTF_CK(hipMemcpyAsync(w.scal, zero4, sizeof(zero4), hipMemcpyHostToDevice, st), "scalars");
    if (N == 0) {
        GTF_CK(hipMemsetAsync(ev->slot_ptr, 0, 4, st), "memset");
        GTF_CK(hipMemsetAsync(ev->out_ptr, 0, 4, st), "memset");
        GTF_CK(hipStreamSynchronize(st), "sync");
        ev->n_edges = 0;
        ev->n_subgraphs = 0;
        return 0;
    }
    const int64_t M2 = N > E2 ? N : E2;
    size_t cb;
    // 1. ids -> CSV index
    hipLaunchKernelGGL(k_iota, dim3(grid(M2)), dim3(BLOCK), 0, st, w.iota, M2);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, (const uint64_t*)ev->node_id, w.ids, w.iota, w.idx, (int)N, 0,
                                              64, st), "sort ids");
    hipLaunchKernelGGL(k_check_ids, dim3(grid(N)), dim3(BLOCK), 0, st, w.ids, N, w.scal);
    // 2. G's successor lists in insertion order
    int32_t m = 0;
    if (R > 0) {
        hipLaunchKernelGGL(k_rows, dim3(grid(R)), dim3(BLOCK), 0, st, ev->row_a, ev->row_b, R, w.ids, w.idx, (int32_t)N,
                           w.ka, w.va);
        cb = w.cub_bytes;
        GTF_CK(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.ka, w.kb, w.va, w.vb, (int)E2, 0, 64, st), "sort pairs");
        hipLaunchKernelGGL(k_first, dim3(grid(E2)), dim3(BLOCK), 0, st, w.kb, w.vb, E2, w.ka, w.va);
        cb = w.cub_bytes;
        GTF_CK(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.ka, w.gk, w.va, w.gv, (int)E2, 0, 64, st), "sort succ");
        hipLaunchKernelGGL(k_count_valid, dim3(grid(E2)), dim3(BLOCK), 0, st, w.gk, E2, w.scal + 2);
    }
    int32_t scal[3];
    GTF_CK(hipMemcpyAsync(scal, w.scal, sizeof(scal), hipMemcpyDeviceToHost, st), "read");
    GTF_CK(hipStreamSynchronize(st), "sync");
    if (scal[0] & ERR_RANGE) { gtf::set_error("gtf_build_event_csr_device: node ids must be in [0, 2^61 - 1)"); return -2; }
    if (scal[0] & ERR_DUP) { gtf::set_error("gtf_build_event_csr_device: duplicate node id"); return -2; }
    m = scal[2];
    const uint64_t* gkey = w.gk;   // kept edges by (u, insertion time); value: v
    const int32_t* gdst = w.gv;
    GTF_CK(hipMemsetAsync(w.gdeg, 0, 4 * (N + 1), st), "memset");
    if (m > 0) hipLaunchKernelGGL(k_gdeg, dim3(grid(m)), dim3(BLOCK), 0, st, gkey, m, w.gdeg);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.gdeg, w.gptr, (int)N + 1, st), "scan");
    // 3. weakly connected components, labelled by their minimum CSV index
    hipLaunchKernelGGL(k_lab_init, dim3(grid(N)), dim3(BLOCK), 0, st, w.lab, N);
    for (int round = 0; m > 0; round++) {
        if (round > 200) return fail("gtf_build_event_csr_device: components did not converge");
        int32_t z = 0, changed = 0;
        GTF_CK(hipMemcpyAsync(w.scal + 1, &z, 4, hipMemcpyHostToDevice, st), "flag");
        hipLaunchKernelGGL(k_hook, dim3(grid(m)), dim3(BLOCK), 0, st, gkey, gdst, m, w.lab, w.scal + 1);
        hipLaunchKernelGGL(k_compress, dim3(grid(N)), dim3(BLOCK), 0, st, w.lab, N);
        GTF_CK(hipMemcpyAsync(&changed, w.scal + 1, 4, hipMemcpyDeviceToHost, st), "flag");
        GTF_CK(hipStreamSynchronize(st), "sync");
        if (!changed) break;
    }
    hipLaunchKernelGGL(k_isroot, dim3(grid(N + 1)), dim3(BLOCK), 0, st, w.lab, N, w.isroot);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.isroot, w.rank, (int)N + 1, st), "scan");
    int32_t n_sub = 0;
    GTF_CK(hipMemcpyAsync(&n_sub, w.rank + N, 4, hipMemcpyDeviceToHost, st), "read");
    GTF_CK(hipMemsetAsync(w.size, 0, 4 * (N + 1), st), "memset");
    hipLaunchKernelGGL(k_comp_of, dim3(grid(N)), dim3(BLOCK), 0, st, w.lab, w.rank, N, w.comp, w.size, w.ka);
    GTF_CK(hipStreamSynchronize(st), "sync");
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.size, w.coff, n_sub + 1, st), "scan");
    // 4. node order of every component's copy: CSV-index order (the stable sort by
    // component), replaced by the set order for components under half the graph
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.ka, w.kb, w.iota, w.memb, (int)N, 0, 32, st),
           "sort members");
    hipLaunchKernelGGL(k_order_sorted, dim3(grid(N)), dim3(BLOCK), 0, st, w.memb, w.comp, w.size, N, ev->order);
    hipLaunchKernelGGL(k_comp_words, dim3(grid(n_sub + 1)), dim3(BLOCK), 0, st, w.size, n_sub, N, w.words);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.words, w.toff, n_sub + 1, st), "scan");
    int64_t words = 0;
    GTF_CK(hipMemcpyAsync(&words, w.toff + n_sub, 8, hipMemcpyDeviceToHost, st), "read");
    GTF_CK(hipStreamSynchronize(st), "sync");
    if ((size_t)words > w.tbl_words) return fail("gtf_build_event_csr_device: set tables exceed the workspace bound");
    GTF_CK(hipMemsetAsync(w.seen, 0, N, st), "memset");
    hipLaunchKernelGGL(k_comp_order, dim3(grid(n_sub)), dim3(BLOCK), 0, st, w.memb, w.coff, w.size, n_sub, N, w.gptr,
                       gkey, gdst, ev->node_id, w.ids, w.idx, w.toff, w.tbl, w.queue, w.seen, ev->order, w.scal);
    hipLaunchKernelGGL(k_pos, dim3(grid(N)), dim3(BLOCK), 0, st, ev->order, w.comp, N, w.pos, ev->sub_id);
    // 5. slots: (packed receiver, packed sender) in order; the out-lists; the key orders
    GTF_CK(hipMemsetAsync(w.rdeg, 0, 4 * (N + 1), st), "memset");
    if (m > 0) {
        hipLaunchKernelGGL(k_slot_keys, dim3(grid(m)), dim3(BLOCK), 0, st, gkey, gdst, m, w.pos, w.ka, w.rdeg);
        cb = w.cub_bytes;
        GTF_CK(hipcub::DeviceRadixSort::SortKeys(w.cub, cb, w.ka, w.kb, m, 0, 64, st), "sort slots");
        hipLaunchKernelGGL(k_slot_src, dim3(grid(m)), dim3(BLOCK), 0, st, w.kb, m, ev->slot_src);
    }
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.rdeg, ev->slot_ptr, (int)N + 1, st), "scan");
    hipLaunchKernelGGL(k_outdeg, dim3(grid(N + 1)), dim3(BLOCK), 0, st, ev->order, w.gdeg, N, w.od);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.od, ev->out_ptr, (int)N + 1, st), "scan");
    if (m > 0)
        hipLaunchKernelGGL(k_out_slot, dim3(grid(m)), dim3(BLOCK), 0, st, gkey, gdst, w.gptr, m, w.pos, ev->slot_ptr,
                           ev->slot_src, ev->out_ptr, ev->out_slot);
    hipLaunchKernelGGL(k_tse_words, dim3(grid(N + 1)), dim3(BLOCK), 0, st, ev->slot_ptr, N, w.words);
    cb = w.cub_bytes;
    GTF_CK(hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.words, w.toff, (int)N + 1, st), "scan");
    GTF_CK(hipMemcpyAsync(&words, w.toff + N, 8, hipMemcpyDeviceToHost, st), "read");
    GTF_CK(hipStreamSynchronize(st), "sync");
    if ((size_t)words > w.tbl_words) return fail("gtf_build_event_csr_device: set tables exceed the workspace bound");
    hipLaunchKernelGGL(k_tse_rank, dim3(grid(N)), dim3(BLOCK), 0, st, ev->order, N, ev->slot_ptr, ev->slot_src, w.gptr,
                       gdst, w.pos, ev->node_id, w.ids, w.idx, w.toff, w.tbl, ev->tse_rank, w.scal);
    GTF_CK(hipGetLastError(), "launch");
    GTF_CK(hipMemcpyAsync(scal, w.scal, 4, hipMemcpyDeviceToHost, st), "read");
    GTF_CK(hipStreamSynchronize(st), "sync");
    if (scal[0] & ERR_OVER) {
        gtf::set_error("gtf_build_event_csr_device: a set held more keys than its table was sized for");
        return -1;
    }
    if (scal[0] & ERR_ASYM) {
        gtf::set_error("gtf_build_event_csr_device: neighbour without an in-edge (graph not symmetric)");
        return -1;
    }
    ev->n_edges = m;
    ev->n_subgraphs = n_sub;
    return 0;
#undef GTF_CK
}

}  // extern "C"
