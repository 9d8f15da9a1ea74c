// gtf_build.cpp -- event conversion's graph build straight to the packed CSR.
//
// The reference builds a networkx DiGraph from the event CSVs (helper.construct_graph,
// helper.py:465-521; event_conversion.py:63-84), splits it into weakly connected
// components and copies each one as a subgraph. Every later stage depends on the
// ORDERS that come out of that: node order inside a subgraph, successor order, and
// the track_state_estimates key order reversed(set(nx.all_neighbors(G, n)))
// (helper.py:277, 350-351). Those orders are CPython set orders, so this file
// reproduces them exactly by running CPython 3.10's set insertion algorithm
// (Objects/setobject.c: linear probes of 9, then perturbed probing, resize at 3/5
// fill to 4x used) on the same key sequences networkx feeds it:
//
//   * components: nx.weakly_connected_components -> set(_plain_bfs(G, n, v)) in BFS
//     yield order (successors then predecessors of each level node);
//   * G.subgraph(c): show_nodes(nbunch_iter(c)).nodes = set(iter(c)), a second set;
//     the copy's node order is that set's order when 2|c| < |G| (FilterAtlas
//     iterates the shorter side), else G's node order restricted to c;
//   * copy(): successors keep G's insertion order; predecessors follow the copy's
//     node order;
//   * TSE keys: set(chain(pred(v), succ(v))) in the copy, reversed.
//
// Node ids hash to themselves (Python ints below 2^61 - 1). Plain host C++; the
// states themselves are computed on the GPU by gtf_track_state_estimates.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "../../include/gtf.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

// CPython 3.10 set of non-negative ints (no deletions, so no dummy entries)
class PySet {
  public:
    PySet() : keys_(8, -1), mask_(7), fill_(0) {}

    void add(int64_t key) {
        const size_t hash = (size_t)key;
        size_t i = hash & mask_;
        size_t perturb = hash;
        for (;;) {
            size_t probes = (i + kLinearProbes <= mask_) ? kLinearProbes : 0;
            size_t j = i;
            for (;;) {
                if (keys_[j] < 0) {
                    keys_[j] = key;
                    fill_++;
                    if (fill_ * 5 >= mask_ * 3) resize(fill_ > 50000 ? fill_ * 2 : fill_ * 4);
                    return;
                }
                if (keys_[j] == key) return;
                if (probes-- == 0) break;
                j++;
            }
            perturb >>= kPerturbShift;
            i = (i * 5 + 1 + perturb) & mask_;
        }
    }

    // iteration order = table order
    template <class F>
    void each(F f) const {
        for (int64_t k : keys_)
            if (k >= 0) f(k);
    }

    size_t size() const { return fill_; }

  private:
    static constexpr size_t kLinearProbes = 9;
    static constexpr size_t kPerturbShift = 5;

    void resize(size_t minused) {
        size_t newsize = 8;
        while (newsize <= minused) newsize <<= 1;
        std::vector<int64_t> old;
        old.swap(keys_);
        keys_.assign(newsize, -1);
        mask_ = newsize - 1;
        for (int64_t k : old)
            if (k >= 0) insert_clean(k);
    }

    void insert_clean(int64_t key) {
        const size_t hash = (size_t)key;
        size_t perturb = hash;
        size_t i = hash & mask_;
        for (;;) {
            if (keys_[i] < 0) { keys_[i] = key; return; }
            if (i + kLinearProbes <= mask_) {
                for (size_t j = 1; j <= kLinearProbes; j++)
                    if (keys_[i + j] < 0) { keys_[i + j] = key; return; }
            }
            perturb >>= kPerturbShift;
            i = (i * 5 + 1 + perturb) & mask_;
        }
    }

    std::vector<int64_t> keys_;
    size_t mask_;
    size_t fill_;
};

}  // namespace

extern "C" {

int gtf_build_event_csr(gtf_event_csr* ev) {
    if (!ev || ev->n_nodes < 0 || ev->n_rows < 0 || (ev->n_nodes && !ev->node_id) ||
        (ev->n_rows && (!ev->row_a || !ev->row_b)) || !ev->order || !ev->sub_id || !ev->slot_ptr || !ev->out_ptr ||
        (ev->n_rows && (!ev->slot_src || !ev->tse_rank || !ev->out_slot))) {
        gtf::set_error("gtf_build_event_csr: bad arguments");
        return -2;
    }
    const int64_t N = ev->n_nodes;
    if (N > INT32_MAX || 2 * ev->n_rows > INT32_MAX) {
        gtf::set_error("gtf_build_event_csr: graph too large for int32 indices");
        return -2;
    }
    std::unordered_map<int64_t, int32_t> idx;
    idx.reserve((size_t)N * 2);
    for (int64_t i = 0; i < N; i++) {
        if (ev->node_id[i] < 0 || ev->node_id[i] >= ((int64_t)1 << 61) - 1) {
            gtf::set_error("gtf_build_event_csr: node ids must be in [0, 2^61 - 1)");
            return -2;
        }
        if (!idx.emplace(ev->node_id[i], (int32_t)i).second) {
            gtf::set_error("gtf_build_event_csr: duplicate node id");
            return -2;
        }
    }
    // G: add_edge(a, b); add_edge(b, a) per row with both ends kept (helper.py:512-518)
    std::vector<std::vector<int32_t>> succ(N);
    auto add_edge = [&](int32_t u, int32_t v) {      // a repeated edge keeps its first position
        for (int32_t w : succ[u])
            if (w == v) return;
        succ[u].push_back(v);
    };
    for (int64_t r = 0; r < ev->n_rows; r++) {
        auto ia = idx.find(ev->row_a[r]), ib = idx.find(ev->row_b[r]);
        if (ia == idx.end() || ib == idx.end()) continue;
        add_edge(ia->second, ib->second);
        add_edge(ib->second, ia->second);
    }
    std::vector<std::vector<int32_t>> pred(N);      // G's predecessors (BFS only needs the set)
    for (int32_t u = 0; u < N; u++)
        for (int32_t v : succ[u]) pred[v].push_back(u);

    // weakly connected components in networkx's order, each copied in set order
    std::vector<uint8_t> seen(N, 0);
    std::vector<int32_t> comp_of(N, -1);
    std::vector<int32_t> pos(N, -1);                 // packed index
    int32_t n_sub = 0, next = 0;
    std::vector<int32_t> level, nextlevel, members;
    for (int32_t s = 0; s < N; s++) {
        if (seen[s]) continue;
        PySet c;
        members.clear();
        seen[s] = 1;
        c.add(ev->node_id[s]);
        members.push_back(s);
        level.assign(1, s);
        while (!level.empty()) {
            nextlevel.clear();
            for (int32_t v : level) {
                for (int32_t w : succ[v])
                    if (!seen[w]) { seen[w] = 1; c.add(ev->node_id[w]); members.push_back(w); nextlevel.push_back(w); }
                for (int32_t w : pred[v])
                    if (!seen[w]) { seen[w] = 1; c.add(ev->node_id[w]); members.push_back(w); nextlevel.push_back(w); }
            }
            level.swap(nextlevel);
        }
        for (int32_t m : members) comp_of[m] = n_sub;
        if (2 * (int64_t)members.size() < N) {
            PySet shown;
            c.each([&](int64_t k) { shown.add(k); });
            shown.each([&](int64_t k) { ev->order[next] = idx[k]; pos[idx[k]] = next; next++; });
        } else {
            std::vector<int32_t> in_order(members);
            std::sort(in_order.begin(), in_order.end());
            for (int32_t m : in_order) { ev->order[next] = m; pos[m] = next; next++; }
        }
        n_sub++;
    }
    // the copy: predecessors in copy node order (== packed order), successors as in G
    std::vector<int32_t> indeg(N, 0);
    for (int32_t u = 0; u < N; u++)
        for (int32_t v : succ[u]) indeg[pos[v]]++;
    int32_t* sp = ev->slot_ptr;
    sp[0] = 0;
    for (int64_t p = 0; p < N; p++) sp[p + 1] = sp[p] + indeg[p];
    std::vector<int32_t> fillp(sp, sp + N);
    for (int64_t p = 0; p < N; p++) {
        const int32_t u = ev->order[p];
        ev->sub_id[p] = comp_of[u];
        for (int32_t v : succ[u]) ev->slot_src[fillp[pos[v]]++] = (int32_t)p;
    }
    // out view (successor order) and the TSE key order
    int32_t* op = ev->out_ptr;
    op[0] = 0;
    for (int64_t p = 0; p < N; p++) {
        const int32_t u = ev->order[p];
        int32_t o = op[p];
        for (int32_t v : succ[u]) {
            const int32_t q = pos[v];
            const int32_t* b = ev->slot_src + sp[q];
            const int32_t* e = ev->slot_src + sp[q + 1];
            ev->out_slot[o++] = (int32_t)(std::lower_bound(b, e, (int32_t)p) - ev->slot_src);
        }
        op[p + 1] = o;
        PySet nb;
        for (int32_t k = sp[p]; k < sp[p + 1]; k++) nb.add(ev->node_id[ev->order[ev->slot_src[k]]]);
        for (int32_t v : succ[u]) nb.add(ev->node_id[v]);
        std::vector<int64_t> keys;
        keys.reserve(nb.size());
        nb.each([&](int64_t k) { keys.push_back(k); });
        const int32_t nk = (int32_t)keys.size();
        for (int32_t k = sp[p]; k < sp[p + 1]; k++) ev->tse_rank[k] = -1;
        for (int32_t r = 0; r < nk; r++) {
            const int32_t q = pos[idx[keys[nk - 1 - r]]];
            const int32_t* b = ev->slot_src + sp[p];
            const int32_t* e = ev->slot_src + sp[p + 1];
            const int32_t* f = std::lower_bound(b, e, q);
            if (f == e || *f != q) {
                gtf::set_error("gtf_build_event_csr: neighbour without an in-edge (graph not symmetric)");
                return -1;
            }
            ev->tse_rank[f - ev->slot_src] = r;
        }
    }
    ev->n_edges = sp[N];
    ev->n_subgraphs = n_sub;
    return 0;
}

int gtf_candidate_order(const gtf_candidate_graph* cg, int32_t* order_key) {
    if (!cg || cg->n_nodes < 0 || !order_key ||
        (cg->n_nodes && (!cg->slot_ptr || !cg->out_ptr || !cg->sub_id || !cg->node_id)) ||
        (cg->n_slots && (!cg->slot_src || !cg->is_edge || !cg->act)) || (cg->n_edges && !cg->out_slot)) {
        gtf::set_error("gtf_candidate_order: bad arguments");
        return -2;
    }
    const int32_t N = cg->n_nodes;
    std::vector<int32_t> dst(cg->n_slots);
    for (int32_t v = 0; v < N; v++)
        for (int32_t k = cg->slot_ptr[v]; k < cg->slot_ptr[v + 1]; k++) dst[k] = v;
    std::vector<uint8_t> seen(N, 0);
    std::vector<int32_t> level, nextlevel, members;
    int32_t lo = 0;
    while (lo < N) {
        int32_t hi = lo + 1;
        while (hi < N && cg->sub_id[hi] == cg->sub_id[lo]) hi++;
        if (cg->sub_id[hi - 1] != cg->sub_id[lo]) { gtf::set_error("gtf_candidate_order: sub_id not grouped"); return -2; }
        bool inactive = false;
        for (int32_t k = cg->slot_ptr[lo]; k < cg->slot_ptr[hi] && !inactive; k++)
            inactive = cg->is_edge[k] && cg->act[k] == 0;
        if (!inactive) {                     // CCA keeps the whole subgraph (:344-345)
            for (int32_t v = lo; v < hi; v++) order_key[v] = v - lo;
            lo = hi;
            continue;
        }
        for (int32_t s = lo; s < hi; s++) {
            if (seen[s]) continue;
            PySet c;
            members.clear();
            auto visit = [&](int32_t w) {
                if (seen[w]) return;
                seen[w] = 1;
                c.add(cg->node_id[w]);
                members.push_back(w);
                nextlevel.push_back(w);
            };
            seen[s] = 1;
            c.add(cg->node_id[s]);
            members.push_back(s);
            level.assign(1, s);
            while (!level.empty()) {
                nextlevel.clear();
                for (int32_t v : level) {
                    for (int32_t j = cg->out_ptr[v]; j < cg->out_ptr[v + 1]; j++) {
                        const int32_t k = cg->out_slot[j];
                        if (cg->act[k] != 0) visit(dst[k]);          // successors, G order
                    }
                    for (int32_t k = cg->slot_ptr[v]; k < cg->slot_ptr[v + 1]; k++)
                        if (cg->is_edge[k] && cg->act[k] != 0) visit(cg->slot_src[k]);   // predecessors
                }
                level.swap(nextlevel);
            }
            if (2 * (int64_t)members.size() < (int64_t)(hi - lo)) {
                std::unordered_map<int64_t, int32_t> at;
                for (int32_t m : members) at.emplace(cg->node_id[m], m);
                PySet shown;
                c.each([&](int64_t k) { shown.add(k); });
                int32_t r = 0;
                shown.each([&](int64_t k) { order_key[at[k]] = r++; });
            } else {
                std::sort(members.begin(), members.end());
                for (size_t r = 0; r < members.size(); r++) order_key[members[r]] = (int32_t)r;
            }
        }
        lo = hi;
    }
    return 0;
}

}  // extern "C"
