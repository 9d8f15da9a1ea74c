// gtf_tags.hip -- tag propagation ("custom CCA") as CSR kernels for gfx950.
// Reference: tag_propagation/tag_propagation.py:97-164. The reference walks a
// dict-of-dicts adjacency and deep-copies the whole graph every sweep; here one
// sweep is one launch over the out-CSR, reading the previous tag array and
// writing the next (Jacobi), with the flip count reduced per wavefront before a
// single atomic per wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace {
constexpr int BLOCK = 256;

// keep[e] = neighbour radius <= node radius (:99-110); processed[u] = any kept (:109-110)
__global__ void __launch_bounds__(BLOCK) k_tag_prepare(gtf_graph g, const double* radius, uint8_t* keep,
                                                       uint8_t* processed, int32_t* n_processed) {
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    int mine = 0;
    if (u < g.n_nodes) {
        const double ru = radius[u];
        int any = 0;
        for (int i = g.out_ptr[u]; i < g.out_ptr[u + 1]; i++) {
            const int w = g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]];
            const uint8_t k = !(radius[w] > ru);
            keep[i] = k;
            any |= k;
        }
        processed[u] = (uint8_t)any;
        mine = any;
    }
    const unsigned long long b = __ballot(mine);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(n_processed, (int)__popcll(b));
}

// tags_out[u] = max(tags_in[u], tags_in[kept successors]) (:141-150 -- max, not min)
__global__ void __launch_bounds__(BLOCK) k_tag_sweep(gtf_graph g, const uint8_t* keep, const uint8_t* processed,
                                                     const int64_t* tin, int64_t* tout, int32_t* flips) {
    const int u = gtf::xcd_local(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    int flipped = 0;
    if (u < g.n_nodes) {
        const int64_t t0 = tin[u];
        int64_t t = t0;
        if (processed[u]) {
            for (int i = g.out_ptr[u]; i < g.out_ptr[u + 1]; i++)
                if (keep[i]) {
                    const int64_t tw = tin[g.out_dst ? g.out_dst[i] : g.slot_dst[g.out_slot[i]]];
                    t = tw > t ? tw : t;
                }
            flipped = (t != t0);
        }
        tout[u] = t;
    }
    const unsigned long long b = __ballot(flipped);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(flips, (int)__popcll(b));
}
}  // namespace

extern "C" {

int gtf_tag_prepare(const gtf_graph* g, const double* radius, uint8_t* keep, uint8_t* processed,
                    int32_t* n_processed, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_prepare")) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(n_processed, 0, sizeof(int32_t), st) != hipSuccess) return -1;
    if (g->n_nodes > 0)
        hipLaunchKernelGGL(k_tag_prepare, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, *g, radius,
                           keep, processed, n_processed);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int gtf_tag_sweep(const gtf_graph* g, const uint8_t* keep, const uint8_t* processed, const int64_t* tags_in,
                  int64_t* tags_out, int32_t* flips, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_tag_sweep")) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(flips, 0, sizeof(int32_t), st) != hipSuccess) return -1;
    if (g->n_nodes > 0)
        hipLaunchKernelGGL(k_tag_sweep, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, *g, keep,
                           processed, tags_in, tags_out, flips);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
