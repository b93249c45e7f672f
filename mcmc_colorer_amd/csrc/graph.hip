// mcmc_colorer_amd/csrc/graph.hip -- device-resident CSR graphs for the sweep.
//
//  mcmc_graph_upload    Graph(Graph* host) device copy (graph/graphGPU.cu:210-226), uint64 offsets.
//  mcmc_graph_simulate  Graph(n, prob, seed) -> setupRnd2 (graph/graphCPU.cpp:291-404), bit-exact,
//                       generated on the GPU: the n(n+1)/2 glibc rand() draws of the upper
//                       triangle (row-major, diagonal included, :307-308) are split into chunks;
//                       each thread jumps the glibc window to its chunk with a precomputed
//                       31x31 jump matrix per power of two (the recurrence is linear over Z/2^32)
//                       and replays its chunk. Pass 1 counts degrees, an exclusive scan gives the
//                       offsets, pass 2 regenerates and scatters both arc directions (:507-529),
//                       and a segmented sort restores the reference's ascending neighbour order.
//  mcmc_graph_er_fast   G(n,p) stand-in for sizes the O(n^2) generator cannot reach.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "mcmc_common.h"
#include "rng.h"

namespace mcmc {
namespace {

constexpr uint32_t kChunkSteps = 31 * 256;   // draws per thread chunk (multiple of 31)

// Jump matrices: J_b = window map for 2^b chunks. Row j of J holds x^(k+j) mod P.
struct JumpTable {
    uint32_t nbits;
    uint32_t* d = nullptr;   // [nbits][31][31]
};

__device__ __forceinline__ void apply_jump(uint32_t (&w)[31], const uint32_t* __restrict__ J) {
    uint32_t o[31];
#pragma unroll
    for (int j = 0; j < 31; j++) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 31; i++) acc += J[j * 31 + i] * w[i];
        o[j] = acc;
    }
#pragma unroll
    for (int j = 0; j < 31; j++) w[j] = o[j];
}

// Upper-triangle coordinates of draw k: row j, column i (i >= j); start(j) = j*n - j(j-1)/2.
__device__ __forceinline__ void tri_coords(uint64_t k, uint64_t n, uint64_t& j, uint64_t& i) {
    const double b = 2.0 * (double)n + 1.0;
    double disc = b * b - 8.0 * (double)k;
    if (disc < 0) disc = 0;
    int64_t jj = (int64_t)((b - sqrt(disc)) * 0.5);
    if (jj < 0) jj = 0;
    if ((uint64_t)jj >= n) jj = (int64_t)n - 1;
    auto start = [n](uint64_t r) { return r * n - (r * (r - 1)) / 2; };
    while (jj > 0 && start((uint64_t)jj) > k) jj--;
    while ((uint64_t)jj + 1 < n && start((uint64_t)jj + 1) <= k) jj++;
    j = (uint64_t)jj;
    i = j + (k - start(j));
}

// One pass over the triangle. MODE 0: degree count. MODE 1: arc scatter with cursors.
template <int MODE>
__global__ __launch_bounds__(256) void er_exact_kernel(uint32_t n, uint64_t total, uint32_t thr,
                                                        const uint32_t* __restrict__ w0,
                                                        const uint32_t* __restrict__ jumps, uint32_t nbits,
                                                        uint32_t* __restrict__ deg,
                                                        const uint64_t* __restrict__ row_off,
                                                        uint32_t* __restrict__ cursor,
                                                        uint32_t* __restrict__ col_idx) {
    const uint64_t chunk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k0 = chunk * kChunkSteps;
    if (k0 >= total) return;
    uint32_t w[31];
#pragma unroll
    for (int i = 0; i < 31; i++) w[i] = w0[i];
    for (uint32_t b = 0; b < nbits; b++)
        if ((chunk >> b) & 1ull) apply_jump(w, jumps + (size_t)b * 961);
    uint64_t j, i;
    tri_coords(k0, n, j, i);
    const uint64_t kend = min(total, k0 + kChunkSteps);
    uint64_t k = k0;
    uint32_t rowcnt = 0;   // MODE 0: arcs of row j found in this chunk (flushed on row change)
    while (k < kend) {
#pragma unroll
        for (int s = 0; s < 31; s++) {
            const uint32_t v = w[s] + w[(s + 28) % 31];
            w[s] = v;
            if (k < kend) {
                const bool edge = ((v >> 1) < thr) && (i != j);
                if (edge) {
                    if (MODE == 0) {
                        rowcnt++;
                        atomicAdd(&deg[i], 1u);
                    } else {
                        const uint32_t pj = atomicAdd(&cursor[j], 1u);
                        col_idx[row_off[j] + pj] = (uint32_t)i;
                        const uint32_t pi = atomicAdd(&cursor[i], 1u);
                        col_idx[row_off[i] + pi] = (uint32_t)j;
                    }
                }
                i++;
                if (i == n) {
                    if (MODE == 0 && rowcnt) { atomicAdd(&deg[j], rowcnt); rowcnt = 0; }
                    j++;
                    i = j;
                }
                k++;
            }
        }
    }
    if (MODE == 0 && rowcnt) atomicAdd(&deg[j], rowcnt);
}

__global__ void deg_to_u64(const uint32_t* __restrict__ deg, uint64_t* __restrict__ d64, uint32_t n) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) d64[v] = deg[v];
}

// Smallest r in [0, 2^31] with (double)r / RAND_MAX >= (double)prob: the edge test of setupRnd2
// (graphCPU.cpp:308) is then exactly r < thr.
uint32_t edge_threshold(float prob) {
    const double p = (double)prob;
    uint64_t lo = 0, hi = 2147483648ull;   // answer in [lo, hi]
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (((double)mid / 2147483647.0) >= p) hi = mid; else lo = mid + 1;
    }
    return (uint32_t)std::min<uint64_t>(lo, 0xFFFFFFFFull);
}

int stats_from_offsets(GraphDev& g) {
    std::vector<uint64_t> off(g.n + 1);
    MCMC_HIP_TRY(hipMemcpy(off.data(), g.row_off, sizeof(uint64_t) * (g.n + 1), hipMemcpyDeviceToHost));
    g.maxDeg = 0;
    g.minDeg = g.n;
    for (uint32_t v = 0; v < g.n; v++) {
        const uint32_t d = (uint32_t)(off[v + 1] - off[v]);
        g.maxDeg = std::max(g.maxDeg, d);
        g.minDeg = std::min(g.minDeg, d);
    }
    g.m = off[g.n];
    return MCMC_OK;
}

}  // namespace

int sort_rows_inplace(GraphDev& g) {
    if (g.sorted || g.m == 0) { g.sorted = true; return MCMC_OK; }
    if (g.m >= (1ull << 31)) return fail(MCMC_E_ARG, "sort_rows_inplace: more than 2^31 arcs");
    MCMC_HIP_TRY(hipSetDevice(g.device));
    uint32_t* sorted = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    MCMC_HIP_TRY(hipMalloc(&sorted, sizeof(uint32_t) * (g.m + 4)));
    MCMC_HIP_TRY(hipMemset(sorted, 0, sizeof(uint32_t) * (g.m + 4)));
    MCMC_HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tmp_bytes, g.col_idx, sorted, (int)g.m, (int)g.n,
                                                            g.row_off, g.row_off + 1));
    MCMC_HIP_TRY(hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 1)));
    MCMC_HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tmp_bytes, g.col_idx, sorted, (int)g.m, (int)g.n,
                                                            g.row_off, g.row_off + 1));
    MCMC_HIP_TRY(hipDeviceSynchronize());
    (void)hipFree(tmp);
    (void)hipFree(g.col_idx);
    g.col_idx = sorted;
    g.sorted = true;
    return MCMC_OK;
}

// bad |= 1 unless every arc (i, j) of rows [vb, vb + nloc) with j in the range has its reverse
// (rows ascending). One wave per row: hub rows are tens of thousands of arcs.
__global__ __launch_bounds__(256) void csr_symcheck_kernel(const uint64_t* __restrict__ row_off,
                                                           const uint32_t* __restrict__ col, uint32_t vb,
                                                           uint32_t nloc, uint32_t* bad) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t l = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; l < nloc; l += nw) {
        const uint32_t i = vb + l;
        const uint64_t e = row_off[i + 1];
        bool ok = true;
        for (uint64_t k = row_off[i] + lane; k < e; k += 64) {
            const uint32_t j = col[k];
            if (j - vb >= nloc) continue;
            uint64_t lo = row_off[j], hi = row_off[j + 1];
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (col[mid] < i) lo = mid + 1; else hi = mid;
            }
            if (lo == row_off[j + 1] || col[lo] != i) ok = false;
        }
        if (__ballot(!ok) && lane == 0) atomicOr(bad, 1u);
    }
}

int csr_symmetric(GraphDev& g, uint32_t vb, uint32_t nloc, hipStream_t s, bool* sym) {
    const bool whole = vb == 0 && nloc == g.n;
    if (whole && g.sym >= 0) { *sym = g.sym == 1; return MCMC_OK; }
    if (!g.row_off) return fail(MCMC_E_STATE, "symmetry check needs a CSR");
    if (!g.sorted) {
        if (int rc = sort_rows_inplace(g)) return rc;
    }
    uint32_t* bad = nullptr;
    MCMC_HIP_TRY(hipMalloc(&bad, sizeof(uint32_t)));
    uint32_t h = 0;
    hipError_t e = hipMemsetAsync(bad, 0, sizeof(uint32_t), s);
    if (e == hipSuccess && nloc) {
        csr_symcheck_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((nloc + 3u) / 4u, 65535u)), 256, 0, s>>>(
            g.row_off, g.col_idx, vb, nloc, bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&h, bad, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(bad);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("symmetry check: ") + hipGetErrorString(e));
    *sym = h == 0;
    if (whole) g.sym = *sym ? 1 : 0;
    return MCMC_OK;
}

}  // namespace mcmc

using namespace mcmc;

extern "C" {

int mcmc_graph_upload(const uint64_t* row_off, const uint32_t* col_idx, uint32_t n, uint64_t m, int device,
                      mcmc_graph** out) {
    if (!row_off || (m && !col_idx) || !out) return fail(MCMC_E_ARG, "NULL argument");
    if (row_off[0] != 0 || row_off[n] != m) return fail(MCMC_E_ARG, "row_off must start at 0 and end at m");
    *out = nullptr;
    MCMC_HIP_TRY(hipSetDevice(device));
    mcmc_graph* g = new mcmc_graph();
    g->g.device = device;
    g->g.n = n;
    g->g.m = m;
    hipError_t e = hipMalloc(&g->g.row_off, sizeof(uint64_t) * ((size_t)n + 1));
    if (e == hipSuccess) e = hipMalloc(&g->g.col_idx, sizeof(uint32_t) * (m + 4));
    if (e == hipSuccess) e = hipMemcpy(g->g.row_off, row_off, sizeof(uint64_t) * ((size_t)n + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(g->g.col_idx, 0, sizeof(uint32_t) * (m + 4));   // zero pad: valid ids
    if (e == hipSuccess && m) e = hipMemcpy(g->g.col_idx, col_idx, sizeof(uint32_t) * m, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        mcmc_graph_destroy(g);
        return fail(MCMC_E_HIP, std::string("graph upload: ") + hipGetErrorString(e));
    }
    g->g.maxDeg = 0;
    g->g.minDeg = n;
    bool sorted = true;
    for (uint32_t v = 0; v < n; v++) {
        const uint32_t d = (uint32_t)(row_off[v + 1] - row_off[v]);
        g->g.maxDeg = std::max(g->g.maxDeg, d);
        g->g.minDeg = std::min(g->g.minDeg, d);
        for (uint64_t k = row_off[v] + 1; sorted && k < row_off[v + 1]; k++) sorted = col_idx[k - 1] <= col_idx[k];
    }
    g->g.sorted = sorted;
    *out = g;
    return MCMC_OK;
}

int mcmc_graph_simulate(uint32_t n, float prob, uint32_t window[31], int device, mcmc_graph** out) {
    if (!window || !out || n == 0) return fail(MCMC_E_ARG, "bad argument");
    *out = nullptr;
    MCMC_HIP_TRY(hipSetDevice(device));
    const uint64_t total = (uint64_t)n * ((uint64_t)n + 1) / 2;
    const uint64_t chunks = (total + kChunkSteps - 1) / kChunkSteps;
    uint32_t nbits = 0;
    while ((1ull << nbits) < chunks) nbits++;
    // host: jump matrices for 2^b chunks
    std::vector<uint32_t> J((size_t)std::max<uint32_t>(nbits, 1) * 961);
    {
        GlibcPoly q = glibc_poly_xpow(kChunkSteps);
        for (uint32_t b = 0; b < nbits; b++) {
            GlibcPoly r = q;
            for (int j = 0; j < 31; j++) {
                for (int i = 0; i < 31; i++) J[(size_t)b * 961 + j * 31 + i] = r.c[i];
                r = glibc_poly_mulx(r);
            }
            q = glibc_poly_mul(q, q);
        }
    }
    const uint32_t thr = edge_threshold(prob);
    mcmc_graph* g = new mcmc_graph();
    g->g.device = device;
    g->g.n = n;
    uint32_t *d_w0 = nullptr, *d_J = nullptr, *d_deg = nullptr, *d_cur = nullptr;
    uint64_t* d_deg64 = nullptr;
    void* d_tmp = nullptr;
    uint32_t* d_sorted = nullptr;
    int rc = MCMC_OK;
    auto cleanup = [&]() {
        (void)hipFree(d_w0); (void)hipFree(d_J); (void)hipFree(d_deg); (void)hipFree(d_cur);
        (void)hipFree(d_deg64); (void)hipFree(d_tmp); (void)hipFree(d_sorted);
    };
#define GTRY(expr)                                                                            \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            cleanup();                                                                        \
            mcmc_graph_destroy(g);                                                            \
            return fail(MCMC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
        }                                                                                     \
    } while (0)
    GTRY(hipMalloc(&d_w0, 31 * sizeof(uint32_t)));
    GTRY(hipMalloc(&d_J, J.size() * sizeof(uint32_t)));
    GTRY(hipMalloc(&d_deg, sizeof(uint32_t) * n));
    GTRY(hipMalloc(&d_cur, sizeof(uint32_t) * n));
    GTRY(hipMalloc(&d_deg64, sizeof(uint64_t) * n));
    GTRY(hipMalloc(&g->g.row_off, sizeof(uint64_t) * ((size_t)n + 1)));
    GTRY(hipMemcpy(d_w0, window, 31 * sizeof(uint32_t), hipMemcpyHostToDevice));
    GTRY(hipMemcpy(d_J, J.data(), J.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    GTRY(hipMemset(d_deg, 0, sizeof(uint32_t) * n));
    GTRY(hipMemset(d_cur, 0, sizeof(uint32_t) * n));
    const uint32_t threads = 256;
    const uint32_t blocks = (uint32_t)((chunks + threads - 1) / threads);
    er_exact_kernel<0><<<blocks, threads>>>(n, total, thr, d_w0, d_J, nbits, d_deg, nullptr, nullptr, nullptr);
    GTRY(hipGetLastError());
    deg_to_u64<<<std::min<uint32_t>((n + 255) / 256, 4096u), 256>>>(d_deg, d_deg64, n);
    GTRY(hipGetLastError());
    size_t tmp_bytes = 0;
    GTRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, d_deg64, g->g.row_off + 1, (int)n));
    GTRY(hipMalloc(&d_tmp, std::max<size_t>(tmp_bytes, 1)));
    GTRY(hipcub::DeviceScan::InclusiveSum(d_tmp, tmp_bytes, d_deg64, g->g.row_off + 1, (int)n));
    GTRY(hipMemset(g->g.row_off, 0, sizeof(uint64_t)));
    uint64_t m = 0;
    GTRY(hipMemcpy(&m, g->g.row_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost));
    g->g.m = m;
    if (m >= (1ull << 31)) {
        cleanup();
        mcmc_graph_destroy(g);
        return fail(MCMC_E_ARG, "mcmc_graph_simulate: more than 2^31 arcs (use a smaller n)");
    }
    GTRY(hipMalloc(&g->g.col_idx, sizeof(uint32_t) * (m + 4)));
    GTRY(hipMemset(g->g.col_idx, 0, sizeof(uint32_t) * (m + 4)));
    er_exact_kernel<1><<<blocks, threads>>>(n, total, thr, d_w0, d_J, nbits, nullptr, g->g.row_off, d_cur, g->g.col_idx);
    GTRY(hipGetLastError());
    if (m) {
        GTRY(hipMalloc(&d_sorted, sizeof(uint32_t) * (m + 4)));
        GTRY(hipMemset(d_sorted, 0, sizeof(uint32_t) * (m + 4)));   // zero pad survives the swap
        (void)hipFree(d_tmp);
        d_tmp = nullptr;
        tmp_bytes = 0;
        GTRY(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tmp_bytes, g->g.col_idx, d_sorted, (int)m, (int)n,
                                                        g->g.row_off, g->g.row_off + 1));
        GTRY(hipMalloc(&d_tmp, std::max<size_t>(tmp_bytes, 1)));
        GTRY(hipcub::DeviceSegmentedRadixSort::SortKeys(d_tmp, tmp_bytes, g->g.col_idx, d_sorted, (int)m, (int)n,
                                                        g->g.row_off, g->g.row_off + 1));
        std::swap(g->g.col_idx, d_sorted);
    }
    GTRY(hipDeviceSynchronize());
#undef GTRY
    cleanup();
    rc = stats_from_offsets(g->g);
    if (rc) { mcmc_graph_destroy(g); return rc; }
    g->g.sorted = true;
    // advance the caller's glibc stream past the generator's draws, as the reference's is
    GlibcWindow w;
    std::memcpy(w.r, window, sizeof(w.r));
    w = glibc_jump(w, total);
    std::memcpy(window, w.r, sizeof(w.r));
    *out = g;
    return MCMC_OK;
}

int mcmc_graph_info(const mcmc_graph* g, uint32_t* n, uint64_t* m, uint32_t* maxDeg, uint32_t* minDeg) {
    if (!g) return fail(MCMC_E_ARG, "NULL graph");
    if (n) *n = g->g.n;
    if (m) *m = g->g.m;
    if (maxDeg) *maxDeg = g->g.maxDeg;
    if (minDeg) *minDeg = g->g.minDeg;
    return MCMC_OK;
}

int mcmc_graph_device_ptrs(const mcmc_graph* g, const uint64_t** row_off, const uint32_t** col_idx) {
    if (!g) return fail(MCMC_E_ARG, "NULL graph");
    if (!g->g.row_off) return fail(MCMC_E_STATE, "generated graph: no device CSR (tiled layout only)");
    if (row_off) *row_off = g->g.row_off;
    if (col_idx) *col_idx = g->g.col_idx;
    return MCMC_OK;
}

int mcmc_graph_download(const mcmc_graph* g, uint64_t* row_off, uint32_t* col_idx) {
    if (!g) return fail(MCMC_E_ARG, "NULL graph");
    MCMC_HIP_TRY(hipSetDevice(g->g.device));
    if (!g->g.row_off) {   // generated graph: rebuild the CSR from its tiled layout
        if (!row_off || !col_idx) return fail(MCMC_E_ARG, "generated graph: download needs both arrays");
        return tiled_to_csr(g, row_off, col_idx);
    }
    if (row_off)
        MCMC_HIP_TRY(hipMemcpy(row_off, g->g.row_off, sizeof(uint64_t) * ((size_t)g->g.n + 1), hipMemcpyDeviceToHost));
    if (col_idx && g->g.m)
        MCMC_HIP_TRY(hipMemcpy(col_idx, g->g.col_idx, sizeof(uint32_t) * g->g.m, hipMemcpyDeviceToHost));
    return MCMC_OK;
}

void mcmc_graph_destroy(mcmc_graph* g) {
    if (!g) return;
    (void)hipSetDevice(g->g.device);
    g->tiles.clear();
    (void)hipFree(g->g.row_off);
    (void)hipFree(g->g.col_idx);
    delete g;
}


}  // extern "C"
