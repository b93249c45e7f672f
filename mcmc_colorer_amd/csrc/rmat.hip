// mcmc_colorer_amd/csrc/rmat.hip -- the R-MAT power-law stand-in for configs[4] (SURVEY.md §8d C5:
// SNAP LiveJournal / Reddit are not in the container), generated on the device as a CSR graph.
// Definition in er_gen.h (rmat_edge); pinned by the numpy restatement oracle/oracle_np.py::rmat.
//
// Pipeline: one thread per edge draw writes both arcs as 64-bit keys (row << 32 | col; a
// self-loop writes two sentinels) -> radix sort -> unique -> row offsets from the first key of
// every row -> col_idx = the keys' low words. Neighbour lists come out ascending, like
// --simulate's (graphCPU.cpp:290-404).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "er_gen.h"
#include "mcmc_common.h"

namespace mcmc {
namespace {

constexpr uint64_t kSentinel = ~0ull;

__global__ void rmat_keys_kernel(uint64_t E, er::RmatConst k, uint64_t* __restrict__ keys) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t i, j;
        er::rmat_edge(e, k, i, j);
        const bool loop = i == j;
        keys[2 * e] = loop ? kSentinel : ((uint64_t)i << 32) | j;
        keys[2 * e + 1] = loop ? kSentinel : ((uint64_t)j << 32) | i;
    }
}

// row_off[r] = first key index whose row is >= r; col_idx[k] = low word of key k.
__global__ void rmat_csr_kernel(const uint64_t* __restrict__ keys, uint64_t m, uint32_t n,
                                uint64_t* __restrict__ row_off, uint32_t* __restrict__ col_idx) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= m; k += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t rp = k == 0 ? -1 : (int64_t)(keys[k - 1] >> 32);
        const int64_t rc = k == m ? (int64_t)n : (int64_t)(keys[k] >> 32);
        for (int64_t r = rp + 1; r <= rc; r++) row_off[r] = k;
        if (k < m) col_idx[k] = (uint32_t)keys[k];
    }
}

uint32_t threshold(double x) { return (uint32_t)std::min(4294967295.0, std::floor(std::max(0.0, x) * 4294967296.0)); }

}  // namespace
}  // namespace mcmc

using namespace mcmc;

extern "C" int mcmc_graph_rmat(uint32_t scale, uint32_t edge_factor, double a, double b, double c, uint64_t seed,
                               int device, mcmc_graph** out) {
    if (!out) return fail(MCMC_E_ARG, "NULL argument");
    *out = nullptr;
    if (scale > 30) return fail(MCMC_E_ARG, "R-MAT: scale <= 30");
    if (!(a >= 0 && b >= 0 && c >= 0 && a + b + c <= 1.0)) return fail(MCMC_E_ARG, "R-MAT: a, b, c >= 0, a+b+c <= 1");
    const uint32_t n = 1u << scale;
    const uint64_t E = (uint64_t)edge_factor * n;
    if (2 * E >= (1ull << 31)) return fail(MCMC_E_ARG, "R-MAT: 2 * edge_factor * 2^scale must stay below 2^31");
    MCMC_HIP_TRY(hipSetDevice(device));
    er::RmatConst k{scale, n - 1u, threshold(a), threshold(a + b), threshold(a + b + c), (uint32_t)seed,
                    (uint32_t)(seed >> 32)};
    mcmc_graph* g = new mcmc_graph();
    g->g.device = device;
    g->g.n = n;
    uint64_t *keys = nullptr, *keys2 = nullptr;
    int* d_num = nullptr;
    void* tmp = nullptr;
    auto cleanup = [&]() { (void)hipFree(keys); (void)hipFree(keys2); (void)hipFree(d_num); (void)hipFree(tmp); };
#define RTRY(expr)                                                                            \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            cleanup();                                                                        \
            mcmc_graph_destroy(g);                                                            \
            return fail(MCMC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
        }                                                                                     \
    } while (0)
    const int N = (int)(2 * E);
    RTRY(hipMalloc(&keys, sizeof(uint64_t) * std::max<uint64_t>(2 * E, 1)));
    RTRY(hipMalloc(&keys2, sizeof(uint64_t) * std::max<uint64_t>(2 * E, 1)));
    RTRY(hipMalloc(&d_num, sizeof(int)));
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((E + 255) / 256, 65536));
    if (E) rmat_keys_kernel<<<blocks, 256>>>(E, k, keys);
    RTRY(hipGetLastError());
    int m_keys = 0;
    if (N) {
        size_t tb_sort = 0, tb_uniq = 0;
        RTRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tb_sort, keys, keys2, N));
        RTRY(hipcub::DeviceSelect::Unique(nullptr, tb_uniq, keys2, keys, d_num, N));
        RTRY(hipMalloc(&tmp, std::max<size_t>(std::max(tb_sort, tb_uniq), 1)));
        RTRY(hipcub::DeviceRadixSort::SortKeys(tmp, tb_sort, keys, keys2, N));
        RTRY(hipcub::DeviceSelect::Unique(tmp, tb_uniq, keys2, keys, d_num, N));
        RTRY(hipMemcpy(&m_keys, d_num, sizeof(int), hipMemcpyDeviceToHost));
        uint64_t last = 0;
        if (m_keys > 0) {
            RTRY(hipMemcpy(&last, keys + (m_keys - 1), sizeof(uint64_t), hipMemcpyDeviceToHost));
            if (last == kSentinel) m_keys--;
        }
    }
    const uint64_t m = (uint64_t)m_keys;
    g->g.m = m;
    RTRY(hipMalloc(&g->g.row_off, sizeof(uint64_t) * ((size_t)n + 1)));
    RTRY(hipMalloc(&g->g.col_idx, sizeof(uint32_t) * (m + 4)));
    RTRY(hipMemset(g->g.col_idx, 0, sizeof(uint32_t) * (m + 4)));   // zero pad: valid ids
    rmat_csr_kernel<<<(uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((m + 256) / 256, 65536)), 256>>>(
        keys, m, n, g->g.row_off, g->g.col_idx);
    RTRY(hipGetLastError());
    std::vector<uint64_t> off((size_t)n + 1);
    RTRY(hipMemcpy(off.data(), g->g.row_off, sizeof(uint64_t) * ((size_t)n + 1), hipMemcpyDeviceToHost));
#undef RTRY
    cleanup();
    g->g.maxDeg = 0;
    g->g.minDeg = n;
    for (uint32_t v = 0; v < n; v++) {
        const uint32_t d = (uint32_t)(off[v + 1] - off[v]);
        g->g.maxDeg = std::max(g->g.maxDeg, d);
        g->g.minDeg = std::min(g->g.minDeg, d);
    }
    g->g.sorted = true;
    *out = g;
    return MCMC_OK;
}
