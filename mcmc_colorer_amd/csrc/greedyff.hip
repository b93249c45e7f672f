// mcmc_colorer_amd/csrc/greedyff.hip -- the reference's parallel greedy first-fit colorer
// (ColoringGreedyFF, graph_coloring/coloringGreedyFF.cu:50-84) on the CSR.
//
// Semantics kept exactly (deterministic; pinned by oracle/oracle_np.py::greedy_ff):
//   round: tentative_coloring (:88-129) -- every uncoloured node adds the colours of its neighbours
//          (the round's input colouring, 0 included) to its forbidden set, which is never cleared
//          (the reference flags a uint32 row with the node's id and never resets it), and takes the
//          first colour i >= 1, i < maxDeg + 1, not forbidden; node 0 always takes colour 1
//          (:99-101); then conflict_detection (:134-163) -- a coloured node with a same-coloured
//          neighbour of smaller id is uncoloured; until no node is uncoloured (:179-190).
// The reference runs thread-per-node kernels over n x maxColors uint32 marks; here one wave per
// node keeps its forbidden set as a bitmask (maxColors bits), staged in LDS while it is extended and
// searched (ds_or + a 64-word ballot per step), and the two phases ping-pong between two colour
// buffers (the reference copies temp -> coloring after each phase).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "mcmc_common.h"

namespace mcmc {
namespace {

constexpr int kGffThreads = 256;   // 4 waves, one node each at a time

__global__ __launch_bounds__(kGffThreads) void gff_tentative_kernel(const uint64_t* __restrict__ ro,
                                                                    const uint32_t* __restrict__ col, uint32_t n,
                                                                    uint32_t W, uint32_t maxColors,
                                                                    const uint32_t* __restrict__ cin,
                                                                    uint32_t* __restrict__ cout,
                                                                    uint32_t* __restrict__ forb) {
    extern __shared__ uint32_t lm[];   // [4 waves][W] forbidden bitmask of the wave's node
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t* m = lm + (size_t)wv * W;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        const uint32_t c0 = cin[v];
        if (v == 0 || c0 != 0) {   // node 0 always takes colour 1; coloured nodes keep theirs
            if (lane == 0) cout[v] = v == 0 ? 1u : c0;
            continue;
        }
        uint32_t* fv = forb + (size_t)v * W;
        for (uint32_t w = lane; w < W; w += 64) m[w] = fv[w];
        for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) {
            const uint32_t c = cin[col[k]];   // < maxColors: first-fit never picks past it
            atomicOr(&m[c >> 5], 1u << (c & 31u));
        }
        uint32_t pick = 0;   // 0: no free colour (the node stays uncoloured this round)
        for (uint32_t wb = 0; wb < W; wb += 64) {
            const uint32_t w = wb + lane;
            uint32_t z = 0;
            if (w < W) {
                z = ~m[w];
                if (w == 0) z &= ~1u;                                    // colour 0 is "uncoloured"
                const uint32_t top = maxColors - 32u * w;                // colours of this word below maxColors
                if (top < 32u) z &= (1u << top) - 1u;
            }
            const unsigned long long b = __ballot(z != 0u);
            if (b) {
                const int f = __ffsll(b) - 1;
                const uint32_t zf = (uint32_t)__shfl((int)z, f, 64);
                pick = 32u * (wb + (uint32_t)f) + (uint32_t)__builtin_ctz(zf);
                break;
            }
        }
        for (uint32_t w = lane; w < W; w += 64) fv[w] = m[w];
        if (lane == 0) cout[v] = pick;
    }
}

// cout[v] = 0 if a same-coloured neighbour has a smaller id, else cin[v]; *left |= uncoloured.
__global__ __launch_bounds__(kGffThreads) void gff_conflict_kernel(const uint64_t* __restrict__ ro,
                                                                   const uint32_t* __restrict__ col, uint32_t n,
                                                                   const uint32_t* __restrict__ cin,
                                                                   uint32_t* __restrict__ cout, uint32_t* left) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        const uint32_t cv = cin[v];
        bool lose = false;
        if (cv != 0) {
            for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) {
                const uint32_t w = col[k];
                if (w < v && cin[w] == cv) lose = true;
            }
        }
        lose = __ballot(lose) != 0ull;
        if (lane == 0) {
            const uint32_t r = lose ? 0u : cv;
            cout[v] = r;
            if (r == 0) atomicOr(left, 1u);
        }
    }
}

}  // namespace
}  // namespace mcmc

using namespace mcmc;

extern "C" int mcmc_greedyff_run(const mcmc_graph* g, uint32_t* colors, uint32_t* num_colors, uint32_t* rounds) {
    if (!g || !colors) return fail(MCMC_E_ARG, "NULL argument");
    const GraphDev& gd = g->g;
    if (!gd.row_off) return fail(MCMC_E_ARG, "greedy first fit needs a CSR graph (mcmc_graph_upload / _simulate)");
    const uint32_t n = gd.n;
    if (num_colors) *num_colors = 0;
    if (rounds) *rounds = 0;
    if (n == 0) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    const uint32_t maxColors = gd.maxDeg + 1;   // :17 (getMaxNodeDeg() + 1)
    const uint32_t W = (maxColors + 31u) / 32u;
    if (W * 4u * sizeof(uint32_t) > 64u * 1024u)
        return fail(MCMC_E_ARG, "greedy first fit: maxDeg beyond 131071 (LDS forbidden sets)");
    uint32_t *A = nullptr, *B = nullptr, *forb = nullptr, *left = nullptr;
    auto cleanup = [&]() { (void)hipFree(A); (void)hipFree(B); (void)hipFree(forb); (void)hipFree(left); };
#define GTRY(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            cleanup();                                                                              \
            return fail(MCMC_E_HIP, std::string("greedy first fit: " #expr ": ") + hipGetErrorString(_e)); \
        }                                                                                           \
    } while (0)
    GTRY(hipMalloc(&A, sizeof(uint32_t) * n));
    GTRY(hipMalloc(&B, sizeof(uint32_t) * n));
    GTRY(hipMalloc(&forb, sizeof(uint32_t) * (size_t)n * W));
    GTRY(hipMalloc(&left, sizeof(uint32_t)));
    GTRY(hipMemset(A, 0, sizeof(uint32_t) * n));
    GTRY(hipMemset(forb, 0, sizeof(uint32_t) * (size_t)n * W));
    const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 3u) / 4u, 65535u));
    const size_t lds = sizeof(uint32_t) * 4u * W;
    GTRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&gff_tentative_kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)std::max<size_t>(lds, 4)));
    uint32_t r = 0, h = 1;
    while (h) {
        r++;
        GTRY(hipMemsetAsync(left, 0, sizeof(uint32_t), 0));
        gff_tentative_kernel<<<blocks, kGffThreads, lds, 0>>>(gd.row_off, gd.col_idx, n, W, maxColors, A, B, forb);
        gff_conflict_kernel<<<blocks, kGffThreads, 0, 0>>>(gd.row_off, gd.col_idx, n, B, A, left);
        GTRY(hipGetLastError());
        GTRY(hipMemcpy(&h, left, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (r > 4u * maxColors + 64u) {   // the reference loops forever when a forbidden set fills up
            cleanup();
            return fail(MCMC_E_DEVICE, "greedy first fit: no progress (a node's forbidden set is full)");
        }
    }
    GTRY(hipMemcpy(colors, A, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
#undef GTRY
    cleanup();
    std::vector<uint32_t> s(colors, colors + n);   // numColors = |set of colours| (:79-80)
    std::sort(s.begin(), s.end());
    if (num_colors) *num_colors = (uint32_t)(std::unique(s.begin(), s.end()) - s.begin());
    if (rounds) *rounds = r;
    return MCMC_OK;
}
