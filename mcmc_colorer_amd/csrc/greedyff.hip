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
//
// The same rounds are the first phase of ColoringVFF (coloringVFF.cu, `--vffgpu`), whose
// rebalancing (mcmc_vff_run below; pinned by oracle/oracle_np.py::vff) follows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "mcmc_common.h"

namespace mcmc {
namespace {

constexpr int kGffThreads = 256;   // 4 waves, one node each at a time

// Orders one wave's LDS accesses between phases (plain stores, then ds_or atomics from other
// lanes, then reads): the HIP memory model does not promise wave lock-step ordering by itself.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
struct DevBuf {   // device allocation freed on every return path
    T* p = nullptr;
    hipError_t alloc(size_t k) { return hipMalloc(&p, sizeof(T) * std::max<size_t>(k, 1)); }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

__global__ __launch_bounds__(kGffThreads) void gff_tentative_kernel(const uint64_t* __restrict__ ro,
                                                                    const uint32_t* __restrict__ col, uint32_t n,
                                                                    uint32_t W, uint32_t maxColors,
                                                                    const uint32_t* __restrict__ cin,
                                                                    uint32_t* __restrict__ cout,
                                                                    uint32_t* __restrict__ forb,
                                                                    uint8_t* __restrict__ fresh) {
    extern __shared__ uint32_t lm[];   // [4 waves][W] forbidden bitmask of the wave's node
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t* m = lm + (size_t)wv * W;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        const uint32_t c0 = cin[v];
        if (v == 0 || c0 != 0) {   // node 0 always takes colour 1; coloured nodes keep theirs
            if (lane == 0) {
                cout[v] = v == 0 ? 1u : c0;
                fresh[v] = (v == 0 && c0 != 1u) ? 1 : 0;
            }
            continue;
        }
        uint32_t* fv = forb + (size_t)v * W;
        for (uint32_t w = lane; w < W; w += 64) m[w] = fv[w];
        wave_lds_sync();
        for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) {
            const uint32_t c = cin[col[k]];   // < maxColors: first-fit never picks past it
            atomicOr(&m[c >> 5], 1u << (c & 31u));
        }
        wave_lds_sync();
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
        wave_lds_sync();   // the next node's stores must not pass these reads
        if (lane == 0) {
            cout[v] = pick;
            fresh[v] = pick != 0 ? 1 : 0;
        }
    }
}

// cout[v] = 0 if a same-coloured neighbour has a smaller id, else cin[v]; *left |= uncoloured.
// On a symmetric CSR only a node coloured this round (fresh) can lose: its pick avoided the colours
// every neighbour had at the round's start, so a conflict needs a neighbour coloured this round
// too, and a pair of older nodes was settled in the round the later of them was coloured -- the
// other rows are not scanned (same result as the reference's full conflict_detection pass). On an
// asymmetric CSR a fresh w < v whose row lacks v may take v's colour, so every coloured row is
// scanned (fresh_only = 0), as the reference does.
__global__ __launch_bounds__(kGffThreads) void gff_conflict_kernel(const uint64_t* __restrict__ ro,
                                                                   const uint32_t* __restrict__ col, uint32_t n,
                                                                   const uint32_t* __restrict__ cin,
                                                                   uint32_t* __restrict__ cout, uint32_t* left,
                                                                   const uint8_t* __restrict__ fresh,
                                                                   uint32_t fresh_only) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        const uint32_t cv = cin[v];
        bool lose = false;
        if (cv != 0 && (fresh[v] || !fresh_only)) {
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

// ---- VFF rebalancing (coloringVFF.cu:101-228) ---------------------------------------------------
// bins[c] = nodes of colour c, c = 1..K (bins[0] stays 0; zeroed by the caller). LDS-privatised
// when the K + 1 counters fit, else global atomics.
__global__ __launch_bounds__(kGffThreads) void vff_bins_kernel(const uint32_t* __restrict__ C, uint32_t n, uint32_t K,
                                                               uint32_t* __restrict__ bins) {
    extern __shared__ uint32_t lb[];
    const bool lds = K + 1 <= 16384u;
    if (lds) {
        for (uint32_t c = threadIdx.x; c <= K; c += blockDim.x) lb[c] = 0;
        __syncthreads();
    }
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint32_t c = C[v];
        if (c >= 1 && c <= K) atomicAdd(lds ? &lb[c] : &bins[c], 1u);
    }
    if (lds) {
        __syncthreads();
        for (uint32_t c = threadIdx.x; c <= K; c += blockDim.x)
            if (lb[c]) atomicAdd(&bins[c], lb[c]);
    }
}

// over = bitmask of the colours whose bin holds more than gamma nodes (BIN_SIZE(.., i) > gamma);
// unb[v] = gamma < bin of C[v] when `detect` (detect_unbalanced_nodes, :300-311).
__global__ __launch_bounds__(kGffThreads) void vff_over_kernel(const uint32_t* __restrict__ bins, uint32_t K,
                                                               uint32_t gamma, uint32_t W, uint32_t* __restrict__ over) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W; w += gridDim.x * blockDim.x) {
        uint32_t m = 0;
        for (uint32_t b = 0; b < 32; b++) {
            const uint32_t c = 32u * w + b;
            if (c >= 1 && c <= K && gamma < bins[c]) m |= 1u << b;
        }
        over[w] = m;
    }
}
__global__ __launch_bounds__(kGffThreads) void vff_detect_kernel(const uint32_t* __restrict__ C, uint32_t n,
                                                                 const uint32_t* __restrict__ bins, uint32_t gamma,
                                                                 uint8_t* __restrict__ unb, uint32_t* flag) {
    bool any = false;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const bool u = gamma < bins[C[v]];
        unb[v] = u ? 1 : 0;
        any |= u;
    }
    if (__ballot(any) && (threadIdx.x & 63u) == 0) *flag = 1;
}

// tentative_rebalancing (:326-365): one wave per node; an unbalanced node other than node 0 (its
// forbidden row is flagged with the memset value 0) forbids its own and its neighbours' colours in
// an LDS bitmask and takes the first colour 1..K not forbidden and over; others keep theirs.
__global__ __launch_bounds__(kGffThreads) void vff_tentative_kernel(const uint64_t* __restrict__ ro,
                                                                    const uint32_t* __restrict__ col, uint32_t n,
                                                                    uint32_t W, const uint32_t* __restrict__ cin,
                                                                    uint32_t* __restrict__ cout,
                                                                    const uint8_t* __restrict__ unb,
                                                                    const uint32_t* __restrict__ over) {
    extern __shared__ uint32_t lm[];   // [4 waves][W]
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t* m = lm + (size_t)wv * W;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        const uint32_t c0 = cin[v];
        if (!unb[v] || v == 0) {
            if (lane == 0) cout[v] = c0;
            continue;
        }
        for (uint32_t w = lane; w < W; w += 64) m[w] = 0;
        wave_lds_sync();
        if (lane == 0) atomicOr(&m[c0 >> 5], 1u << (c0 & 31u));
        for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) {
            const uint32_t c = cin[col[k]];
            atomicOr(&m[c >> 5], 1u << (c & 31u));
        }
        wave_lds_sync();
        uint32_t pick = c0;
        for (uint32_t wb = 0; wb < W; wb += 64) {
            const uint32_t w = wb + lane;
            const uint32_t z = w < W ? (~m[w] & over[w]) : 0u;
            const unsigned long long b = __ballot(z != 0u);
            if (b) {
                const int f = __ffsll(b) - 1;
                const uint32_t zf = (uint32_t)__shfl((int)z, f, 64);
                pick = 32u * (wb + (uint32_t)f) + (uint32_t)__builtin_ctz(zf);
                break;
            }
        }
        wave_lds_sync();   // the next node's clearing stores must not pass the search's reads
        if (lane == 0) cout[v] = pick;
    }
}

// solve_conflicts (:386-409): an unbalanced node stays so iff a neighbour of smaller id has its
// colour; its colour is not reverted.
__global__ __launch_bounds__(kGffThreads) void vff_solve_kernel(const uint64_t* __restrict__ ro,
                                                                const uint32_t* __restrict__ col, uint32_t n,
                                                                const uint32_t* __restrict__ C,
                                                                uint8_t* __restrict__ unb) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        if (!unb[v]) continue;
        const uint32_t cv = C[v];
        bool stay = false;
        for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w < v && C[w] == cv) stay = true;
        }
        stay = __ballot(stay) != 0ull;
        if (lane == 0 && !stay) unb[v] = 0;
    }
}

// is_unbalanced + the history of ensure_not_looping (:412-434): ring[t % 9] = this iteration's
// unbalanced set; flags[0] = any unbalanced, flags[1] = differs from one of the 8 before it (slots
// not yet written hold the reference's all-false rows).
__global__ __launch_bounds__(kGffThreads) void vff_history_kernel(const uint8_t* __restrict__ unb, uint32_t n,
                                                                  uint8_t* __restrict__ ring, uint32_t t,
                                                                  uint32_t* flags) {
    bool any = false, diff = false;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint8_t u = unb[v];
        ring[(size_t)(t % 9u) * n + v] = u;
        any |= u != 0;
        for (uint32_t o = 1; o <= 8; o++) diff |= ring[(size_t)((t + 9u - o) % 9u) * n + v] != u;
    }
    if (__ballot(any) && (threadIdx.x & 63u) == 0) flags[0] = 1;
    if (__ballot(diff) && (threadIdx.x & 63u) == 0) flags[1] = 1;
}

}  // namespace
}  // namespace mcmc

using namespace mcmc;

namespace {

// The GreedyFF rounds (ColoringGreedyFF::run :50-84; ColoringVFF::run_coloring :58-99) into the
// device colouring A (n words, zeroed here); *rounds = loop iterations.
int gff_color(const GraphDev& gd, uint32_t* A, uint32_t* B, uint32_t* forb, uint32_t* left, uint32_t* rounds) {
    const uint32_t n = gd.n;
    DevBuf<uint8_t> fresh;
    MCMC_HIP_TRY(fresh.alloc(n));
    // sym: the conflict pass may scan only the rows coloured this round (gff_conflict_kernel). The
    // check needs ascending rows; it never reorders the caller's graph: an unsorted CSR (or one the
    // check cannot handle) takes the conservative pass over every coloured row, correct either way.
    bool sym = false;
    if (gd.sym >= 0) {
        sym = gd.sym == 1;
    } else if (gd.sorted) {
        GraphDev probe = gd;   // csr_symmetric caches into its argument: keep the caller's handle const
        if (csr_symmetric(probe, 0, n, 0, &sym) != MCMC_OK) sym = false;
    }
    const uint32_t maxColors = gd.maxDeg + 1;   // :17 (getMaxNodeDeg() + 1)
    const uint32_t W = (maxColors + 31u) / 32u;
    MCMC_HIP_TRY(hipMemset(A, 0, sizeof(uint32_t) * n));
    MCMC_HIP_TRY(hipMemset(forb, 0, sizeof(uint32_t) * (size_t)n * W));
    const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 3u) / 4u, 65535u));
    const size_t lds = sizeof(uint32_t) * 4u * W;
    MCMC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&gff_tentative_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)std::max<size_t>(lds, 4)));
    uint32_t r = 0, h = 1;
    while (h) {
        r++;
        MCMC_HIP_TRY(hipMemsetAsync(left, 0, sizeof(uint32_t), 0));
        gff_tentative_kernel<<<blocks, kGffThreads, lds, 0>>>(gd.row_off, gd.col_idx, n, W, maxColors, A, B, forb,
                                                              fresh.p);
        gff_conflict_kernel<<<blocks, kGffThreads, 0, 0>>>(gd.row_off, gd.col_idx, n, B, A, left, fresh.p,
                                                            sym ? 1u : 0u);
        MCMC_HIP_TRY(hipGetLastError());
        MCMC_HIP_TRY(hipMemcpy(&h, left, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (r > 4u * maxColors + 64u)   // the reference loops forever when a forbidden set fills up
            return fail(MCMC_E_DEVICE, "greedy first fit: no progress (a node's forbidden set is full)");
    }
    *rounds = r;
    return MCMC_OK;
}

}  // namespace

extern "C" int mcmc_greedyff_run(const mcmc_graph* g, uint32_t* colors, uint32_t* num_colors, uint32_t* rounds) {
    if (!g || !colors) return fail(MCMC_E_ARG, "NULL argument");
    const GraphDev& gd = g->g;
    if (!gd.row_off) return fail(MCMC_E_ARG, "greedy first fit needs a CSR graph (mcmc_graph_upload / _simulate)");
    const uint32_t n = gd.n;
    if (num_colors) *num_colors = 0;
    if (rounds) *rounds = 0;
    if (n == 0) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    const uint32_t W = (gd.maxDeg + 1u + 31u) / 32u;
    if (W * 4u * sizeof(uint32_t) > 64u * 1024u)
        return fail(MCMC_E_ARG, "greedy first fit: maxDeg beyond 131071 (LDS forbidden sets)");
    DevBuf<uint32_t> A, B, forb, left;
    MCMC_HIP_TRY(A.alloc(n));
    MCMC_HIP_TRY(B.alloc(n));
    MCMC_HIP_TRY(forb.alloc((size_t)n * W));
    MCMC_HIP_TRY(left.alloc(1));
    uint32_t r = 0;
    if (int rc = gff_color(gd, A.p, B.p, forb.p, left.p, &r)) return rc;
    MCMC_HIP_TRY(hipMemcpy(colors, A.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    std::vector<uint32_t> s(colors, colors + n);   // numColors = |set of colours| (:79-80)
    std::sort(s.begin(), s.end());
    if (num_colors) *num_colors = (uint32_t)(std::unique(s.begin(), s.end()) - s.begin());
    if (rounds) *rounds = r;
    return MCMC_OK;
}

extern "C" int mcmc_vff_run(const mcmc_graph* g, uint32_t* colors, uint32_t* num_colors, uint32_t* iterations,
                            int* valid) {
    if (!g || !colors) return fail(MCMC_E_ARG, "NULL argument");
    const GraphDev& gd = g->g;
    if (!gd.row_off) return fail(MCMC_E_ARG, "VFF needs a CSR graph (mcmc_graph_upload / _simulate)");
    const uint32_t n = gd.n;
    if (num_colors) *num_colors = 0;
    if (iterations) *iterations = 0;
    if (valid) *valid = 1;
    if (n == 0) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    const uint32_t W0 = (gd.maxDeg + 1u + 31u) / 32u;
    if (W0 * 4u * sizeof(uint32_t) > 64u * 1024u)
        return fail(MCMC_E_ARG, "VFF: maxDeg beyond 131071 (LDS forbidden sets)");
    DevBuf<uint32_t> A, B, forb, flags;
    MCMC_HIP_TRY(A.alloc(n));
    MCMC_HIP_TRY(B.alloc(n));
    MCMC_HIP_TRY(forb.alloc((size_t)n * W0));
    MCMC_HIP_TRY(flags.alloc(4));
    uint32_t r = 0;
    if (int rc = gff_color(gd, A.p, B.p, forb.p, flags.p, &r)) return rc;
    // numColors = |set of greedy colours| (:95-98); gamma = n / numColors (:103)
    std::vector<uint32_t> gff(n);
    MCMC_HIP_TRY(hipMemcpy(gff.data(), A.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    std::vector<uint32_t> s(gff);
    std::sort(s.begin(), s.end());
    const uint32_t K = (uint32_t)(std::unique(s.begin(), s.end()) - s.begin());
    if (s.front() < 1 || s.back() != K)
        return fail(MCMC_E_DEVICE, "VFF: greedy colours are not 1..numColors (the reference reads past its bins)");
    const uint32_t gamma = n / K;
    const uint32_t W = (K + 1u + 31u) / 32u;
    DevBuf<uint32_t> bins, over;
    DevBuf<uint8_t> unb, ring;
    MCMC_HIP_TRY(bins.alloc(K + 1));
    MCMC_HIP_TRY(over.alloc(W));
    MCMC_HIP_TRY(unb.alloc(n));
    MCMC_HIP_TRY(ring.alloc(9ull * n));
    MCMC_HIP_TRY(hipMemset(ring.p, 0, 9ull * n));   // the history rows start all-false (:106-107)
    const uint32_t tblocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + kGffThreads - 1) / kGffThreads, 4096u));
    const uint32_t wblocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 3u) / 4u, 65535u));
    const size_t blds = (K + 1u <= 16384u) ? sizeof(uint32_t) * (K + 1u) : 0;
    const size_t tlds = sizeof(uint32_t) * 4u * W;
    MCMC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&vff_tentative_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)std::max<size_t>(tlds, 4)));
    auto count = [&](const uint32_t* C) -> hipError_t {
        hipError_t e = hipMemsetAsync(bins.p, 0, sizeof(uint32_t) * (K + 1), 0);
        if (e != hipSuccess) return e;
        vff_bins_kernel<<<tblocks, kGffThreads, blds, 0>>>(C, n, K, bins.p);
        vff_over_kernel<<<std::max<uint32_t>(1u, (W + kGffThreads - 1) / kGffThreads), kGffThreads, 0, 0>>>(
            bins.p, K, gamma, W, over.p);
        return hipGetLastError();
    };
    MCMC_HIP_TRY(count(A.p));
    MCMC_HIP_TRY(hipMemsetAsync(flags.p, 0, 4 * sizeof(uint32_t), 0));
    vff_detect_kernel<<<tblocks, kGffThreads, 0, 0>>>(A.p, n, bins.p, gamma, unb.p, flags.p);
    MCMC_HIP_TRY(hipGetLastError());
    uint32_t h[2] = {0, 1};
    MCMC_HIP_TRY(hipMemcpy(h, flags.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
    uint32_t t = 0;
    bool notLooping = true;
    uint32_t *cin = A.p, *cout = B.p;
    while (h[0] && notLooping) {
        if (++t > 100000u) return fail(MCMC_E_DEVICE, "VFF: no progress (the unbalanced set cycles)");
        vff_tentative_kernel<<<wblocks, kGffThreads, tlds, 0>>>(gd.row_off, gd.col_idx, n, W, cin, cout, unb.p, over.p);
        MCMC_HIP_TRY(count(cout));   // update_bins + the inclusive scan (:166-176): sizes for the next pick
        vff_solve_kernel<<<wblocks, kGffThreads, 0, 0>>>(gd.row_off, gd.col_idx, n, cout, unb.p);
        std::swap(cin, cout);        // update_coloring_GPU (:178)
        MCMC_HIP_TRY(hipMemsetAsync(flags.p, 0, 2 * sizeof(uint32_t), 0));
        vff_history_kernel<<<tblocks, kGffThreads, 0, 0>>>(unb.p, n, ring.p, t, flags.p);
        MCMC_HIP_TRY(hipGetLastError());
        MCMC_HIP_TRY(hipMemcpy(h, flags.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
        notLooping = h[1] != 0;   // ensure_not_looping: the set equals the 8 before it -> stop
    }
    if (notLooping) MCMC_HIP_TRY(hipMemcpy(colors, cin, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    else std::copy(gff.begin(), gff.end(), colors);   // "Coloring resetted to Greedy First Fit" (:205-207)
    if (num_colors) *num_colors = K;
    if (iterations) *iterations = t;
    if (valid) *valid = notLooping ? 1 : 0;
    return MCMC_OK;
}
