// mcmc_colorer_amd/csrc/tailcut.hip -- tail cutting after the sweep loop, on the device.
//
// Reference: ColoringMCMC_CPU::run(), coloringMCMC_CPU.cpp:272-311. After the loop, when z > 0
// the colour order colorIdx is sorted by ascending colour histogram (:272-278); then, while
// Cviol > 0, every vertex i flagged in Cviols (ascending i) takes the first colour of colorIdx not
// used by any neighbour, reading the colouring as it is being modified (a Gauss-Seidel pass,
// :281-305), and Cviol/Cviols are recounted (:308). The reference's inner loop increments i
// instead of k (:289) and never terminates; this is the corrected pass (k++), bounded by a pass
// cap, exactly as the oracle's tail_cut() (oracle/mcmc_cpu_ref.cpp) states it.
//
// Quirk kept: run() swaps C/Cstar and the counts but not the flag vectors (:259-260), so the
// first pass visits the vertices flagged in the colouring BEFORE the last accepted sweep (or the
// initial colouring when no sweep was accepted). The sweep kernels keep those flags when a
// context has tail cutting enabled (SweepArgs::vflags, mcmc_sweep.hip).
//
// The reference GPU colorer's tail cut (coloringMCMC_main.cu:271-290, coloringMCMC_utils.cu:73-119;
// reference-GPU-semantics mode) shares the kernels: conflicts are counted as edges (a flagged vertex
// has a same-colour neighbour with a larger id), the repair keeps a free own colour and otherwise
// takes the first free colour of orderedIndex (the last one when none is free), and a pass stops
// after conflictCounter flagged vertices.
//
// Kernels (one context, whole graph):
//   tail_count_kernel   one wave per row: flag = any neighbour with the row's colour; Cviol.
//   rocprim::select     flagged rows -> ascending list (order-preserving compaction).
//   tail_repair_kernel  ONE workgroup walks the list in order; per vertex the 16 waves scan the
//                       row, OR the neighbours' colours into an occupancy mask, thread 0 writes
//                       the first free colour of colorIdx. Sequential by definition (each vertex
//                       sees the colours written for earlier vertices of the same pass); the list
//                       is the handful of conflicts left at loop exit (<= z when converged).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "mcmc_common.h"

namespace mcmc {

namespace {

// Neighbours of local row l, from the CSR (global ids) or the tiled layout (block-local 16-bit
// ids, segments padded with copies of a real neighbour -- harmless for occupancy and conflicts).
// Calls f(w) for every neighbour at positions part, part + parts, ... of the row's arc stream.
// SKIP_PADS: leave out the padding (a segment's padding count is in its table entry's low bits).
template <bool SKIP_PADS = false, class F>
__device__ __forceinline__ void for_neighbours(const TailView& g, uint32_t l, uint32_t part, uint32_t parts, F&& f) {
    if (g.row_off) {
        const uint64_t rs = g.row_off[g.csr_row0 + l], re = g.row_off[g.csr_row0 + l + 1];
        for (uint64_t k = rs + part; k < re; k += parts) f(g.col_idx[k]);
        return;
    }
    const uint32_t grp = l / g.R, r = l - grp * g.R;
    const uint16_t* ids = g.tcol + g.gbase[grp];
    const uint32_t stride = tseg_stride(g.R);
    const uint32_t* ts = g.tseg + (size_t)grp * g.nb * stride;
    for (uint32_t b = 0; b < g.nb; b++) {
        const uint32_t raw = ts[(size_t)b * stride + r];
        const uint32_t s0 = raw & kTsegPos, s1 = (ts[(size_t)b * stride + r + 1] & kTsegPos) - (SKIP_PADS ? raw & 7u : 0u);
        const uint32_t hi = b << g.block_log2;
        for (uint32_t k = s0 + part; k < s1; k += parts) f(hi | ids[k]);
    }
}

// EDGES = false: flag = any same-colour neighbour (violation_count), count = flagged vertices.
// EDGES = true: per-vertex same-colour neighbours with a larger id (conflictCounter kernel),
// flag = nonzero, count = their sum (calcConflicts).
// CT: the replica's colour type (uint8_t; uint16_t for the wide sweep's nCol > 256).
template <bool EDGES, typename CT>
__global__ __launch_bounds__(256) void tail_count_kernel(TailView g, const CT* __restrict__ C,
                                                         uint8_t* __restrict__ flags,
                                                         unsigned long long* __restrict__ count) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    unsigned long long wave_total = 0;
    for (uint32_t l = gw; l < g.n; l += nw) {
        const CT cv = C[g.vb + l];
        uint32_t hits = 0;
        if (EDGES) {
            for_neighbours<true>(g, l, lane, 64u, [&](uint32_t w) { hits += (C[w] == cv && w > g.vb + l) ? 1u : 0u; });
            for (int off = 32; off > 0; off >>= 1) hits += __shfl_xor(hits, off, 64);
        } else {
            bool hit = false;
            for_neighbours(g, l, lane, 64u, [&](uint32_t w) { hit |= C[w] == cv; });
            hits = __ballot(hit) != 0 ? 1u : 0u;
        }
        if (lane == 0) flags[l] = hits != 0;
        wave_total += hits;
    }
    if (lane == 0 && wave_total) atomicAdd(count, wave_total);
}

constexpr uint32_t kRepairThreads = 1024;
constexpr int kMaskWords = 8;            // nCol <= 256 (uint8 colours): masks in registers
constexpr uint32_t kWideMaskWords = 2048;   // nCol <= 65535 (uint16 colours): the mask in LDS

// REF = false: the corrected CPU rule (first free colour of colorIdx, unchanged when none is free).
// REF = true: tailCutting (coloringMCMC_utils.cu:73-101): an own colour that is free (or >= nCol)
// stays; otherwise the first free colour of orderedIndex, the last one when none is free. At most
// `limit` listed vertices (resolved < conflictCounter). CT = uint16_t: the wide sweep's replicas;
// the occupancy mask (nCol bits) is built in LDS.
template <bool REF, typename CT>
__global__ __launch_bounds__(kRepairThreads) void tail_repair_kernel(TailView g, CT* C,
                                                                     const uint32_t* __restrict__ list,
                                                                     const uint32_t* __restrict__ list_len,
                                                                     const uint32_t* __restrict__ colorIdx,
                                                                     uint32_t nCol, unsigned long long limit) {
    constexpr bool WIDE = sizeof(CT) == 2;
    constexpr uint32_t MW = WIDE ? kWideMaskWords : (uint32_t)kMaskWords;
    __shared__ uint32_t mask[MW];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t L = (uint32_t)min((unsigned long long)*list_len, limit);
    const uint32_t words = WIDE ? (nCol + 31u) >> 5 : (uint32_t)kMaskWords;
    // colours of this pass are read with volatile (L1-bypassing) loads: vertex k must see the
    // colour thread 0 stored for an earlier vertex of the list
    const volatile CT* Cv = C;
    for (uint32_t k = 0; k < L; k++) {
        const uint32_t li = list[k];   // local row; i: its vertex (the replica's index)
        const uint32_t i = g.vb + li;
        for (uint32_t w = tid; w < words; w += blockDim.x) mask[w] = 0;
        __syncthreads();
        if (WIDE) {
            for_neighbours(g, li, tid, kRepairThreads, [&](uint32_t w) {
                const uint32_t c = Cv[w];
                if (c < nCol) atomicOr(&mask[c >> 5], 1u << (c & 31));
            });
        } else {
            uint32_t m[kMaskWords] = {};
            for_neighbours(g, li, tid, kRepairThreads, [&](uint32_t w) {
                const uint32_t c = Cv[w];
#pragma unroll
                for (int q = 0; q < kMaskWords; q++) m[q] |= (c >> 5) == (uint32_t)q ? 1u << (c & 31) : 0u;
            });
#pragma unroll
            for (int q = 0; q < kMaskWords; q++) {
                uint32_t x = m[q];
                for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
                if (lane == 0 && x) atomicOr(&mask[q], x);
            }
        }
        __syncthreads();
        if (tid == 0) {
            auto used = [&](uint32_t c) { return c < nCol && ((mask[c >> 5] >> (c & 31)) & 1u); };
            if (REF) {
                uint32_t c = Cv[i];
                for (uint32_t j = 0; used(c) && j < nCol; j++) c = colorIdx[j];
                C[i] = (CT)c;
            } else {
                for (uint32_t j = 0; j < nCol; j++) {      // first free colour in colorIdx order
                    const uint32_t c = colorIdx[j];
                    if (!used(c)) { C[i] = (CT)c; break; }
                }
            }
            __threadfence();
        }
        __syncthreads();
    }
}

}  // namespace

int tail_count(const TailView& g, const void* C, uint32_t cbytes, uint8_t* flags, unsigned long long* count,
               hipStream_t s, bool edges) {
    MCMC_HIP_TRY(hipMemsetAsync(count, 0, sizeof(unsigned long long), s));
    if (g.n == 0) return MCMC_OK;
    const uint32_t blocks = std::min<uint32_t>((g.n + 3) / 4, 8192u);   // 4 rows (waves) per block
    if (cbytes == 2) {
        const uint16_t* c = static_cast<const uint16_t*>(C);
        if (edges) tail_count_kernel<true, uint16_t><<<blocks, 256, 0, s>>>(g, c, flags, count);
        else tail_count_kernel<false, uint16_t><<<blocks, 256, 0, s>>>(g, c, flags, count);
    } else {
        const uint8_t* c = static_cast<const uint8_t*>(C);
        if (edges) tail_count_kernel<true, uint8_t><<<blocks, 256, 0, s>>>(g, c, flags, count);
        else tail_count_kernel<false, uint8_t><<<blocks, 256, 0, s>>>(g, c, flags, count);
    }
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

int tail_select(const uint8_t* flags, uint32_t n, uint32_t* list, uint32_t* list_len, void** tmp, size_t* tmp_bytes,
                hipStream_t s) {
    rocprim::counting_iterator<uint32_t> ids(0u);
    size_t need = 0;
    MCMC_HIP_TRY(rocprim::select(nullptr, need, ids, flags, list, list_len, n, s));
    if (need > *tmp_bytes) {
        if (*tmp) MCMC_HIP_TRY(hipFree(*tmp));
        *tmp = nullptr;
        MCMC_HIP_TRY(hipMalloc(tmp, need));
        *tmp_bytes = need;
    }
    MCMC_HIP_TRY(rocprim::select(*tmp, need, ids, flags, list, list_len, n, s));
    return MCMC_OK;
}

int tail_repair(const TailView& g, void* C, uint32_t cbytes, const uint32_t* list, const uint32_t* list_len,
                const uint32_t* colorIdx, uint32_t nCol, hipStream_t s, bool ref, unsigned long long limit) {
    if (cbytes == 2) {
        if (nCol > 32u * kWideMaskWords) return MCMC_E_ARG;
        uint16_t* c = static_cast<uint16_t*>(C);
        if (ref) tail_repair_kernel<true, uint16_t><<<1, kRepairThreads, 0, s>>>(g, c, list, list_len, colorIdx, nCol, limit);
        else tail_repair_kernel<false, uint16_t><<<1, kRepairThreads, 0, s>>>(g, c, list, list_len, colorIdx, nCol, limit);
    } else {
        if (nCol > 32u * kMaskWords) return MCMC_E_ARG;
        uint8_t* c = static_cast<uint8_t*>(C);
        if (ref) tail_repair_kernel<true, uint8_t><<<1, kRepairThreads, 0, s>>>(g, c, list, list_len, colorIdx, nCol, limit);
        else tail_repair_kernel<false, uint8_t><<<1, kRepairThreads, 0, s>>>(g, c, list, list_len, colorIdx, nCol, limit);
    }
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

}  // namespace mcmc
