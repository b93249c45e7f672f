// mcmc_colorer_amd/csrc/tiled_layout.hip -- the tiled adjacency layout the sweep streams
// (DESIGN.md §4): built from a CSR (get_tiled_layout), or written directly by the counter-based
// G(n, p) generator (mcmc_graph_er_fast*, er_gen.h) where no CSR fits (C3: 1e11 arcs).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "er_gen.h"
#include "mcmc_common.h"

namespace mcmc {

// ---- tiled layout construction (once per context) ----------------------------------------------
// Padded (to 8 ids) total of every group over all blocks.
__global__ void tile_group_total_kernel(const uint32_t* __restrict__ seg, uint32_t nloc, uint32_t nb, uint32_t R,
                                        uint32_t G, uint64_t* __restrict__ totals) {
    __shared__ unsigned long long red[256];
    for (uint32_t g = blockIdx.x; g < G; g += gridDim.x) {
        const uint32_t r0 = g * R, rows = min(R, nloc - r0);
        unsigned long long s = 0;
        for (uint32_t i = threadIdx.x; i < rows * nb; i += blockDim.x) {
            const uint32_t b = i / rows, r = i % rows;
            const uint32_t len = seg[(size_t)(b + 1) * nloc + r0 + r] - seg[(size_t)b * nloc + r0 + r];
            s += (len + 7u) & ~7u;
        }
        red[threadIdx.x] = s;
        __syncthreads();
        for (uint32_t k = blockDim.x / 2; k > 0; k >>= 1) {
            if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
            __syncthreads();
        }
        if (threadIdx.x == 0) totals[g] = red[0];
        __syncthreads();
    }
}

// tseg[g][b][r] = padded start of row r's block-b segment relative to the group base (a multiple
// of 8) | the segment's padding count (0..7) in the low 3 bits; entry R of every block = its end
// (= the next block's start). Readers mask with ~7 (kTsegPos); the padding count gives the true end
// (the reference-GPU-semantics scan counts arcs exactly). Block scan over the rows, blocks in order.
__global__ void tile_seg_kernel(const uint32_t* __restrict__ seg, uint32_t nloc, uint32_t nb, uint32_t R,
                                uint32_t G, uint32_t* __restrict__ tseg) {
    __shared__ uint32_t part[256];
    __shared__ uint32_t run_sh;
    for (uint32_t g = blockIdx.x; g < G; g += gridDim.x) {
        const uint32_t r0 = g * R, rows = min(R, nloc - r0);
        const uint32_t per = (R + blockDim.x - 1) / blockDim.x;   // consecutive rows per thread
        if (threadIdx.x == 0) run_sh = 0;
        __syncthreads();
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t ra = threadIdx.x * per, rb = min(R, ra + per);
            uint32_t local = 0;
            for (uint32_t r = ra; r < rb; r++) {
                const uint32_t len = (r < rows) ? seg[(size_t)(b + 1) * nloc + r0 + r] - seg[(size_t)b * nloc + r0 + r] : 0u;
                local += (len + 7u) & ~7u;
            }
            part[threadIdx.x] = local;
            __syncthreads();
            if (threadIdx.x == 0) {   // exclusive scan of the per-thread sums (blockDim <= 256)
                uint32_t acc = 0;
                for (uint32_t k = 0; k < blockDim.x; k++) { const uint32_t x = part[k]; part[k] = acc; acc += x; }
            }
            __syncthreads();
            const uint32_t run = run_sh;
            uint32_t* out = tseg + ((size_t)g * nb + b) * tseg_stride(R);
            uint32_t acc = run + part[threadIdx.x];
            for (uint32_t r = ra; r < rb; r++) {
                const uint32_t len = (r < rows) ? seg[(size_t)(b + 1) * nloc + r0 + r] - seg[(size_t)b * nloc + r0 + r] : 0u;
                out[r] = acc | (((len + 7u) & ~7u) - len);
                acc += (len + 7u) & ~7u;
            }
            __syncthreads();
            if (threadIdx.x == blockDim.x - 1) {
                out[R] = acc;   // the last thread's running value is the block's end
                run_sh = acc;
            }
            __syncthreads();
        }
    }
}

// Scatter: wave per local row; every arc to its padded block segment as a 16-bit local id, then
// each segment's padding filled with copies of its first id (OR-idempotent).
__global__ void tile_scatter_kernel(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ col_idx,
                                    const uint32_t* __restrict__ seg, const uint64_t* __restrict__ gbase,
                                    const uint32_t* __restrict__ tseg, uint32_t nloc, uint32_t nb, uint32_t R,
                                    uint32_t block_log2, uint16_t* __restrict__ tcol) {
    const int lane = threadIdx.x & 63;
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t bmask = (1u << block_log2) - 1u;
    for (uint32_t l = gw; l < nloc; l += nw) {
        const uint32_t g = l / R, r = l % R;
        const uint64_t rs = row_off[l], re = row_off[l + 1];
        const uint64_t base = gbase[g];
        const uint32_t* ts = tseg + (size_t)g * nb * tseg_stride(R);
        for (uint64_t k = rs + lane; k < re; k += 64) {
            const uint32_t c = col_idx[k];
            const uint32_t b = c >> block_log2;
            const uint32_t rel = (uint32_t)(k - rs) - seg[(size_t)b * nloc + l];
            tcol[base + (ts[(size_t)b * tseg_stride(R) + r] & kTsegPos) + rel] = (uint16_t)(c & bmask);
        }
        for (uint32_t b = lane; b < nb; b += 64) {
            const uint32_t s0 = seg[(size_t)b * nloc + l], s1 = seg[(size_t)(b + 1) * nloc + l];
            const uint32_t len = s1 - s0;
            if (len & 7u) {
                const uint16_t first = (uint16_t)(col_idx[rs + s0] & bmask);
                const uint64_t p0 = base + (ts[(size_t)b * tseg_stride(R) + r] & kTsegPos);
                for (uint32_t i = len; i < ((len + 7u) & ~7u); i++) tcol[p0 + i] = first;
            }
        }
    }
}

// Segment offsets of every local row by column block: seg[b][l] = #neighbours of row l with id
// < b*B (rows ascending), b = 0..nb. Thread per (block boundary, row) binary search.
__global__ void segment_kernel(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ col_idx,
                               uint32_t nloc, uint32_t nb, uint32_t block_log2, uint32_t* __restrict__ seg) {
    const uint64_t total = (uint64_t)(nb + 1) * nloc;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(i / nloc), l = (uint32_t)(i % nloc);
        const uint64_t rs = row_off[l], re = row_off[l + 1];
        if (b == 0) { seg[i] = 0; continue; }
        if (b == nb) { seg[i] = (uint32_t)(re - rs); continue; }
        const uint64_t key = (uint64_t)b << block_log2;
        uint64_t lo = rs, hi = re;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (col_idx[mid] < key) lo = mid + 1; else hi = mid;
        }
        seg[i] = (uint32_t)(lo - rs);
    }
}

TiledLayout::~TiledLayout() {
    (void)hipFree(tcol);
    (void)hipFree(gbase);
    (void)hipFree(tseg);
}

namespace {

// Shared layout steps: from seg[b][l] (per-row cumulative segment offsets over the blocks,
// (nb+1) x nloc) to gbase (padded group sizes, scanned), tseg, and a zeroed tcol.
int layout_from_seg(TiledLayout& L, const uint32_t* seg, hipStream_t s) {
    const uint32_t nloc = L.v_end - L.v_begin, nb = L.nblocks, G = L.ngroups, R = L.grp_rows;
    uint64_t* totals = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
    chk(hipMalloc(&totals, sizeof(uint64_t) * (G + 1)));
    chk(hipMalloc(&L.gbase, sizeof(uint64_t) * (G + 1)));
    chk(hipMalloc(&L.tseg, sizeof(uint32_t) * std::max<size_t>((size_t)G * nb * tseg_stride(R), 4)));
    if (e == hipSuccess && nloc) {
        tile_group_total_kernel<<<std::min<uint32_t>(G, 65535), 256, 0, s>>>(seg, nloc, nb, R, G, totals);
        chk(hipMemsetAsync(totals + G, 0, sizeof(uint64_t), s));
        chk(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, totals, L.gbase, G + 1, s));
        chk(hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16)));
        if (e == hipSuccess) chk(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, totals, L.gbase, G + 1, s));
        chk(hipMemcpyAsync(&L.ids, L.gbase + G, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        chk(hipStreamSynchronize(s));
    }
    if (e == hipSuccess) chk(hipMalloc(&L.tcol, sizeof(uint16_t) * (L.ids + 64)));
    if (e == hipSuccess) chk(hipMemsetAsync(L.tcol, 0, sizeof(uint16_t) * (L.ids + 64), s));
    if (e == hipSuccess && nloc) {
        tile_seg_kernel<<<std::min<uint32_t>(G, 65535), 256, 0, s>>>(seg, nloc, nb, R, G, L.tseg);
        chk(hipGetLastError());
    }
    (void)hipStreamSynchronize(s);
    (void)hipFree(totals);
    (void)hipFree(tmp);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("tiled layout: ") + hipGetErrorString(e));
    return MCMC_OK;
}

TiledLayout* new_layout(uint32_t n, uint32_t v_begin, uint32_t v_end, uint32_t R, uint32_t block_log2) {
    auto* L = new TiledLayout();
    const uint32_t nloc = v_end - v_begin;
    L->v_begin = v_begin;
    L->v_end = v_end;
    L->grp_rows = R;
    L->block_log2 = block_log2;
    L->nblocks = (uint32_t)((((uint64_t)n + 15) / 16 * 16 + (1ull << block_log2) - 1) >> block_log2);
    L->ngroups = (nloc + R - 1) / R;
    return L;
}

// ---- counter-based G(n, p) straight into the tiled layout (er_gen.h) ---------------------------
struct ErArgs {
    uint64_t seed;
    double inv_l1p;
    int p_mode;         // 0 regular, 1 complete, 2 empty
    uint32_t n, vb, ve, nb;
};

__device__ __forceinline__ uint64_t tile_pos(const uint64_t* gbase, const uint32_t* tseg, uint32_t R, uint32_t nb,
                                             uint32_t l, uint32_t b) {
    const uint32_t g = l / R, r = l - g * R;
    return gbase[g] + (tseg[((size_t)g * nb + b) * tseg_stride(R) + r] & kTsegPos);
}

// Streams (i, Y) whose edges touch rows [vb, ve): row i own (any Y >= block(i)), or column block Y
// meeting [vb, ve) (transposed arcs into own rows). blockIdx.y = Y; rows grid-strided.
// FILL = false: counts per (block, own row) into cnt[b * nloc + l]. FILL = true: cnt holds write
// cursors; the direct arcs of a stream take one cursor bump (two walks), transposed arcs one each.
template <bool FILL>
__global__ __launch_bounds__(256) void er_tiled_kernel(ErArgs e, uint32_t* __restrict__ cnt,
                                                       const uint64_t* __restrict__ gbase,
                                                       const uint32_t* __restrict__ tseg, uint32_t R,
                                                       uint16_t* __restrict__ tcol) {
    constexpr uint32_t T = 1u << er::kBlockLog2;
    const uint32_t Y = blockIdx.y;
    const uint64_t y0 = (uint64_t)Y * T, y1 = std::min<uint64_t>(e.n, y0 + T);
    const bool yhit = y0 < e.ve && y1 > e.vb;
    const uint32_t lo = yhit ? 0u : e.vb;
    const uint32_t hi = (uint32_t)std::min<uint64_t>(e.ve, y1);
    const uint32_t nloc = e.ve - e.vb;
    for (uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += gridDim.x * blockDim.x) {
        const bool own_i = i >= e.vb;
        const uint32_t Xi = i >> er::kBlockLog2;
        if (!yhit && !own_i) continue;
        if (!FILL) {
            uint32_t cdir = 0;
            er::walk_stream(e.seed, e.inv_l1p, e.p_mode, e.n, i, Y, [&](uint32_t j) {
                cdir++;
                if (j >= e.vb && j < e.ve) atomicAdd(&cnt[(size_t)Xi * nloc + (j - e.vb)], 1u);
            });
            if (own_i && cdir) atomicAdd(&cnt[(size_t)Y * nloc + (i - e.vb)], cdir);
        } else {
            uint16_t* drow = nullptr;
            if (own_i) {
                const uint32_t c = er::walk_stream(e.seed, e.inv_l1p, e.p_mode, e.n, i, Y, [](uint32_t) {});
                if (c) {
                    const uint32_t l = i - e.vb;
                    const uint32_t base = atomicAdd(&cnt[(size_t)Y * nloc + l], c);
                    drow = tcol + tile_pos(gbase, tseg, R, e.nb, l, Y) + base;
                }
            }
            if (!drow && !yhit) continue;
            uint32_t k = 0;
            er::walk_stream(e.seed, e.inv_l1p, e.p_mode, e.n, i, Y, [&](uint32_t j) {
                if (drow) drow[k++] = (uint16_t)(j & (T - 1));
                if (j >= e.vb && j < e.ve) {
                    const uint32_t l = j - e.vb;
                    const uint32_t slot = atomicAdd(&cnt[(size_t)Xi * nloc + l], 1u);
                    tcol[tile_pos(gbase, tseg, R, e.nb, l, Xi) + slot] = (uint16_t)(i & (T - 1));
                }
            });
        }
    }
}

// In place: cnt[b][l] (lengths, (nb+1) x nloc with row nb spare) -> seg[b][l] = cumulative offsets,
// seg[nb][l] = degree; degree statistics on the side.
__global__ void er_prefix_kernel(uint32_t* cnt, uint32_t nloc, uint32_t nb, unsigned long long* stats) {
    unsigned long long sum = 0;
    uint32_t mx = 0, mn = 0xFFFFFFFFu;
    for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < nloc; l += gridDim.x * blockDim.x) {
        uint32_t run = 0;
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t x = cnt[(size_t)b * nloc + l];
            cnt[(size_t)b * nloc + l] = run;
            run += x;
        }
        cnt[(size_t)nb * nloc + l] = run;
        sum += run;
        mx = std::max(mx, run);
        mn = std::min(mn, run);
    }
    if (sum) atomicAdd(&stats[0], sum);
    atomicMax(reinterpret_cast<unsigned int*>(&stats[1]), mx);
    atomicMin(reinterpret_cast<unsigned int*>(&stats[2]), mn);
}

// Padding of every (row, block) segment to whole quads with copies of its first id.
__global__ void er_pad_kernel(const uint32_t* __restrict__ cur, const uint64_t* __restrict__ gbase,
                              const uint32_t* __restrict__ tseg, uint32_t R, uint32_t nloc, uint32_t nb,
                              uint16_t* __restrict__ tcol) {
    const uint64_t total = (uint64_t)nb * nloc;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(x / nloc), l = (uint32_t)(x % nloc);
        const uint32_t len = cur[x];
        if (!(len & 7u)) continue;
        uint16_t* p = tcol + tile_pos(gbase, tseg, R, nb, l, b);
        const uint16_t first = p[0];
        for (uint32_t k = len; k < ((len + 7u) & ~7u); k++) p[k] = first;
    }
}

}  // namespace

// Builds (or finds in the graph's cache) the tiled layout of rows [v_begin, v_end) from the CSR.
int get_tiled_layout(mcmc_graph* gh, uint32_t v_begin, uint32_t v_end, uint32_t R, uint32_t block_log2,
                     hipStream_t s, const TiledLayout** out) {
    for (auto& t : gh->tiles)
        if (t->v_begin == v_begin && t->v_end == v_end && t->block_log2 == block_log2 &&
            (t->grp_rows == R || !gh->g.row_off)) {
            *out = t.get();
            return MCMC_OK;
        }
    GraphDev& gd = gh->g;
    if (!gd.row_off)
        return fail(MCMC_E_STATE, "generated graph has no tiled layout for rows [" + std::to_string(v_begin) + ", " +
                                      std::to_string(v_end) + ") (generate it for this range)");
    if (!gd.sorted) {   // segments need ascending rows; neighbour order does not affect the sweep
        int rs = sort_rows_inplace(gd);
        if (rs) return rs;
    }
    std::unique_ptr<TiledLayout> L(new_layout(gd.n, v_begin, v_end, R, block_log2));
    const uint32_t nloc = v_end - v_begin, nb = L->nblocks;
    uint32_t* seg = nullptr;
    const size_t segn = (size_t)(nb + 1) * std::max<uint32_t>(nloc, 1);
    MCMC_HIP_TRY(hipMalloc(&seg, sizeof(uint32_t) * segn));
    if (nloc)
        segment_kernel<<<(uint32_t)std::min<size_t>((segn + 255) / 256, 65536), 256, 0, s>>>(
            gd.row_off + v_begin, gd.col_idx, nloc, nb, block_log2, seg);
    int rc = layout_from_seg(*L, seg, s);
    if (!rc && nloc) {
        tile_scatter_kernel<<<2048, 256, 0, s>>>(gd.row_off + v_begin, gd.col_idx, seg, L->gbase, L->tseg, nloc, nb,
                                                 R, block_log2, L->tcol);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = fail(MCMC_E_HIP, std::string("tiled scatter: ") + hipGetErrorString(e));
    }
    (void)hipFree(seg);
    if (rc) return rc;
    uint64_t ends[2] = {0, 0};
    MCMC_HIP_TRY(hipMemcpy(&ends[0], gd.row_off + v_begin, sizeof(uint64_t), hipMemcpyDeviceToHost));
    MCMC_HIP_TRY(hipMemcpy(&ends[1], gd.row_off + v_end, sizeof(uint64_t), hipMemcpyDeviceToHost));
    L->arcs = ends[1] - ends[0];
    *out = L.get();
    gh->tiles.push_back(std::move(L));
    return MCMC_OK;
}

// Group rows of the tiled layout a context on `nloc` rows picks by default (mcmc_create and the
// generator agree): the group count a multiple of the CU count (k groups per workgroup, so no
// workgroup finishes a group later than the others: C4's 1.25e6 rows per rank at R = 1792 were 698
// groups = 2 or 3 per workgroup), R at most `rmax`, at least 32.
uint32_t tiled_default_rows(uint32_t nloc, uint32_t cus, uint32_t rmax) {
    cus = std::max<uint32_t>(cus, 1);
    rmax = std::max<uint32_t>(rmax, 1);
    const uint64_t k = std::max<uint64_t>(1, ((uint64_t)nloc + (uint64_t)cus * rmax - 1) / ((uint64_t)cus * rmax));
    const uint32_t R = (uint32_t)(((uint64_t)nloc + k * cus - 1) / (k * cus));
    return std::max<uint32_t>(std::min<uint32_t>(32u, rmax), std::min<uint32_t>(rmax, R));
}

// Selected rows of a full-range tiled layout (test hook mcmc_graph_rows; all rows for
// mcmc_graph_materialize_csr): thread per row walks its nb segments; pass 1 (ids == nullptr) the
// degrees, pass 2 the ids at off[i].
__global__ void tile_rows_kernel(const uint16_t* __restrict__ tcol, const uint64_t* __restrict__ gbase,
                                 const uint32_t* __restrict__ tseg, uint32_t R, uint32_t nb, uint32_t block_log2,
                                 const uint32_t* __restrict__ rows, uint32_t k, const uint64_t* __restrict__ off,
                                 uint64_t* __restrict__ deg, uint32_t* __restrict__ ids, uint64_t* __restrict__ pos) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const uint32_t v = rows ? rows[i] : i, g = v / R, r = v - g * R;   // rows == nullptr: all rows
    uint64_t d = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t* t = tseg + ((size_t)g * nb + b) * tseg_stride(R);
        const uint64_t q0 = gbase[g] + (t[r] & kTsegPos), q1 = gbase[g] + (t[r + 1] & kTsegPos) - (t[r] & 7u);
        if (b == 0 && pos) pos[i] = q0;
        if (ids)
            for (uint64_t q = q0; q < q1; q++) ids[off[i] + d + (q - q0)] = (b << block_log2) | tcol[q];
        d += q1 - q0;
    }
    if (deg) deg[i] = d;
}

// CSR of a generated graph whose layout covers all rows (tests and small exports): every row's
// padded segments concatenated, padding duplicates dropped, ascending.
int tiled_to_csr(const mcmc_graph* gh, uint64_t* row_off, uint32_t* col_idx) {
    const TiledLayout* L = nullptr;
    for (auto& t : gh->tiles)
        if (t->v_begin == 0 && t->v_end == gh->g.n) L = t.get();
    if (!L) return fail(MCMC_E_STATE, "graph has neither a CSR nor a full-range tiled layout");
    const uint32_t n = gh->g.n, R = L->grp_rows, nb = L->nblocks, G = L->ngroups;
    std::vector<uint16_t> tc(L->ids);
    std::vector<uint64_t> gb(G + 1);
    std::vector<uint32_t> ts((size_t)G * nb * tseg_stride(R));
    MCMC_HIP_TRY(hipSetDevice(gh->g.device));
    MCMC_HIP_TRY(hipMemcpy(tc.data(), L->tcol, sizeof(uint16_t) * L->ids, hipMemcpyDeviceToHost));
    MCMC_HIP_TRY(hipMemcpy(gb.data(), L->gbase, sizeof(uint64_t) * (G + 1), hipMemcpyDeviceToHost));
    MCMC_HIP_TRY(hipMemcpy(ts.data(), L->tseg, sizeof(uint32_t) * ts.size(), hipMemcpyDeviceToHost));
    uint64_t k = 0;
    std::vector<uint32_t> row;
    for (uint32_t v = 0; v < n; v++) {
        const uint32_t g = v / R, r = v % R;
        row.clear();
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t* t = ts.data() + ((size_t)g * nb + b) * tseg_stride(R);
            const uint64_t q0 = gb[g] + (t[r] & kTsegPos), q1 = gb[g] + (t[r + 1] & kTsegPos) - (t[r] & 7u);
            for (uint64_t q = q0; q < q1; q++) row.push_back((b << L->block_log2) | tc[q]);
        }
        std::sort(row.begin(), row.end());
        row_off[v] = k;
        for (uint32_t w : row) {
            if (k >= gh->g.m) return fail(MCMC_E_STATE, "tiled layout holds more arcs than the graph's m");
            col_idx[k++] = w;
        }
    }
    row_off[n] = k;
    if (k != gh->g.m) return fail(MCMC_E_STATE, "tiled layout arcs != m");
    return MCMC_OK;
}

}  // namespace mcmc

using namespace mcmc;

// Counter-based G(n, p) (er_gen.h) generated straight into the tiled layout of rows [vb, ve); the
// graph handle carries no CSR.
static int er_fast_range(uint32_t n, double prob, uint64_t seed, uint32_t vb, uint32_t ve, int device,
                         mcmc_graph** out) {
    if (!out) return fail(MCMC_E_ARG, "NULL argument");
    *out = nullptr;
    if (n == 0 || vb > ve || ve > n) return fail(MCMC_E_ARG, "bad n or row range");
    if ((uint64_t)n + 65536 > 0xFFFFFFFFull) return fail(MCMC_E_ARG, "n too large");
    MCMC_HIP_TRY(hipSetDevice(device));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const uint32_t nloc = ve - vb;
    const uint32_t R = tiled_default_rows(nloc, (uint32_t)cus, kTileGenRowsMax);
    std::unique_ptr<mcmc_graph> g(new mcmc_graph());
    g->g.device = device;
    g->g.n = n;
    g->g.sorted = false;
    g->g.simple_sym = 1;   // one draw per unordered pair, both arcs, no loops (tests/test_er_generator.py)
    g->g.partial_rows = vb != 0 || ve != n;
    std::unique_ptr<TiledLayout> L(new_layout(n, vb, ve, R, er::kBlockLog2));
    const uint32_t nb = L->nblocks;
    ErArgs e{};
    e.seed = seed;
    const double p = (double)(float)prob;
    e.p_mode = p >= 1.0 ? 1 : (p <= 0.0 ? 2 : 0);
    e.inv_l1p = e.p_mode == 0 ? 1.0 / std::log1p(-p) : 0.0;
    e.n = n;
    e.vb = vb;
    e.ve = ve;
    e.nb = nb;
    hipStream_t s = nullptr;
    uint32_t* cnt = nullptr;
    unsigned long long* stats = nullptr;
    const size_t cntn = (size_t)(nb + 1) * std::max<uint32_t>(nloc, 1);
    MCMC_HIP_TRY(hipMalloc(&cnt, sizeof(uint32_t) * cntn));
    std::unique_ptr<uint32_t, void (*)(uint32_t*)> cnt_guard(cnt, [](uint32_t* p) { (void)hipFree(p); });
    MCMC_HIP_TRY(hipMalloc(&stats, 3 * sizeof(unsigned long long)));
    std::unique_ptr<unsigned long long, void (*)(unsigned long long*)> st_guard(
        stats, [](unsigned long long* p) { (void)hipFree(p); });
    const unsigned long long init[3] = {0ull, 0ull, 0xFFFFFFFFull};
    MCMC_HIP_TRY(hipMemcpy(stats, init, sizeof(init), hipMemcpyHostToDevice));
    MCMC_HIP_TRY(hipMemset(cnt, 0, sizeof(uint32_t) * cntn));
    const dim3 egrid(std::max<uint32_t>(1u, std::min<uint32_t>(4096u, (n + 255) / 256)), nb);
    if (nloc) {
        er_tiled_kernel<false><<<egrid, 256, 0, s>>>(e, cnt, nullptr, nullptr, R, nullptr);
        er_prefix_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>(4096u, (nloc + 255) / 256)), 256, 0, s>>>(
            cnt, nloc, nb, stats);
        MCMC_HIP_TRY(hipGetLastError());
        MCMC_HIP_TRY(hipStreamSynchronize(s));
    }
    int rc = layout_from_seg(*L, cnt, s);
    if (rc) return rc;
    if (nloc) {
        MCMC_HIP_TRY(hipMemset(cnt, 0, sizeof(uint32_t) * (size_t)nb * nloc));   // write cursors
        er_tiled_kernel<true><<<egrid, 256, 0, s>>>(e, cnt, L->gbase, L->tseg, R, L->tcol);
        er_pad_kernel<<<8192, 256, 0, s>>>(cnt, L->gbase, L->tseg, R, nloc, nb, L->tcol);
        MCMC_HIP_TRY(hipGetLastError());
        MCMC_HIP_TRY(hipStreamSynchronize(s));
    }
    unsigned long long h[3];
    MCMC_HIP_TRY(hipMemcpy(h, stats, sizeof(h), hipMemcpyDeviceToHost));
    L->arcs = h[0];
    g->g.m = h[0];                 // arcs of the generated rows (the whole graph for the full range)
    g->g.maxDeg = nloc ? (uint32_t)h[1] : 0;
    g->g.minDeg = nloc ? (uint32_t)h[2] : 0;
    g->tiles.push_back(std::move(L));
    *out = g.release();
    return MCMC_OK;
}

// Test hook: rows of a graph as stored on the device -- the full-range tiled layout of a generated
// graph (CSR-less), or the CSR. off: [k + 1] (off[0] = 0); ids: NULL for the degrees only, else
// cap >= off[k] entries, each row's ids in layout order; pos: optional [k], the tcol index of each
// row's first stored id (layout graphs; 0 for a CSR).
extern "C" int mcmc_graph_rows(const mcmc_graph* g, const uint32_t* rows, uint32_t k, uint64_t* off, uint32_t* ids,
                               uint64_t cap, uint64_t* pos) {
    if (!g || (k && (!rows || !off))) return fail(MCMC_E_ARG, "NULL argument");
    for (uint32_t i = 0; i < k; i++)
        if (rows[i] >= g->g.n) return fail(MCMC_E_ARG, "row out of range");
    MCMC_HIP_TRY(hipSetDevice(g->g.device));
    off[0] = 0;
    if (k == 0) return MCMC_OK;
    if (g->g.row_off) {
        std::vector<uint64_t> ro(2);
        for (uint32_t i = 0; i < k; i++) {
            MCMC_HIP_TRY(hipMemcpy(ro.data(), g->g.row_off + rows[i], 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
            off[i + 1] = off[i] + (ro[1] - ro[0]);
            if (pos) pos[i] = 0;
            if (ids) {
                if (off[i + 1] > cap) return fail(MCMC_E_ARG, "ids capacity too small");
                MCMC_HIP_TRY(hipMemcpy(ids + off[i], g->g.col_idx + ro[0], sizeof(uint32_t) * (ro[1] - ro[0]),
                                       hipMemcpyDeviceToHost));
            }
        }
        return MCMC_OK;
    }
    const TiledLayout* L = nullptr;
    for (auto& t : g->tiles)
        if (t->v_begin == 0 && t->v_end == g->g.n) L = t.get();
    if (!L) return fail(MCMC_E_STATE, "graph has neither a CSR nor a full-range tiled layout");
    uint32_t* d_rows = nullptr;
    uint64_t *d_off = nullptr, *d_deg = nullptr, *d_pos = nullptr;
    uint32_t* d_ids = nullptr;
    hipError_t e = hipMalloc(&d_rows, sizeof(uint32_t) * k);
    if (e == hipSuccess) e = hipMalloc(&d_off, sizeof(uint64_t) * (k + 1));
    if (e == hipSuccess) e = hipMalloc(&d_deg, sizeof(uint64_t) * k);
    if (e == hipSuccess) e = hipMalloc(&d_pos, sizeof(uint64_t) * k);
    if (e == hipSuccess) e = hipMemcpy(d_rows, rows, sizeof(uint32_t) * k, hipMemcpyHostToDevice);
    const uint32_t blocks = (k + 255) / 256;
    if (e == hipSuccess) {
        tile_rows_kernel<<<blocks, 256>>>(L->tcol, L->gbase, L->tseg, L->grp_rows, L->nblocks, L->block_log2, d_rows,
                                          k, nullptr, d_deg, nullptr, d_pos);
        e = hipDeviceSynchronize();
    }
    std::vector<uint64_t> deg(k);
    if (e == hipSuccess) e = hipMemcpy(deg.data(), d_deg, sizeof(uint64_t) * k, hipMemcpyDeviceToHost);
    if (e == hipSuccess && pos) e = hipMemcpy(pos, d_pos, sizeof(uint64_t) * k, hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < k; i++) off[i + 1] = off[i] + deg[i];
    if (e == hipSuccess && ids) {
        if (off[k] > cap) e = hipErrorInvalidValue;
        if (e == hipSuccess) e = hipMalloc(&d_ids, sizeof(uint32_t) * std::max<uint64_t>(off[k], 1));
        if (e == hipSuccess) e = hipMemcpy(d_off, off, sizeof(uint64_t) * (k + 1), hipMemcpyHostToDevice);
        if (e == hipSuccess) {
            tile_rows_kernel<<<blocks, 256>>>(L->tcol, L->gbase, L->tseg, L->grp_rows, L->nblocks, L->block_log2,
                                              d_rows, k, d_off, nullptr, d_ids, nullptr);
            e = hipDeviceSynchronize();
        }
        if (e == hipSuccess) e = hipMemcpy(ids, d_ids, sizeof(uint32_t) * off[k], hipMemcpyDeviceToHost);
    }
    (void)hipFree(d_rows);
    (void)hipFree(d_off);
    (void)hipFree(d_deg);
    (void)hipFree(d_pos);
    (void)hipFree(d_ids);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("graph rows: ") + hipGetErrorString(e));
    return MCMC_OK;
}

// The CSR of a generated graph (uint64 offsets, uint32 ids), built on the device from its tiled
// layout: for callers that need the reference's layout itself (the refstruct baseline at full
// occupancy, the wide sweep's slab layout and walks when nCol > 256). A row-partial graph (a rank's
// rows, mcmc_graph_er_fast_rows) gets a whole-graph offset array whose rows outside its layout are
// empty. Rows keep layout order (not sorted: above 2^31 arcs the segmented sort does not apply);
// the sweep and the layout are unaffected. Fails with the byte counts when the CSR does not fit in
// free device memory (C3: 4.0e11 B of ids beside the 2.2e11 B layout on a 288 GB device).
extern "C" int mcmc_graph_materialize_csr(mcmc_graph* g) {
    if (!g) return fail(MCMC_E_ARG, "NULL graph");
    if (g->g.row_off) return MCMC_OK;
    const TiledLayout* L = nullptr;
    for (auto& t : g->tiles)
        if (!L || t->v_end - t->v_begin > L->v_end - L->v_begin) L = t.get();
    if (!L) return fail(MCMC_E_STATE, "graph has no tiled layout");
    MCMC_HIP_TRY(hipSetDevice(g->g.device));
    const uint32_t n = g->g.n, vb = L->v_begin, nloc = L->v_end - L->v_begin;
    {
        size_t fr = 0, tot = 0;
        MCMC_HIP_TRY(hipMemGetInfo(&fr, &tot));
        const uint64_t need = 4ull * (L->arcs + 4) + 16ull * ((uint64_t)n + 1) + (64ull << 20);
        if (need > fr)
            return fail(MCMC_E_NOMEM, "materialize CSR: " + std::to_string(L->arcs) + " arcs need " +
                                          std::to_string(need) + " B of device memory, " + std::to_string(fr) +
                                          " B free (the tiled layout holds " + std::to_string(2ull * L->ids) + " B)");
    }
    uint64_t *deg = nullptr, *off = nullptr;
    uint32_t* idx = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e = hipMalloc(&deg, sizeof(uint64_t) * ((size_t)n + 1));
    if (e == hipSuccess) e = hipMalloc(&off, sizeof(uint64_t) * ((size_t)n + 1));
    if (e == hipSuccess) e = hipMemset(deg, 0, sizeof(uint64_t) * ((size_t)n + 1));
    const uint32_t blocks = (nloc + 255) / 256;
    if (e == hipSuccess && nloc) {   // local row i of the layout is vertex vb + i
        tile_rows_kernel<<<blocks, 256>>>(L->tcol, L->gbase, L->tseg, L->grp_rows, L->nblocks, L->block_log2,
                                          nullptr, nloc, nullptr, deg + vb, nullptr, nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, deg, off, n + 1);
    if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16));
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, deg, off, n + 1);
    uint64_t m = 0;
    if (e == hipSuccess) e = hipMemcpy(&m, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && (m != g->g.m || m != L->arcs)) e = hipErrorInvalidValue;
    if (e == hipSuccess) e = hipMalloc(&idx, sizeof(uint32_t) * (m + 4));
    if (e == hipSuccess) e = hipMemset(idx, 0, sizeof(uint32_t) * (m + 4));
    if (e == hipSuccess && nloc) {
        tile_rows_kernel<<<blocks, 256>>>(L->tcol, L->gbase, L->tseg, L->grp_rows, L->nblocks, L->block_log2,
                                          nullptr, nloc, off + vb, nullptr, idx, nullptr);
        e = hipDeviceSynchronize();
    }
    (void)hipFree(deg);
    (void)hipFree(tmp);
    if (e != hipSuccess) {
        (void)hipFree(off);
        (void)hipFree(idx);
        return fail(MCMC_E_HIP, std::string("materialize CSR: ") + hipGetErrorString(e));
    }
    g->g.row_off = off;
    g->g.col_idx = idx;
    g->g.sorted = false;
    return MCMC_OK;
}

extern "C" int mcmc_graph_er_fast(uint32_t n, double prob, uint64_t seed, int device, mcmc_graph** out) {
    return er_fast_range(n, prob, seed, 0, n, device, out);
}

extern "C" int mcmc_graph_er_fast_part(uint32_t n, double prob, uint64_t seed, uint32_t world, uint32_t rank,
                                       int device, mcmc_graph** out) {
    if (rank >= world) return fail(MCMC_E_ARG, "rank >= world");
    std::vector<uint32_t> b((size_t)world + 1);
    int rc = mcmc_part_plan_rows(n, world, b.data());
    if (rc) return rc;
    return er_fast_range(n, prob, seed, b[rank], b[rank + 1], device, out);
}

extern "C" int mcmc_graph_er_fast_rows(uint32_t n, double prob, uint64_t seed, uint32_t v_begin, uint32_t v_end,
                                       int device, mcmc_graph** out) {
    return er_fast_range(n, prob, seed, v_begin, v_end, device, out);
}
