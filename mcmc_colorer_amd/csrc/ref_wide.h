// mcmc_colorer_amd/csrc/ref_wide.h -- the reference-GPU-semantics sweep (--mcmcgpu-ref, SURVEY.md
// §8f row 2) for nCol > 255: uint16 colour replicas over the CSR (the reference's default colour count
// is maxDeg, main.cu:53,162, so a power-law graph runs with tens of thousands of colours). Included
// by mcmc_sweep.hip (SweepArgs, DevState, commit_control_ref).
//
// Per vertex v and sweep t (selectStarColoringBalanceDynamic, coloringMCMC_balance.cu:79-143, as
// oracle/mcmc_gpu_ref.cpp restates it):
//   conflictCounter: arcs (v, w), w > v, C[w] == C[v] (coloringMCMC_utils.cu:103-119), summed;
//   taboo'd: count down, keep the colour;
//   own colour free (< nCol): one curand_uniform, the walk q_i = hi at the own colour, eps elsewhere,
//     stopping at threshold >= u -- the binade-exact run walk of cdf_walk.h (x >= u <=> x > pred(u));
//   own colour occupied (or >= nCol): the occupancy mask (nCol bits); Zp == 0 keeps the colour with
//     no draw; otherwise reminder = sum over occupied colours, ascending, of (p[c] - eps) in fp32,
//     r = reminder / Zp and the walk q_i = eps (occupied) / p[i] + r (free), p the dynamic
//     distribution of C_t's histogram (coloringMCMC_utils.cu:64-70).
// Launches per sweep (one hipGraph node each): refw_scan_kernel (4 lanes per vertex for rows of at most
// kRefwShort arcs: count, own-colour test, the free-own-colour walk; longer rows and violators are
// listed), refw_rows_kernel<16>/<1024> (16 lanes / a workgroup per listed long / hub row), refw_walk_kernel
// <1>/<16> (a wave / a workgroup per violator: LDS mask, then the serial fp32 sums on one wave with
// chunks of 64 colours -- q >= 0 makes the partial sums monotone, so a chunk whose total stays below
// u is added without per-step tests), refw_commit_kernel (the reference's loop control).
#pragma once

constexpr uint32_t kRefwShort = 64;     // rows up to this many arcs: scanned by their own lane
constexpr uint32_t kRefwBig = 2048;     // rows / violators above this many arcs: a 1024-thread workgroup
constexpr uint32_t kRefwWalkWaves = 4;  // waves per 256-thread block of the wave-per-item kernels
constexpr int kRefwSC = 8;              // walk: chunks of 64 colours whose table loads go out together

// list sections of a.rw_lists (n entries each) and their counters a.rw_cnt[k]
enum : uint32_t { kRwViol = 0, kRwViolBig = 1, kRwLong = 2, kRwHub = 3 };

__device__ __forceinline__ float refw_p(const SweepArgs& a, const uint32_t* __restrict__ H, uint32_t c) {
    return (1.0f - ((float)H[c] / (float)a.n)) / (float)(a.nCol - 1u);   // genDynamicDistribution
}

// p of every colour from a histogram into a.ptab (the walks load it instead of dividing per colour).
__device__ __forceinline__ void refw_fill_ptab(const SweepArgs& a, const uint32_t* __restrict__ H) {
    for (uint32_t c = threadIdx.x + blockIdx.x * blockDim.x; c < a.nCol; c += blockDim.x * gridDim.x)
        a.ptab[c] = refw_p(a, H, c);
}
__global__ void refw_ptab_kernel(SweepArgs a, uint32_t parity) { refw_fill_ptab(a, a.hist + parity * a.hist_words); }

// thr + q_0 + ... + q_63 (one 64-colour chunk, lane i holds q_i >= 0, fp32 left to right) when every
// partial sum stays in thr's binade [2^e, 2^(e+1)): there the sums are multiples of U = ulp(thr), and
// adding q moves the mantissa integer k by d = round(q / U), independent of k unless q / U is a tie
// (a half-integer) -- so the chunk is an integer prefix sum across the wave. Returns false (the
// caller steps serially) for thr = 0 or subnormal, a tie, or a chunk that leaves the binade. On
// success: `total` = the sum after the chunk, `kpre` = this lane's inclusive mantissa integer.
__device__ __forceinline__ bool refw_binade_chunk(float thr, float q, float& total, uint32_t& kpre) {
    const uint32_t bt = f32_bits(thr);
    const uint32_t E = bt >> 23;
    if (!(thr >= 1.17549435e-38f) || E >= 254u) return false;
    const float dr = ldexpf(q, 150 - (int)E);   // q / U, exact (power-of-two scaling of a normal q)
    const float dn = rintf(dr);                  // round half to even
    const bool bad = !(dr < 16777216.0f) || (dr - floorf(dr) == 0.5f);
    if (__ballot(bad)) return false;
    uint32_t d = (uint32_t)dn;
    // inclusive prefix sum of d over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(d, off, 64);
        if ((threadIdx.x & 63) >= (uint32_t)off) d += y;
    }
    const uint32_t k0 = (bt & 0x7FFFFFu) | 0x800000u;
    const uint32_t kend = k0 + (uint32_t)__shfl(d, 63, 64);
    if (kend >= 0x1000000u) return false;         // leaves the binade
    kpre = k0 + d;
    total = f32_from((E << 23) | (kend & 0x7FFFFFu));
    return true;
}

// The walk q_i = (i == cv ? hi : eps), `do { thr += q_i; i++; } while (thr < u && i < nCol)`,
// star = i - 1: the first colour whose inclusive sum reaches u, nCol - 1 if none does. u in (0, 1]
// (curand_uniform), so thr >= u <=> thr > pred(u) and cdf_walk's strict walks apply; with the table
// E[k] = k eps summed in fp32 (eps_table) the sums before cv are E[k]: one load of E[cv] and, only
// when u falls below it, a binary search (walk_own_tab_e).
__device__ __forceinline__ uint32_t refw_walk_own(const float* __restrict__ E, uint32_t nCol, uint32_t cv, float eps,
                                                  float hi, float u) {
    const float up = f32_from(f32_bits(u) - 1u);
    if (cv >= nCol) {   // every q_i = eps
        if (!(eps > 0.0f)) {
            float cdf = 0.0f;
            const uint32_t s = cdf_run(cdf, eps, nCol, up);
            return s ? s - 1u : nCol - 1u;
        }
        if (!(E[nCol] > up)) return nCol - 1u;
        uint32_t lo = 1, hi_k = nCol;   // first k with E[k] > pred(u): colour k - 1
        while (lo < hi_k) {
            const uint32_t mid = (lo + hi_k) >> 1;
            if (E[mid] > up) hi_k = mid; else lo = mid + 1u;
        }
        return lo - 1u;
    }
    const uint32_t s = walk_own_tab_e(E, eps > 0.0f ? E[cv] : 0.0f, nCol, cv, eps, hi, up);
    return s < nCol ? s : nCol - 1u;
}

__device__ __forceinline__ xw::State refw_load(const uint32_t* __restrict__ X, uint32_t n, uint32_t v) {
    xw::State s;
#pragma unroll
    for (int k = 0; k < xw::kWords; k++) s.v[k] = X[(size_t)k * n + v];
    s.d = X[(size_t)xw::kWords * n + v];
    return s;
}

__device__ __forceinline__ void refw_store(uint32_t* __restrict__ Y, uint32_t n, uint32_t v, const xw::State& s) {
#pragma unroll
    for (int k = 0; k < xw::kWords; k++) Y[(size_t)k * n + v] = s.v[k];
    Y[(size_t)xw::kWords * n + v] = s.d;
}

struct RefwSweep;
__device__ __forceinline__ void refw_hist_move(const RefwSweep& w, uint32_t from, uint32_t to, uint32_t nCol);

struct RefwSweep {
    uint32_t t;
    const uint16_t* C;
    uint16_t* Cs;
    const uint32_t* X;
    uint32_t* Y;
    const uint32_t* H;   // C_t's histogram
    uint32_t* Hn;        // C_(t+1)'s, accumulated here
};

// C_(t+1)'s histogram starts as a copy of C_t's (refw_commit_kernel / mcmc_ref_init) and follows
// the vertices whose colour changed: two atomics per change instead of one per vertex (a colour
// keeps its value for all but about nCol eps of the non-violating vertices).
__device__ __forceinline__ void refw_hist_move(const RefwSweep& w, uint32_t from, uint32_t to, uint32_t nCol) {
    if (from == to) return;
    atomicSub(&w.Hn[min(from, nCol)], 1u);
    atomicAdd(&w.Hn[min(to, nCol)], 1u);
}

__device__ __forceinline__ RefwSweep refw_sweep(const SweepArgs& a, uint32_t t) {
    RefwSweep w;
    w.t = t;
    w.C = reinterpret_cast<const uint16_t*>((t & 1u) ? a.colors1 : a.colors0);
    w.Cs = reinterpret_cast<uint16_t*>((t & 1u) ? a.colors0 : a.colors1);
    w.X = (t & 1u) ? a.xw1 : a.xw0;
    w.Y = (t & 1u) ? a.xw0 : a.xw1;
    w.H = a.hist + (t & 1u) * a.hist_words;
    w.Hn = a.hist + ((t + 1u) & 1u) * a.hist_words;
    return w;
}

// Global append to list k (one returning atomic on its counter: callers with many appends batch
// them, refw_scan_kernel through LDS -- a single word takes only ~90 returning atomics per us).
__device__ __forceinline__ void refw_append_global(const SweepArgs& a, uint32_t k, uint32_t v) {
    const uint32_t i = atomicAdd(&a.rw_cnt[k], 1u);
    a.rw_lists[(size_t)k * a.n + i] = v;
}

// One vertex after its row scan (single lane): taboo'd, the free-own-colour walk, or listed as a
// violator (own colour occupied, or a colour >= nCol: its walk needs the full mask).
template <class Append>
__device__ __forceinline__ void refw_vertex(const SweepArgs& a, const RefwSweep& w, uint32_t v, uint32_t cv,
                                            bool own_occ, uint64_t deg, Append&& append) {
    const uint32_t tab = a.taboo ? a.taboo[v] : 0u;
    if (tab > 0) {
        a.taboo[v] = tab - 1u;
        refw_store(w.Y, a.n, v, refw_load(w.X, a.n, v));
        w.Cs[v] = (uint16_t)cv;   // unchanged: Hn (a copy of H) needs no update
        return;
    }
    if (cv >= a.nCol || own_occ) {
        append(deg > kRefwBig ? kRwViolBig : kRwViol, v);
        return;
    }
    xw::State s = refw_load(w.X, a.n, v);
    const float u = xw::uniform(xw::next(s));
    const uint32_t star = refw_walk_own(a.etab, a.nCol, cv, a.eps, a.ref_hi, u);
    if (a.taboo) a.taboo[v] = (star == cv) ? a.tabooIteration : 0u;
    refw_store(w.Y, a.n, v, s);
    w.Cs[v] = (uint16_t)star;
    refw_hist_move(w, cv, star, a.nCol);
}

// Four lanes per vertex: rows of at most kRefwShort arcs are scanned (four independent gathers per
// lane in flight) and finished here; longer ones are listed (a ballot per wave, one counter atomic)
// for refw_rows_kernel.
constexpr uint32_t kRefwLq = 1024;   // refw_scan_kernel: LDS entries per list before a global flush
__global__ __launch_bounds__(256) void refw_scan_kernel(SweepArgs a) {
    __shared__ uint32_t lq[4][kRefwLq];
    __shared__ uint32_t lqn[4], lqb[4];
    DevState* __restrict__ st = a.st;
    if (st->done) return;
    const RefwSweep w = refw_sweep(a, st->t);
    const int lane = threadIdx.x & 63;
    const uint32_t li = (uint32_t)lane & 3u;
    const bool lead = li == 0;
    if (threadIdx.x < 4) lqn[threadIdx.x] = 0;
    __syncthreads();
    // lists collect in LDS; one counter atomic per list and block at the end (a full buffer spills
    // to the global counter directly)
    auto append = [&](uint32_t k, uint32_t v) {
        const uint32_t i = atomicAdd(&lqn[k], 1u);
        if (i < kRefwLq) lq[k][i] = v;
        else refw_append_global(a, k, v);
    };
    unsigned long long cnt = 0;
    const uint32_t vstride = (gridDim.x * blockDim.x) >> 2;
    for (uint32_t v0 = (blockIdx.x * blockDim.x) >> 2; v0 < a.n; v0 += vstride) {   // block-uniform
        const uint32_t v = v0 + (threadIdx.x >> 2);
        const bool valid = v < a.n;
        uint64_t b0 = 0, b1 = 0;
        if (valid) {
            b0 = a.row_off[v];
            b1 = a.row_off[v + 1];
        }
        const bool longrow = valid && b1 - b0 > kRefwShort;
        if (longrow) {   // long rows: a wave each; hubs: a workgroup each
            if (lead) append(b1 - b0 > kRefwBig ? kRwHub : kRwLong, v);
            continue;
        }
        if (!valid) continue;   // uniform over the vertex's four lanes
        const uint32_t cv = w.C[v];
        uint32_t c = 0, occ = 0;
        for (uint64_t k = b0 + li; k < b1; k += 16u) {
            uint32_t x[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint64_t kj = k + 4u * (uint64_t)j;
                ok[j] = kj < b1;
                x[j] = ok[j] ? a.col_idx[kj] : v;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool same = ok[j] && w.C[x[j]] == cv;
                c += (same && x[j] > v) ? 1u : 0u;
                occ |= same ? 1u : 0u;
            }
        }
        c += __shfl_xor(c, 1, 64);
        c += __shfl_xor(c, 2, 64);
        occ |= __shfl_xor(occ, 1, 64);
        occ |= __shfl_xor(occ, 2, 64);
        if (lead) {
            cnt += c;
            refw_vertex(a, w, v, cv, occ && cv < a.nCol, b1 - b0, append);
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0 && cnt) atomicAdd(&st->viol, cnt);
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint32_t m = min(lqn[threadIdx.x], kRefwLq);
        lqb[threadIdx.x] = m ? atomicAdd(&a.rw_cnt[threadIdx.x], m) : 0u;
    }
    __syncthreads();
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t m = min(lqn[k], kRefwLq);
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) a.rw_lists[(size_t)k * a.n + lqb[k] + i] = lq[k][i];
    }
}

// T lanes per listed row (T = 16: long rows, sixteen per 256-thread block; T = 1024: hub rows, one
// per block): the count and the own-colour test over the row (four independent gathers per lane in
// flight), then the vertex.
template <uint32_t T>
__global__ __launch_bounds__(T <= 64 ? 256 : T) void refw_rows_kernel(SweepArgs a, uint32_t which) {
    constexpr uint32_t NW = T > 64 ? T / 64 : 1;   // waves per row
    __shared__ unsigned long long red_c[NW], blk_c;
    __shared__ uint32_t red_o[NW];
    __shared__ uint32_t lq[2][kRefwLq], lqn[2], lqb[2];
    DevState* __restrict__ st = a.st;
    if (st->done) return;
    if (threadIdx.x < 2) lqn[threadIdx.x] = 0;
    if (threadIdx.x == 0) blk_c = 0;
    __syncthreads();
    // the block's violators and conflicting arcs: LDS first, one global atomic each at the end
    auto append = [&](uint32_t k, uint32_t v) {
        const uint32_t i = atomicAdd(&lqn[k], 1u);
        if (i < kRefwLq) lq[k][i] = v;
        else refw_append_global(a, k, v);
    };
    const RefwSweep w = refw_sweep(a, st->t);
    const int lane = threadIdx.x & 63;
    const uint32_t G = blockDim.x / T;                              // rows per block at a time
    const uint32_t grp = threadIdx.x / T, tid = threadIdx.x % T, wv = tid >> 6;
    const uint32_t count = a.rw_cnt[which];
    const uint32_t* list = a.rw_lists + (size_t)which * a.n;
    for (uint32_t i0 = blockIdx.x * G; i0 < count; i0 += gridDim.x * G) {   // block-uniform
        const uint32_t i = i0 + grp;
        const bool act = i < count;
        const uint32_t v = act ? list[i] : 0u;
        uint64_t b0 = 0, b1 = 0;
        if (act) {
            b0 = a.row_off[v];
            b1 = a.row_off[v + 1];
        }
        const uint32_t cv = act ? w.C[v] : 0u;
        unsigned long long c = 0;
        uint32_t occ = 0;
        for (uint64_t k = b0 + tid; k < b1; k += 4u * T) {
            uint32_t x[4];
            bool ok[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint64_t kj = k + (uint64_t)j * T;
                ok[j] = kj < b1;
                x[j] = ok[j] ? a.col_idx[kj] : v;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool same = ok[j] && w.C[x[j]] == cv;
                c += (same && x[j] > v) ? 1u : 0u;
                occ |= same ? 1u : 0u;
            }
        }
        for (uint32_t off = 1; off < (T < 64 ? T : 64u); off <<= 1) {   // within the row's lanes
            c += __shfl_xor(c, (int)off, 64);
            occ |= __shfl_xor(occ, (int)off, 64);
        }
        if (NW > 1) {
            if (lane == 0) {
                red_c[wv] = c;
                red_o[wv] = occ;
            }
            __syncthreads();
            if (tid == 0)
                for (uint32_t k = 1; k < NW; k++) {
                    c += red_c[k];
                    occ |= red_o[k];
                }
        }
        if (act && tid == 0) {
            if (c) atomicAdd(&blk_c, c);
            refw_vertex(a, w, v, cv, occ && cv < a.nCol, b1 - b0, append);
        }
        if (NW > 1) __syncthreads();
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const uint32_t m = min(lqn[threadIdx.x], kRefwLq);
        lqb[threadIdx.x] = m ? atomicAdd(&a.rw_cnt[threadIdx.x], m) : 0u;   // kRwViol, kRwViolBig
    }
    if (threadIdx.x == 0 && blk_c) atomicAdd(&st->viol, blk_c);
    __syncthreads();
    for (uint32_t k = 0; k < 2; k++) {
        const uint32_t m = min(lqn[k], kRefwLq);
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) a.rw_lists[(size_t)k * a.n + lqb[k] + i] = lq[k][i];
    }
}

// W waves per violator: the occupancy mask of its row in LDS (all W waves gather), then wave 0 runs
// Zp, the draw, the reminder and the walk (fp32, ascending, exactly the reference's order).
template <int W>
__global__ __launch_bounds__(W == 1 ? 256 : 1024) void refw_walk_kernel(SweepArgs a, uint32_t which) {
    extern __shared__ uint32_t refw_lds[];
    __shared__ uint32_t red_z[W];
    DevState* __restrict__ st = a.st;
    if (st->done) return;
    const RefwSweep w = refw_sweep(a, st->t);
    const int lane = threadIdx.x & 63;
    const uint32_t T = 64u * W, G = blockDim.x / T;
    const uint32_t grp = threadIdx.x / T, tid = threadIdx.x % T, wv = tid >> 6;
    const uint32_t nCol = a.nCol, words = (nCol + 31u) >> 5, wstride = (words + 3u) & ~3u;
    uint32_t* mask = refw_lds + grp * wstride;
    const uint32_t count = a.rw_cnt[which];
    const uint32_t* list = a.rw_lists + (size_t)which * a.n;
    auto sync = [&]() {
        if (W > 1) {
            __syncthreads();
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    };
    for (uint32_t i0 = blockIdx.x * G; i0 < count; i0 += gridDim.x * G) {   // block-uniform
        const uint32_t i = i0 + grp;
        const bool act = i < count;   // wave-uniform (T >= 64)
        const uint32_t v = act ? list[i] : 0u;
        for (uint32_t k = tid; k < words; k += T) mask[k] = 0;
        sync();
        if (act) {
            const uint64_t b0 = a.row_off[v], b1 = a.row_off[v + 1];
            for (uint64_t k = b0 + tid; k < b1; k += 4u * T) {   // four independent gathers in flight
                uint32_t x[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint64_t kj = k + (uint64_t)j * T;
                    x[j] = kj < b1 ? a.col_idx[kj] : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t c = x[j] != 0xFFFFFFFFu ? (uint32_t)w.C[x[j]] : nCol;
                    if (c < nCol) atomicOr(&mask[c >> 5], 1u << (c & 31));
                }
            }
        }
        sync();
        uint32_t zn = 0;
        for (uint32_t k = tid; k < words; k += T) zn += __popc(mask[k]);
        for (int off = 32; off > 0; off >>= 1) zn += __shfl_xor(zn, off, 64);
        if (W > 1) {
            if (lane == 0) red_z[wv] = zn;
            __syncthreads();
            zn = 0;
            for (int k = 0; k < W; k++) zn += red_z[k];
        }
        if (act && wv == 0) {   // one wave: uniform values, serial sums by readlane
            const uint32_t cv = w.C[v];
            const uint32_t Zp = nCol - zn;
            xw::State s = refw_load(w.X, a.n, v);
            uint32_t star = cv;
            if (Zp != 0) {
                const float u = xw::uniform(xw::next(s));
                const bool own = cv < nCol && ((mask[cv >> 5] >> (cv & 31)) & 1u);
                if (own) {
                    auto occ = [&](uint32_t c) -> bool { return c < nCol && ((mask[c >> 5] >> (c & 31)) & 1u); };
                    // reminder: occupied colours ascending; kRefwSC chunks of 64 per round, their table
                    // loads all in flight before the serial adds
                    float rem = 0.0f;
                    for (uint32_t c0 = 0; c0 < nCol; c0 += 64u * kRefwSC) {
                        // the super-chunk's 2 kRefwSC mask words: nothing occupied, nothing to add
                        const uint32_t wi = (c0 >> 5) + (uint32_t)lane;
                        if (__ballot(lane < 2 * kRefwSC && wi < words && mask[wi] != 0u) == 0ull) continue;
                        float val[kRefwSC];
                        uint64_t om[kRefwSC];
#pragma unroll
                        for (int j = 0; j < kRefwSC; j++) {
                            const uint32_t c = c0 + 64u * j + (uint32_t)lane;
                            const bool o = occ(c);
                            om[j] = __ballot(o);
                            val[j] = o ? (a.ptab[c] - a.eps) : 0.0f;
                        }
#pragma unroll
                        for (int j = 0; j < kRefwSC; j++) {
                            uint64_t m = om[j];
                            while (m) {
                                const int k = __builtin_ctzll(m);
                                m &= m - 1ull;
                                rem += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(val[j]), k));
                            }
                        }
                    }
                    const float r = rem / (float)Zp;
                    float thr = 0.0f;
                    star = nCol - 1u;
                    bool hit = false;
                    // one chunk of 64 colours from cb (lanes past nCol hold +0.0f: no effect on thr >= 0,
                    // and no stop can fall there)
                    auto chunk = [&](float q, uint32_t cb) {
                        float e;
                        uint32_t kp;
                        if (refw_binade_chunk(thr, q, e, kp)) {
                            if (e < u) {
                                thr = e;
                                return;
                            }
                            // u in thr's binade (e < 2^(e+1) <= any u of a higher one): the first
                            // colour whose mantissa integer reaches u's
                            const uint32_t T = (f32_bits(u) & 0x7FFFFFu) | 0x800000u;
                            const uint64_t hb = __ballot(kp >= T);
                            const int k = __builtin_ctzll(hb);
                            star = cb + (uint32_t)k;
                            hit = true;
                            return;
                        }
                        if (__ballot(!(q >= 0.0f)) == 0ull) {   // partial sums monotone: the total first
                            float t2 = thr;
#pragma unroll
                            for (int k = 0; k < 64; k++) t2 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q), k));
                            if (t2 < u) {
                                thr = t2;
                                return;
                            }
                        }
                        for (int k = 0; k < 64; k++) {
                            thr += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q), k));
                            if (thr >= u && cb + (uint32_t)k < nCol) {
                                star = cb + (uint32_t)k;
                                hit = true;
                                return;
                            }
                        }
                    };
                    auto load_q = [&](uint32_t c0, float (&q)[kRefwSC]) {
#pragma unroll
                        for (int j = 0; j < kRefwSC; j++) {
                            const uint32_t c = c0 + 64u * j + (uint32_t)lane;
                            q[j] = c < nCol ? (occ(c) ? a.eps : (a.ptab[c] + r)) : 0.0f;
                        }
                    };
                    // super-chunks of kRefwSC x 64 colours, the next one's table loads in flight while
                    // this one is summed
                    float qa[kRefwSC], qb[kRefwSC];
                    load_q(0, qa);
                    for (uint32_t c0 = 0; c0 < nCol && !hit; c0 += 2u * 64u * kRefwSC) {
                        if (c0 + 64u * kRefwSC < nCol) load_q(c0 + 64u * kRefwSC, qb);
#pragma unroll
                        for (int j = 0; j < kRefwSC; j++)
                            if (!hit) chunk(qa[j], c0 + 64u * j);
                        if (hit || c0 + 64u * kRefwSC >= nCol) break;
                        if (c0 + 2u * 64u * kRefwSC < nCol) load_q(c0 + 2u * 64u * kRefwSC, qa);
#pragma unroll
                        for (int j = 0; j < kRefwSC; j++)
                            if (!hit) chunk(qb[j], c0 + 64u * kRefwSC + 64u * j);
                    }
                } else {
                    star = refw_walk_own(a.etab, nCol, cv, a.eps, a.ref_hi, u);
                }
                if (lane == 0 && a.taboo) a.taboo[v] = (star == cv) ? a.tabooIteration : 0u;
            }
            if (lane == 0) {
                refw_store(w.Y, a.n, v, s);
                w.Cs[v] = (uint16_t)star;
                refw_hist_move(w, cv, star, nCol);
            }
        }
        sync();   // the mask is cleared for the next violator
    }
}

// The loop control of the reference's run() (commit_control_ref) on the sweep's conflicting-arc count;
// the lists are emptied for the next sweep.
__global__ __launch_bounds__(1024) void refw_commit_kernel(SweepArgs a) {
    __shared__ uint32_t sh_done, sh_t;
    __shared__ unsigned long long sh_c;
    DevState* st = a.st;
    if (threadIdx.x == 0) {
        sh_done = st->done;
        sh_t = st->t;
        sh_c = st->viol;
    }
    __syncthreads();
    if (sh_done) return;
    if (threadIdx.x == 0) st->viol = 0;
    if (threadIdx.x < 4) a.rw_cnt[threadIdx.x] = 0;
    // p of sweep t + 1 from C_(t+1)'s histogram (read by nothing else now; used only if the loop goes
    // on), and that histogram copied into the buffer sweep t + 1 adjusts (refw_hist_move)
    const uint32_t* Hn = a.hist + ((sh_t + 1u) & 1u) * a.hist_words;
    refw_fill_ptab(a, Hn);
    commit_control_ref(a, sh_t, sh_c, Hn);
}

// Initial colouring (initColoring, coloringMCMC_utils.cu:24-33) into uint16 replicas, and C_0's
// histogram (nCol + 1 bins: a colour may equal nCol).
__global__ void refw_init_kernel(uint16_t* __restrict__ C, uint32_t* __restrict__ X, uint32_t n, uint32_t nCol,
                                 uint32_t* __restrict__ hist) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        xw::State s = refw_load(X, n, v);
        const uint32_t c = (uint32_t)(int)(xw::uniform(xw::next(s)) * (float)nCol);
        C[v] = (uint16_t)c;
        refw_store(X, n, v, s);
        atomicAdd(&hist[min(c, nCol)], 1u);
    }
}
