// mcmc_colorer_amd/csrc/dense_counts.h -- the dense-count sweep (tiled contexts, nCol <= 256).
// Included by mcmc_sweep.hip inside namespace mcmc, after the tiled sweep (evaluate_lane,
// sweep_tail, the tiled layout helpers).
//
// Everything loop 1 of run() takes from a row is its occupancy mask -- count_free_colors
// (coloringMCMC_CPU.cpp:361-383) is nCol minus its popcount, violation_count (:329-351) is "own
// colour in the mask", fill_p (:392-481) depends on nothing else. The mask is an OR over all
// neighbours, so once the neighbours inside ANY fixed column range cover every colour it is the
// full mask, whatever the other neighbours hold. Each context fixes a dense column range
// S = [dc_s0, dc_s1) inside its own rows, sized so that a row's expected neighbours in S number
// nCol (ln nCol + 10) (a row misses a colour there with probability ~nCol e^-(ln nCol + 10)), and
// keeps per local row w
//     cnt[w][c] = #{u in S : (w, u) an arc, C_t[u] = c}    (uint32)
// and the occupancy bits of those counts (dense mask). A sweep is then two launches:
//   dc_update_kernel  moves the counts by the vertices of S whose colour the previous sweep changed
//                     (u's old colour -1, new colour +1 in every row holding u; a count crossing 0
//                     flips its mask bit). For a simple symmetric graph the rows holding u are u's
//                     own neighbours, and row u is a local row (S lies inside the context's rows),
//                     so the tiled layout lists them. The first sweep after a colouring is set, or
//                     one after more changes than pay, rebuilds every count from the layout.
//   dc_eval_kernel    lane per row: a full dense mask is the row's mask and the row is evaluated at
//                     once; a row whose dense mask is not full first scans its other
//                     column blocks (the wave together, colours from the replica, stopping once the
//                     mask is full). evaluate_lane lists the vertices of S that change colour for
//                     the next update; the last workgroup commits (sweep_tail), and the commit's
//                     glibc replay lists the overflow events of S (commit_accept, dc_commit).
// Exact, not approximate: the counts are integers and the mask is the set the full scan ORs
// together (tests/test_dense.py: every variant against the early-exit scan and the oracle).
// Reference counterpart: the per-sweep neighbour scans of ColoringMCMC_CPU::run (:136-270).

__device__ __forceinline__ void dc_lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Real ids [s0, s1) (padding excluded) of local row l's segment in column block b, relative to gc.
__device__ __forceinline__ void dc_segment(const SweepArgs& a, uint32_t l, uint32_t b, uint32_t& s0, uint32_t& s1,
                                           const uint16_t*& gc) {
    const uint32_t R = a.grp_rows, g = l / R, r = l - g * R;
    const uint32_t* ts = a.tseg + ((size_t)g * a.nblocks + b) * tseg_stride(R);
    const uint32_t raw = ts[r];
    s0 = raw & kTsegPos;
    s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
    gc = a.tcol + a.gbase[g];
}

// Vertex u of S moved from colour ca to cb: row lw's counts and dense mask.
template <int NW>
__device__ __forceinline__ void dc_move(const SweepArgs& a, uint32_t lw, uint32_t ca, uint32_t cb) {
    uint32_t* cw = a.dc_cnt + (size_t)lw * a.dc_cw;
    uint32_t* mw = a.dc_mask + (size_t)lw * NW;
    const uint32_t oa = atomicSub(&cw[ca], 1u);   // >= 1: u itself holds colour ca
    const uint32_t ob = atomicAdd(&cw[cb], 1u);
    // a count crossing zero flips its bit; crossings of one count alternate in the order of its
    // atomics, so the flips leave the bit = (count > 0) whatever the interleaving
    if (oa == 1u) atomicXor(&mw[ca >> 5], 1u << (ca & 31u));
    if (ob == 0u) atomicXor(&mw[cb >> 5], 1u << (cb & 31u));
}

// Sweep t's update of the dense counts (all waves; grid-stride). Rebuild: a wave per local row,
// its segments in the blocks overlapping S, colours of C_t counted in an LDS histogram. Incremental:
// a wave per (listed vertex u, column block b of the local rows): u's neighbours in block b.
template <int NW>
__global__ __launch_bounds__(256) void dc_update_kernel(SweepArgs a) {
    __shared__ uint32_t hist[4][256];
    const DevState* st = a.st;
    if (st->done) return;
    const uint32_t t = st->t;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;   // C_t
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwv = (gridDim.x * blockDim.x) >> 6;
    const uint32_t bl = a.block_log2;
    if (a.dc_ctl[kDcMode]) {
        uint32_t* h = hist[threadIdx.x >> 6];
        const uint32_t b0 = a.dc_s0 >> bl, b1 = (a.dc_s1 - 1u) >> bl, sw = a.dc_s1 - a.dc_s0;
        for (uint32_t l = wave; l < nloc; l += nwv) {
            for (uint32_t i = lane; i < a.dc_cw; i += 64u) h[i] = 0;
            dc_lds_wait();
            for (uint32_t b = b0; b <= b1; b++) {
                uint32_t s0, s1;
                const uint16_t* gc;
                dc_segment(a, l, b, s0, s1, gc);
                const uint32_t base = b << bl;
                for (uint32_t k = s0 + lane; k < s1; k += 64u) {
                    const uint32_t u = base | (uint32_t)gc[k];
                    if (u - a.dc_s0 < sw) atomicAdd(&h[C[u]], 1u);
                }
            }
            dc_lds_wait();
            uint32_t* cr = a.dc_cnt + (size_t)l * a.dc_cw;
            for (uint32_t i = lane; i < a.dc_cw; i += 64u) cr[i] = h[i];
            uint32_t* mk = a.dc_mask + (size_t)l * NW;
            for (uint32_t c0 = 0; c0 < 32u * NW; c0 += 64u) {
                const uint32_t c = c0 + lane;
                const uint64_t bm = __ballot(c < a.nCol && h[c] != 0u);
                if (lane == 0) {
                    mk[c0 >> 5] = (uint32_t)bm;
                    if ((c0 >> 5) + 1u < (uint32_t)NW) mk[(c0 >> 5) + 1u] = (uint32_t)(bm >> 32);
                }
            }
            dc_lds_wait();   // every lane's reads of h are done before the next row clears it
        }
        return;
    }
    const uint32_t p = t & 1u;
    const uint32_t len = min(a.dc_ctl[kDcLen + p], a.dc_cap);
    if (len == 0) return;
    const uint8_t* __restrict__ P = (t & 1) ? a.colors0 : a.colors1;   // C_t-1 (sweep t overwrites it later)
    const uint32_t* __restrict__ L = a.dc_list + (size_t)p * a.dc_cap;
    const uint32_t bl0 = a.v_begin >> bl, nbl = ((a.v_end - 1u) >> bl) - bl0 + 1u;
    const uint64_t tasks = (uint64_t)len * nbl;
    for (uint64_t task = wave; task < tasks; task += nwv) {
        const uint32_t i = (uint32_t)(task / nbl), b = bl0 + (uint32_t)(task - (uint64_t)i * nbl);
        const uint32_t u = L[i];
        const uint32_t ca = P[u], cb = C[u];
        if (ca == cb) continue;
        uint32_t s0, s1;
        const uint16_t* gc;
        dc_segment(a, u - a.v_begin, b, s0, s1, gc);
        const uint32_t base = b << bl;
        for (uint32_t k = s0 + lane; k < s1; k += 64u) {
            const uint32_t lw = (base | (uint32_t)gc[k]) - a.v_begin;
            if (lw < nloc) dc_move<NW>(a, lw, ca, cb);
        }
    }
}

// Rows of this wave whose dense mask is not full (`open`): each in turn, the whole wave scans its
// segments in the column blocks not inside S (colours of C_t from the replica), OR-ing into its
// mask until it is full or the blocks run out; lane j's mask comes back full. Out of line (rare:
// C3 ~0.005 % of rows) and with everything passed by value -- a reference to the kernel's
// SweepArgs would copy the whole struct to scratch in every lane.
template <int NW>
struct DcMask {
    uint32_t w[NW];
};
struct DcScan {
    const uint32_t* tseg;
    const uint64_t* gbase;
    const uint16_t* tcol;
    uint32_t R, nb, bl, s0, s1;
};
template <int NW>
__device__ __noinline__ DcMask<NW> dc_open_scan(DcScan d, const uint8_t* __restrict__ C, uint32_t l, bool open,
                                                DcMask<NW> acc, DcMask<NW> fullw, int lane) {
    uint64_t pend = __ballot(open);
    while (pend) {
        const int j = __ffsll((long long)pend) - 1;
        pend &= pend - 1ull;
        const uint32_t lj = __shfl(l, j, 64);
        const uint32_t g = lj / d.R, r = lj - g * d.R;
        const uint16_t* __restrict__ gc = d.tcol + d.gbase[g];
        uint32_t cur[NW];
#pragma unroll
        for (int i = 0; i < NW; i++) cur[i] = __shfl(acc.w[i], j, 64);
        for (uint32_t b = 0; b < d.nb; b++) {
            const uint32_t lo = b << d.bl;
            if (lo >= d.s0 && lo + (1u << d.bl) <= d.s1) continue;   // inside S: in the counts
            const uint32_t* ts = d.tseg + ((size_t)g * d.nb + b) * tseg_stride(d.R);
            const uint32_t raw = ts[r];
            const uint32_t s0 = raw & kTsegPos, s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
            uint32_t m[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) m[i] = 0;
            for (uint32_t k = s0 + (uint32_t)lane; k < s1; k += 64u) set_color_bit<NW>(m, C[lo | (uint32_t)gc[k]]);
            bool full = true;
#pragma unroll
            for (int i = 0; i < NW; i++) {
                cur[i] |= wave_or_uniform(m[i]);
                full = full && ((cur[i] & fullw.w[i]) == fullw.w[i]);
            }
            if (full) break;
        }
        if (lane == j) {
#pragma unroll
            for (int i = 0; i < NW; i++) acc.w[i] = cur[i];
        }
    }
    return acc;
}

// Sweep t's evaluation: persistent, one 1024-thread workgroup per CU; wave w of the grid takes the
// 64-row tiles w, w + W, w + 2 W, ... (W = all waves), kDcTiles of them per step, the next step's
// loads in flight while this step is evaluated; lane per row. A full mask holds the row's own colour
// and no free colour -- fill_p's case (i) -- so with the closed-form walk (SweepArgs::ewalk) a row
// keeps its colour exactly when u in [E[cv], S[cv]) (evaluate_lane's shortcut); a tile whose valid
// rows all do is written directly (C_t+1 = C_t, Cviol, taboo reset), any other takes evaluate_lane. u_v of row l is x_t 16807^(v_begin + l + 1): 16807^(64 W) (a.dc_apow) steps a tile's power to
// the next tile of the wave.
constexpr int kDcTiles = 4;
template <int NW>
__global__ __launch_bounds__(1024) void dc_eval_kernel(SweepArgs a) {
    extern __shared__ uint4 dc_lds[];
    __shared__ TailShared sh;
    __shared__ float2 ewl[256];
    DevState* __restrict__ st = a.st;
    if (a.check_done && st->done) return;
    if (threadIdx.x == 0) {
        sh.wg_viol = 0;
        sh.wg_ev = 0;
        sh.viol = 0;
    }
    const uint32_t t = st->t;
    const uint32_t x_t = st->x_t;
    const uint32_t err0 = st->err;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;
    uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;
    const uint32_t nloc = a.v_end - a.v_begin;
    uint8_t* const vf = a.vflags ? a.vflags + (size_t)(t & 1u) * nloc : nullptr;
    const float2* ew = nullptr;
    if (a.ewalk) {
        for (uint32_t i = threadIdx.x; i < a.nCol; i += blockDim.x) ewl[i] = a.ewalk[i];
        ew = ewl;
    }
    uint32_t fullw[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint32_t lo = 32u * i;
        fullw[i] = a.nCol >= lo + 32u ? ~0u : (a.nCol > lo ? (1u << (a.nCol - lo)) - 1u : 0u);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t nwaves = blockDim.x >> 6;
    const uint32_t gw = blockIdx.x * nwaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), GW = gridDim.x * nwaves;
    const uint32_t ntiles = (nloc + 63u) >> 6;
    uint32_t wave_viol = 0, wave_ev = 0, wave_open = 0;
    const uint32_t lpow = kMinstdLanePow[lane];
    uint32_t apk[kDcTiles];   // 16807^(64 W k)
    apk[0] = 1u;
#pragma unroll
    for (int k = 1; k < kDcTiles; k++) apk[k] = minstd_mulmod(apk[k - 1], a.dc_apow);
    const uint32_t astep = minstd_mulmod(apk[kDcTiles - 1], a.dc_apow);
    uint32_t xb = gw < ntiles ? minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)a.v_begin + 64ull * gw + 1ull)) : 0u;
    xb = __builtin_amdgcn_readfirstlane(xb);   // wave-uniform: the tile powers run on the scalar unit
    // Steps over ping-pong register sets: step s + 1's loads are in flight while step s is evaluated.
    // The step's open rows are scanned BEFORE the next loads are issued, and evaluation has no early
    // exit (a tile past the wave's end evaluates nothing): hipcc's wait counting drains every load
    // after an out-of-line call or on a path that skips a set's uses, so neither may sit between a
    // set's loads and their use. Loads past the end read nothing (exec-masked).
#define DC_LOAD(ACC, CV, TAB, T0)                                                                   \
    _Pragma("unroll") for (int k = 0; k < kDcTiles; k++) {                                          \
        const uint32_t l = 64u * ((T0) + k * GW) + (uint32_t)lane;                                  \
        const bool valid = (T0) < ntiles && l < nloc;                                               \
        _Pragma("unroll") for (int i = 0; i < NW; i++) ACC[k][i] = valid ? a.dc_mask[(size_t)l * NW + i] : 0u; \
        CV[k] = valid ? (uint32_t)C[a.v_begin + l] : 0u;                                            \
        TAB[k] = (a.taboo != nullptr && valid) ? a.taboo[l] : 0u;                                   \
    }
#define DC_OPEN(ACC, T0)                                                                            \
    {                                                                                               \
        bool anyo = false;                                                                          \
        _Pragma("unroll") for (int k = 0; k < kDcTiles; k++) {                                      \
            const uint32_t l = 64u * ((T0) + k * GW) + (uint32_t)lane;                              \
            bool full = true;                                                                       \
            _Pragma("unroll") for (int i = 0; i < NW; i++) full = full && ((ACC[k][i] & fullw[i]) == fullw[i]); \
            anyo = anyo || (l < nloc && !full);                                                     \
        }                                                                                           \
        if (__ballot(anyo)) {                                                                       \
            for (int k = 0; k < kDcTiles; k++) {                                                    \
                const uint32_t l = 64u * ((T0) + k * GW) + (uint32_t)lane;                          \
                bool full = true;                                                                   \
                for (int i = 0; i < NW; i++) full = full && ((ACC[k][i] & fullw[i]) == fullw[i]);   \
                const bool open = l < nloc && !full;                                                \
                const uint64_t ob = __ballot(open);                                                 \
                if (!ob) continue;                                                                  \
                wave_open += (uint32_t)__popcll(ob);                                                \
                DcMask<NW> m, fw;                                                                   \
                for (int i = 0; i < NW; i++) {                                                      \
                    m.w[i] = ACC[k][i];                                                             \
                    fw.w[i] = fullw[i];                                                             \
                }                                                                                   \
                const DcScan ds{a.tseg, a.gbase, a.tcol, a.grp_rows, a.nblocks, a.block_log2, a.dc_s0, a.dc_s1}; \
                m = dc_open_scan<NW>(ds, C, l, open, m, fw, lane);                                  \
                for (int i = 0; i < NW; i++) ACC[k][i] = m.w[i];                                    \
            }                                                                                       \
        }                                                                                           \
    }
#define DC_EVAL(ACC, CV, TAB, T0)                                                                   \
    _Pragma("unroll") for (int k = 0; k < kDcTiles; k++) {                                          \
        const uint32_t l = 64u * ((T0) + k * GW) + (uint32_t)lane;                                  \
        const bool valid = l < nloc;                                                                \
        const uint32_t x = minstd_mulmod(minstd_mulmod(xb, apk[k]), lpow);                          \
        bool keep = false;                                                                          \
        if (ew != nullptr) {                                                                        \
            bool full = true;                                                                       \
            _Pragma("unroll") for (int i = 0; i < NW; i++) full = full && ((ACC[k][i] & fullw[i]) == fullw[i]); \
            const float u = minstd_canonical(x);                                                    \
            const float2 es = ew[CV[k]];                                                            \
            keep = full && TAB[k] == 0u && u >= es.x && es.y > u;                                   \
        }                                                                                           \
        const uint64_t vb = __ballot(valid);                                                        \
        if (!__ballot(valid && !keep)) {                                                            \
            if (valid) {                                                                            \
                Cs[a.v_begin + l] = (uint8_t)CV[k];                                                 \
                if (vf != nullptr) vf[l] = 1u;                                                      \
                if (a.taboo != nullptr) a.taboo[l] = a.tabooIteration;                              \
            }                                                                                       \
            wave_viol += (uint32_t)__popcll(vb);                                                    \
        } else {                                                                                    \
            wave_viol += evaluate_lane<NW>(a, st, Cs, valid, l, ACC[k], lane, wave_ev, vf, CV[k], TAB[k], x, ew); \
        }                                                                                           \
    }                                                                                               \
    xb = minstd_mulmod(xb, astep);
    uint32_t accA[kDcTiles][NW], cvA[kDcTiles], tabA[kDcTiles];
    uint32_t accB[kDcTiles][NW], cvB[kDcTiles], tabB[kDcTiles];
    uint32_t tau0 = gw;
    const uint32_t stride = kDcTiles * GW;
    DC_LOAD(accA, cvA, tabA, tau0)
    while (tau0 < ntiles) {
        DC_OPEN(accA, tau0)
        DC_LOAD(accB, cvB, tabB, tau0 + stride)
        DC_EVAL(accA, cvA, tabA, tau0)
        tau0 += stride;
        if (tau0 >= ntiles) break;
        DC_OPEN(accB, tau0)
        DC_LOAD(accA, cvA, tabA, tau0 + stride)
        DC_EVAL(accB, cvB, tabB, tau0)
        tau0 += stride;
    }
#undef DC_LOAD
#undef DC_OPEN
#undef DC_EVAL
    if (wave_open) {   // statistics; the commit reads the word (this workgroup releases)
        if (lane == 0) atomicAdd(&a.dc_ctl[kDcOpen], wave_open);
        wave_ev = 1u;
    }
    __syncthreads();   // ewl's last readers are done before the commit may reuse LDS (it uses dc_lds)
    sweep_tail(a, st, sh, wave_viol, wave_ev, lane, reinterpret_cast<uint32_t*>(dc_lds), a.lds_sort_cap, t, err0);
}

template <int NW>
void launch_dc(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    dc_update_kernel<NW><<<g.x * 8u, 256, 0, s>>>(a);
    dc_eval_kernel<NW><<<g, b, lds, s>>>(a);
}
template <int NW>
hipError_t allow_lds_dc(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&dc_eval_kernel<NW>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
