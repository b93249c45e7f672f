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
// and the occupancy bits of those counts (dense mask), plus one "open" bit per row and mask word
// (that word of the dense mask is not full). A sweep is one launch, dc_eval_kernel, in two phases:
//   update            (dc_update_tasks) brings the buffer the sweep writes (it holds C_t-1) to C_t
//                     on the local rows (the previous sweep's restore list of changed rows, or a
//                     full copy), then moves the counts by the vertices of S whose colour the
//                     previous sweep changed (u's old colour -1, new colour +1 in every row holding
//                     u; a count crossing 0 flips its mask bit and, when the word's fullness
//                     changed, its open bit). For a simple symmetric graph the rows holding u are
//                     u's own neighbours, and row u is a local row (S lies inside the context's
//                     rows), so the tiled layout lists them. The first sweep after a colouring is
//                     set, or one after more changes than pay, rebuilds every count from the layout.
//   evaluation        lane per row, reading the row's colour and its tile's open words: a row that
//                     is not open has the full mask and is evaluated at once; an open row first
//                     scans its other column blocks (the wave together, colours from the replica,
//                     stopping once the mask is full). Only rows that change colour are written
//                     (both lists take them); the last workgroup commits (sweep_tail), and the
//                     commit's glibc replay lists the overflow events (commit_accept,
//                     dc_list_change, dc_commit).
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

// Word i of a full mask (colours [32 i, 32 i + 32) below nCol).
__device__ __forceinline__ uint32_t dc_fullw(uint32_t nCol, uint32_t i) {
    const uint32_t lo = 32u * i;
    return nCol >= lo + 32u ? ~0u : (nCol > lo ? (1u << (nCol - lo)) - 1u : 0u);
}

// Open word wi (= (row >> 6) NW + mask word) went from o to n: when that crossed zero, flip its
// summary bit and move the count of nonzero open words (dc_osum). Every change of an open word is
// an atomic returning the old value, so the crossings of one word alternate in the order of its
// atomics: the summary bit ends as (word != 0) and the count as the number of such words,
// whatever the interleaving (both start consistent: all zero with the open words, setup_dense).
__device__ __forceinline__ void dc_osum_note(const SweepArgs& a, size_t wi, unsigned long long o, unsigned long long n) {
    if (a.dc_osum == nullptr || ((o == 0ull) == (n == 0ull))) return;
    atomicXor(&a.dc_osum[1 + (wi >> 6)], 1ull << (wi & 63u));
    atomicAdd(reinterpret_cast<uint32_t*>(a.dc_osum), o == 0ull ? 1u : 0xFFFFFFFFu);
}

// Row lw's count of colour c crossed zero: flip its mask bit, and its open bit when that changed
// whether mask word c / 32 is full. Flips of one word are ordered by its atomics, so the open bit
// ends as (word not full) whatever the interleaving.
template <int NW>
__device__ __forceinline__ void dc_flip(const SweepArgs& a, uint32_t lw, uint32_t c) {
    const uint32_t i = c >> 5, bit = 1u << (c & 31u), fw = dc_fullw(a.nCol, i);
    const uint32_t o = atomicXor(&a.dc_mask[(size_t)lw * NW + i], bit);
    if (((o & fw) == fw) != (((o ^ bit) & fw) == fw)) {
        const size_t wi = (size_t)(lw >> 6) * NW + i;
        const unsigned long long ob = 1ull << (lw & 63u);
        const unsigned long long oo = atomicXor(&a.dc_open[wi], ob);
        dc_osum_note(a, wi, oo, oo ^ ob);
    }
}

// Vertex u of S moved from colour ca to cb: row lw's counts, dense mask and open bits.
template <int NW>
__device__ __forceinline__ void dc_move(const SweepArgs& a, uint32_t lw, uint32_t ca, uint32_t cb) {
    uint32_t* cw = a.dc_cnt + (size_t)lw * a.dc_cw;
    const uint32_t oa = atomicSub(&cw[ca], 1u);   // >= 1: u itself holds colour ca
    const uint32_t ob = atomicAdd(&cw[cb], 1u);
    if (oa == 1u) dc_flip<NW>(a, lw, ca);
    if (ob == 0u) dc_flip<NW>(a, lw, cb);
}

// Sweep t's update, at the start of the evaluation launch (every workgroup of it). First the
// buffer sweep t writes (it holds C_t-1) is brought to C_t on the local rows: the vertices on the
// restore list are copied, or every local row when that list overflowed or the counts are rebuilt
// -- the evaluation then writes only the rows that change. Then the counts. Rebuild: a wave per
// local row, its segments in the blocks overlapping S, colours of C_t counted in an LDS histogram,
// mask and open bits written. Incremental: a wave per (listed vertex u, column block b of the local
// rows): u's neighbours in block b. The work is cut into tasks that the workgroups claim from a
// counter (kDcTask); each adds its completed tasks to kDcDone once (a release) and every workgroup
// waits for all of them (an acquire) before evaluating. A waiting workgroup only waits for tasks a
// running workgroup has claimed, so the grid need not be co-resident; with nothing to update (the
// usual converged sweep) no counter is touched.
constexpr uint32_t kDcCopyRows = 16384;   // copy task: 1024 threads x 16 B
constexpr uint32_t kDcRebuildRows = 64;   // rebuild task: 4 rows per wave
// The control words the update reads (loaded by thread 0 at the launch's start, both parities).
struct DcCtl {
    uint32_t mode, ovf[2], chg[2], len[2];
};
__device__ __forceinline__ void dc_ctl_load(const SweepArgs& a, DcCtl& w) {
    w.mode = a.dc_ctl[kDcMode];
    for (int q = 0; q < 2; q++) {
        w.ovf[q] = a.dc_ctl[kDcChgOvf + q];
        w.chg[q] = a.dc_ctl[kDcChgLen + q];
        w.len[q] = a.dc_ctl[kDcLen + q];
    }
}
// The rebuild of one chunk of a row group's rows (the streaming form, SweepArgs::dc_rbrows = rows
// per chunk): rows [r0, r0 + rows) of group g. Per column block b overlapping S, the colours of
// b's part of S go to LDS (the slice) and the chunk's segments of block b -- contiguous in tcol,
// the rows following each other -- are streamed by the whole workgroup, a 16-byte quad (8 ids of
// one row: segments are padded to multiples of 8) per thread and step, its row found by a binary
// search of the segment starts; each real id in S adds 1 to its row's count of its colour in an
// LDS histogram (two uint16 counts per word: setup_dense takes this form only when no row has
// 65536 arcs). Then the counts, masks and open bits of the chunk's rows are written. Replaces a
// wave per row (one chain of dependent loads each) by coalesced streaming of the ids.
// lds: [histogram rows x hw words][segment starts rows + 1 words] (64 KiB) + [slice: 64 KiB].
template <int NW>
__device__ __forceinline__ void dc_rebuild_chunk(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t g,
                                                 uint32_t r0, uint32_t rows, uint32_t* lds) {
    const uint32_t R = a.grp_rows, bl = a.block_log2, nCol = a.nCol, hw = (nCol + 1u) >> 1;
    uint32_t* const hist = lds;
    uint32_t* const tab = lds + rows * hw;
    uint8_t* const sl = reinterpret_cast<uint8_t*>(lds + kDcEvalLds / 4u);
    for (uint32_t i = threadIdx.x; i < rows * hw; i += blockDim.x) hist[i] = 0u;
    const uint16_t* __restrict__ gc = a.tcol + a.gbase[g];
    const uint32_t sb0 = a.dc_s0 >> bl, sb1 = (a.dc_s1 - 1u) >> bl;
    // diagnostics (MCMC_SOLO_TRACE): workgroup 0's first chunk, stamps at the end of solo_ts
    unsigned long long* const rts = (a.solo_ts && blockIdx.x == 0 && threadIdx.x == 0 && a.solo_ts[8u * 4096u - 1u] == 0ull)
                                        ? a.solo_ts + 8u * 4096u - 64u : nullptr;
    if (rts) rts[0] = wall_clock64();
    for (uint32_t b = sb0; b <= sb1; b++) {
        const uint32_t blo = b << bl;
        const uint32_t lo = max(blo, a.dc_s0) - blo, hi = min(blo + (1u << bl), a.dc_s1) - blo;   // S in block b
        const uint32_t* ts = a.tseg + ((size_t)g * a.nblocks + b) * tseg_stride(R) + r0;
        __syncthreads();   // the last block's readers of sl / tab are done
        for (uint32_t j = threadIdx.x; j <= rows; j += blockDim.x) tab[j] = ts[j];
        {   // the slice [lo, hi) of block b's colours (16-byte loads where aligned)
            const uint32_t q0 = (lo + 15u) & ~15u, q1 = max(hi & ~15u, q0);
            for (uint32_t i = q0 + 16u * threadIdx.x; i < q1; i += 16u * blockDim.x)
                *reinterpret_cast<uint4*>(sl + i) = *reinterpret_cast<const uint4*>(C + blo + i);
            for (uint32_t i = lo + threadIdx.x; i < min(q0, hi); i += blockDim.x) sl[i] = C[blo + i];
            for (uint32_t i = max(q1, lo) + threadIdx.x; i < hi; i += blockDim.x) sl[i] = C[blo + i];
        }
        __syncthreads();
        if (rts && b - sb0 < 28u) rts[1u + 2u * (b - sb0)] = wall_clock64();
        const uint32_t p0 = tab[0] & kTsegPos, p1 = tab[rows] & kTsegPos, nq = (p1 - p0) >> 3;
        // kRbQ quads per thread in flight (one HBM round trip for a block's whole chunk at C3: ~7
        // quads per thread), then their rows (independent binary searches) and histogram adds
        constexpr uint32_t kRbQ = 8;
        for (uint32_t q0 = 0; q0 < nq; q0 += kRbQ * blockDim.x) {
            uint4 v[kRbQ];
#pragma unroll
            for (uint32_t r = 0; r < kRbQ; r++) {
                const uint32_t q = q0 + r * blockDim.x + threadIdx.x;
                v[r] = q < nq ? *reinterpret_cast<const uint4*>(gc + p0 + 8u * q) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t r = 0; r < kRbQ; r++) {
                const uint32_t q = q0 + r * blockDim.x + threadIdx.x;
                if (q >= nq) continue;
                const uint32_t pos = p0 + 8u * q;
                uint32_t L = 0, H = rows;   // the row j with start(j) <= pos < start(j + 1)
                while (H - L > 1u) {
                    const uint32_t mid = (L + H) >> 1;
                    if ((tab[mid] & kTsegPos) <= pos) L = mid;
                    else H = mid;
                }
                const uint32_t end = (tab[L + 1] & kTsegPos) - (tab[L] & 7u);
                uint32_t* const hr = hist + L * hw;
                const uint32_t w4[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t id = (w4[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    if (pos + (uint32_t)k < end && id - lo < hi - lo) {
                        const uint32_t c = sl[id];
                        atomicAdd(&hr[c >> 1], 1u << (16u * (c & 1u)));
                    }
                }
            }
        }
        if (rts && b - sb0 < 28u) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            rts[2u + 2u * (b - sb0)] = wall_clock64();
        }
    }
    __syncthreads();
    // write-out: counts (coalesced), masks, then the chunk's open words
    const uint32_t l0 = g * R + r0;   // first local row of the chunk
    uint32_t* const cnt = a.dc_cnt + (size_t)l0 * a.dc_cw;
    for (uint32_t i = threadIdx.x; i < rows * nCol; i += blockDim.x) {
        const uint32_t j = i / nCol, c = i - j * nCol;
        cnt[(size_t)j * a.dc_cw + c] = (hist[j * hw + (c >> 1)] >> (16u * (c & 1u))) & 0xFFFFu;
    }
    // per (row, mask word): the mask word, and whether it is full; open bits gathered per open word
    // in LDS (the slice is free now), then one AND + one OR per open word (the words at the chunk's
    // ends are shared with the neighbouring chunks' rows)
    const uint32_t w0 = l0 >> 6, nwo = ((l0 + rows - 1u) >> 6) - w0 + 1u;   // open words (per mask word)
    unsigned long long* const ob = reinterpret_cast<unsigned long long*>(sl);   // [nwo][NW]
    for (uint32_t i = threadIdx.x; i < nwo * NW; i += blockDim.x) ob[i] = 0ull;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < rows * NW; i += blockDim.x) {
        const uint32_t j = i / NW, wi = i - j * NW;
        uint32_t mw = 0;
        for (uint32_t c = 32u * wi; c < min(nCol, 32u * wi + 32u); c++)
            mw |= (((hist[j * hw + (c >> 1)] >> (16u * (c & 1u))) & 0xFFFFu) != 0u ? 1u : 0u) << (c & 31u);
        a.dc_mask[(size_t)(l0 + j) * NW + wi] = mw;
        const uint32_t fw = dc_fullw(nCol, wi);
        if ((mw & fw) != fw) atomicOr(&ob[(((l0 + j) >> 6) - w0) * NW + wi], 1ull << ((l0 + j) & 63u));
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nwo * NW; i += blockDim.x) {
        const uint32_t ow = i / NW, wi = i - ow * NW;
        const uint32_t rlo = max((w0 + ow) << 6, l0), rhi = min(((w0 + ow) << 6) + 64u, l0 + rows);   // rows here
        const unsigned long long span = (rhi - rlo >= 64u ? ~0ull : ((1ull << (rhi - rlo)) - 1ull)) << (rlo & 63u);
        const unsigned long long nb = ob[i];
        const size_t idx = (size_t)(w0 + ow) * NW + wi;
        const unsigned long long o1 = atomicAnd(&a.dc_open[idx], ~span | nb);
        dc_osum_note(a, idx, o1, o1 & (~span | nb));
        if (nb) {
            const unsigned long long o2 = atomicOr(&a.dc_open[idx], nb);
            dc_osum_note(a, idx, o2, o2 | nb);
        }
    }
    if (rts) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rts[62] = wall_clock64();
        rts[63] = 1ull;   // (only the first chunk is traced)
    }
}

// The lane rebuild (nCol <= 32, SweepArgs::dc_rbl): a lane per row, a task of blockDim consecutive
// local rows per workgroup. Per column block b overlapping S the
// workgroup's slice of colours sits in LDS (double-buffered: block b + 1's arrives by LDS-DMA while
// block b is counted), and every lane streams its row's segment of block b itself (16-byte quads,
// 8 ids each, kDcLaneQ in flight; the next block's segment bounds are loaded meanwhile). A row's counts of its 32 possible colours live in registers
// as bit planes -- plane k's bit c is bit k of the count of colour c -- so counting an id is a shift
// (its colour's one-hot word) and a quad's eight one-hots are summed per colour by a carry-save tree
// into a 4-bit number that is added into the planes with a short carry ripple. No LDS atomics, no
// search of the quad's row, every id read once from HBM in 16-byte loads. A segment is padded to a
// multiple of 8 ids with copies of its first id: inside S the padding is counted with the rest and
// subtracted once per segment; in a block that S covers only in part every id is tested instead.
// At the end the planes are transposed into counts (one word per colour) and written with the
// mask word and the wave's open word. Replaces dc_rebuild_chunk's LDS histograms (per id: a colour
// read, a histogram atomic, and per quad a binary search of the segment starts) for nCol <= 32.
constexpr uint32_t kDcPlanes = 16;
constexpr uint32_t kDcSliceBuf = 65536;   // one block's colours (2^block_log2 <= 2^16 bytes)

// s = a + b + c and the carry, per bit (32 colours at once)
__device__ __forceinline__ void dc_fa(uint32_t a, uint32_t b, uint32_t c, uint32_t& s, uint32_t& co) {
    const uint32_t t = a ^ b;
    s = t ^ c;
    co = (t & c) | (~t & a);
}
// The eight one-hot words x[] summed per colour: b0 + 2 b1 + 4 b2 + 8 b3 (a carry-save tree)
__device__ __forceinline__ void dc_sum8(const uint32_t (&x)[8], uint32_t& b0, uint32_t& b1, uint32_t& b2, uint32_t& b3) {
    uint32_t sa, ca, sb, cb, cd, s2, c3a;
    dc_fa(x[0], x[1], x[2], sa, ca);
    dc_fa(x[3], x[4], x[5], sb, cb);
    const uint32_t sc = x[6] ^ x[7], cc = x[6] & x[7];
    dc_fa(sa, sb, sc, b0, cd);           // weight 1
    dc_fa(ca, cb, cc, s2, c3a);          // weight 2 (three of four)
    b1 = s2 ^ cd;
    const uint32_t c3b = s2 & cd;
    b2 = c3a ^ c3b;                      // weight 4
    b3 = c3a & c3b;                      // weight 8
}
// The carry c into planes K.. (a ripple that stops once no lane of the wave carries; counts <
// 2^np: no carry leaves the top plane). Templates instead of a loop with an exit, so every plane
// stays a named register.
template <int K>
__device__ __forceinline__ void dc_ripple(uint32_t (&A)[kDcPlanes], uint32_t np, uint32_t c) {
    if constexpr (K < (int)kDcPlanes) {
        if ((uint32_t)K < np && __ballot(c != 0u) != 0ull) {
            const uint32_t nc = A[K] & c;
            A[K] ^= c;
            dc_ripple<K + 1>(A, np, nc);
        }
    }
}
// Planes A (np >= 4 of them) += b0 + 2 b1 + 4 b2 + 8 b3 per colour
__device__ __forceinline__ void dc_planes_add(uint32_t (&A)[kDcPlanes], uint32_t np, uint32_t b0, uint32_t b1,
                                              uint32_t b2, uint32_t b3) {
    uint32_t c = A[0] & b0, s;
    A[0] ^= b0;
    dc_fa(A[1], b1, c, s, c);
    A[1] = s;
    dc_fa(A[2], b2, c, s, c);
    A[2] = s;
    dc_fa(A[3], b3, c, s, c);
    A[3] = s;
    dc_ripple<4>(A, np, c);
}
// The borrow br out of planes K.. (as dc_ripple)
template <int K>
__device__ __forceinline__ void dc_unborrow(uint32_t (&A)[kDcPlanes], uint32_t np, uint32_t br) {
    if constexpr (K < (int)kDcPlanes) {
        if ((uint32_t)K < np && __ballot(br != 0u) != 0ull) {
            const uint32_t x = A[K];
            A[K] = x ^ br;
            dc_unborrow<K + 1>(A, np, ~x & br);
        }
    }
}
// Planes A -= pad x oh (pad <= 7; every colour of oh was counted at least pad times: no borrow out)
__device__ __forceinline__ void dc_planes_sub(uint32_t (&A)[kDcPlanes], uint32_t np, uint32_t oh, uint32_t pad) {
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t b = ((pad >> k) & 1u) ? oh : 0u;
        const uint32_t x = A[k];
        A[k] = x ^ b ^ br;
        br = (~x & (b | br)) | (b & br);
    }
    dc_unborrow<3>(A, np, br);
}
// One quad (8 ids) of a row segment into the row's planes: the eight colours read from the slice
// first, then their one-hot words. CHK (the block is not wholly inside S): id j counts only if it is
// one of the segment's nv real ids and lies in [lo, lo + span); else all eight count (padding is
// subtracted per segment). qok: the quad lies inside the lane's segment. Branch-free: the wave
// runs it once per quad position that any lane holds.
template <bool CHK>
__device__ __forceinline__ void dc_lane_quad(uint32_t (&A)[kDcPlanes], uint32_t np, uint4 v, const uint8_t* __restrict__ sl,
                                             bool qok, int nv, uint32_t lo, uint32_t span) {
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    uint32_t id[8], c[8], x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) id[k] = (w4[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
#pragma unroll
    for (int k = 0; k < 8; k++) c[k] = sl[id[k]];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        bool ok = qok;
        if constexpr (CHK) ok = ok && (k < nv) && (id[k] - lo < span);
        x[k] = ok ? (1u << c[k]) : 0u;
    }
    uint32_t b0, b1, b2, b3;
    dc_sum8(x, b0, b1, b2, b3);
    dc_planes_add(A, np, b0, b1, b2, b3);
}
// A row segment's quads [s0, e) (8 ids each; real ids below s1) into the planes, kDcLaneQ quads per
// lane in flight: every lane loads kDcLaneQ quads (positions past its segment load its first quad
// again -- harmless, they are not counted), so the loads are straight-line and the waits counted;
// the few lanes with a longer segment load the rest in predicated rounds of 4.
template <bool CHK, uint32_t kDcLaneQ>
__device__ __forceinline__ void dc_lane_segment(uint32_t (&A)[kDcPlanes], uint32_t np, const uint16_t* __restrict__ gc,
                                                uint32_t s0, uint32_t s1, uint32_t e, const uint8_t* __restrict__ sl,
                                                uint32_t lo, uint32_t span) {
    {   // the first kDcLaneQ quads: straight-line loads (a lane past its segment reloads its first quad)
        uint4 v[kDcLaneQ];
#pragma unroll
        for (uint32_t q = 0; q < kDcLaneQ; q++) {
            const uint32_t pos = s0 + 8u * q;
            v[q] = *reinterpret_cast<const uint4*>(gc + (pos < e ? pos : s0));
        }
#pragma unroll
        for (uint32_t q = 0; q < kDcLaneQ; q++) {
            const uint32_t pos = s0 + 8u * q;
            if (__ballot(pos < e)) dc_lane_quad<CHK>(A, np, v[q], sl, pos < e, (int)(s1 - pos), lo, span);
        }
    }
    // the rest of the longer segments, 4 quads per round, loaded only by the lanes that hold them
    for (uint32_t j = kDcLaneQ; __ballot(s0 + 8u * j < e); j += 4u) {
        uint4 v[4];
#pragma unroll
        for (uint32_t q = 0; q < 4u; q++) {
            const uint32_t pos = s0 + 8u * (j + q);
            v[q] = make_uint4(0u, 0u, 0u, 0u);
            if (pos < e) v[q] = *reinterpret_cast<const uint4*>(gc + pos);
        }
#pragma unroll
        for (uint32_t q = 0; q < 4u; q++) {
            const uint32_t pos = s0 + 8u * (j + q);
            if (__ballot(pos < e)) dc_lane_quad<CHK>(A, np, v[q], sl, pos < e, (int)(s1 - pos), lo, span);
        }
    }
}
// Counts of one row from its planes: the 32 x 32 bit transpose (T[c] bit k = plane k bit c), then
// the row's nCol counts written.
__device__ __forceinline__ void dc_lane_write(const SweepArgs& a, const uint32_t (&A)[kDcPlanes], uint32_t l) {
    uint32_t T[32];
#pragma unroll
    for (int k = 0; k < 16; k++) {   // stage 16: the upper planes are zero
        T[k + 16] = A[k] >> 16;
        T[k] = A[k] & 0xFFFFu;
    }
    auto stage = [&](const int j, const uint32_t m) {
#pragma unroll
        for (int k = 0; k < 32; k++) {
            if (k & j) continue;
            const uint32_t t = ((T[k] >> j) ^ T[k + j]) & m;
            T[k + j] ^= t;
            T[k] ^= t << j;
        }
    };
    stage(8, 0x00FF00FFu);
    stage(4, 0x0F0F0F0Fu);
    stage(2, 0x33333333u);
    stage(1, 0x55555555u);
    uint32_t* const cw = a.dc_cnt + (size_t)l * a.dc_cw;
    if ((a.nCol & 3u) == 0u) {
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (4u * q < a.nCol) *reinterpret_cast<uint4*>(cw + 4 * q) = make_uint4(T[4 * q], T[4 * q + 1], T[4 * q + 2], T[4 * q + 3]);
    } else {
#pragma unroll
        for (int c = 0; c < 32; c++)
            if ((uint32_t)c < a.nCol) cw[c] = T[c];
    }
}

// The tile-transposed copy of S's ids (the host's dc_build_tid, once per context): tile t = local
// rows [64 t, 64 t + 64); for each S block in order, Qt = the tile's longest segment in quads, then
// quad k of lane j at [k][j] (16 bytes each; quads past a row's segment are zero and never counted).
// A wave's k-th quad load of the rebuild is then 1 KiB contiguous: the per-lane form loads 64 16-byte
// pieces of 64 different lines per instruction, and most of each line it pulls from L2 into the CU's
// cache is gone before the lane's next quad (measured at C3: coalesced loads of the same quads count
// in 4.1 ms, the per-lane form 6.45 ms).
__device__ __forceinline__ uint32_t dc_wave_max(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return __builtin_amdgcn_readfirstlane(x);
}
// Row l's segment of block b: [s0, e) in its group's ids (e: the padded end), raw = its tseg entry.
__device__ __forceinline__ void dc_tid_seg(const SweepArgs& a, uint32_t l, uint32_t b, uint32_t& raw, uint32_t& nxt,
                                           const uint16_t*& gc) {
    const uint32_t R = a.grp_rows, g = l / R, r = l - g * R;
    const uint32_t* ts = a.tseg + ((size_t)g * a.nblocks + b) * tseg_stride(R);
    raw = ts[r];
    nxt = ts[r + 1];
    gc = a.tcol + a.gbase[g];
}
// Quads per tile (x 64), a wave per tile.
__global__ __launch_bounds__(256) void dc_tid_size_kernel(SweepArgs a, uint64_t* __restrict__ tsize, uint32_t ntiles) {
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
    if (t >= ntiles) return;   // (wave-uniform)
    const uint32_t nloc = a.v_end - a.v_begin, l = 64u * t + lane, bl = a.block_log2;
    const uint32_t sb0 = a.dc_s0 >> bl, sb1 = (a.dc_s1 - 1u) >> bl;
    uint64_t tot = 0;
    for (uint32_t b = sb0; b <= sb1; b++) {
        uint32_t raw = 0, nxt = 0;
        const uint16_t* gc;
        if (l < nloc) dc_tid_seg(a, l, b, raw, nxt, gc);
        tot += dc_wave_max(((nxt & kTsegPos) - (raw & kTsegPos)) >> 3);
    }
    if (lane == 0) tsize[t] = 64ull * tot;
}
// The copy, a wave per tile: lane j's quads of each block (its own segment, 16-byte loads), stored
// transposed; the tile's quads past a lane's segment are zero.
__global__ __launch_bounds__(256) void dc_tid_fill_kernel(SweepArgs a, uint32_t ntiles) {
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
    if (t >= ntiles) return;
    const uint32_t nloc = a.v_end - a.v_begin, l = 64u * t + lane, bl = a.block_log2;
    const uint32_t sb0 = a.dc_s0 >> bl, sb1 = (a.dc_s1 - 1u) >> bl;
    uint4* __restrict__ out = const_cast<uint4*>(a.dc_tid) + a.dc_toff[t];
    for (uint32_t b = sb0; b <= sb1; b++) {
        uint32_t raw = 0, nxt = 0;
        const uint16_t* gc = a.tcol;
        if (l < nloc) dc_tid_seg(a, l, b, raw, nxt, gc);
        const uint32_t s0 = raw & kTsegPos, qr = ((nxt & kTsegPos) - s0) >> 3, Qt = dc_wave_max(qr);
        for (uint32_t k = 0; k < Qt; k++)
            out[64u * k + lane] = k < qr ? *reinterpret_cast<const uint4*>(gc + s0 + 8u * k) : make_uint4(0u, 0u, 0u, 0u);
        out += 64u * Qt;
    }
}
// A row's quads of one block from the transposed copy: tq = the tile's quads of this block, Qt of
// them (wave-uniform), qr the lane's own, nv its real ids; first = the lane's first id.
template <bool CHK, uint32_t Q>
__device__ __forceinline__ void dc_tid_segment(uint32_t (&A)[kDcPlanes], uint32_t np, const uint4* __restrict__ tq,
                                               uint32_t Qt, uint32_t qr, int nv, const uint8_t* __restrict__ sl,
                                               uint32_t lo, uint32_t span, uint32_t lane, uint32_t& first) {
    {
        uint4 v[Q];
#pragma unroll
        for (uint32_t q = 0; q < Q; q++) v[q] = q < Qt ? tq[64u * q + lane] : make_uint4(0u, 0u, 0u, 0u);
        first = v[0].x & 0xFFFFu;
#pragma unroll
        for (uint32_t q = 0; q < Q; q++)
            if (q < Qt) dc_lane_quad<CHK>(A, np, v[q], sl, q < qr, nv - 8 * (int)q, lo, span);
    }
    for (uint32_t j = Q; j < Qt; j += 4u) {
        uint4 v[4];
#pragma unroll
        for (uint32_t q = 0; q < 4u; q++) v[q] = j + q < Qt ? tq[64u * (j + q) + lane] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (uint32_t q = 0; q < 4u; q++)
            if (j + q < Qt) dc_lane_quad<CHK>(A, np, v[q], sl, j + q < qr, nv - 8 * (int)(j + q), lo, span);
    }
}

template <int NW, uint32_t Q, bool TID, uint32_t NB>
__device__ __forceinline__ void dc_rebuild_lanes(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t task,
                                                 uint32_t* lds) {
    const uint32_t nloc = a.v_end - a.v_begin, R = a.grp_rows, bl = a.block_log2, np = a.dc_planes;
    const uint32_t sb0 = a.dc_s0 >> bl, sb1 = (a.dc_s1 - 1u) >> bl, bsz = 1u << bl;
    const uint32_t wv = threadIdx.x >> 6, nwv = blockDim.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t lds0 = lds_addr(lds);
    const uint32_t padn = (a.n + 15u) & ~15u;
    uint8_t* const slb = reinterpret_cast<uint8_t*>(lds);
    // the slice of block b (whole 16-byte pieces, below n rounded up) into buffer `buf` by LDS-DMA:
    // 1 KiB per wave-instruction
    auto dma = [&](uint32_t b, uint32_t buf) {
        const uint32_t blo = b << bl, npc = (min(bsz, padn - blo) + 15u) >> 4;
        for (uint32_t w = wv; w * 64u < npc; w += nwv) {
            const uint32_t p = min(w * 64u + lane, npc - 1u);
            glds16(C + blo + 16u * p, __builtin_amdgcn_readfirstlane(lds0 + buf * kDcSliceBuf + w * 1024u));
        }
    };
    // this lane's row, its group and position in the group; its segment table entries of block b
    const uint32_t l = task * blockDim.x + threadIdx.x;
    const bool in = l < nloc;
    const uint32_t g = in ? l / R : 0u, r = l - g * R;
    const uint16_t* __restrict__ gc = a.tcol + (in ? a.gbase[g] : 0ull);
    const uint32_t* __restrict__ tsg = a.tseg + (size_t)g * a.nblocks * tseg_stride(R) + r;
    uint32_t raw = 0, nxt = 0;
    if (in) {
        raw = tsg[(size_t)sb0 * tseg_stride(R)];
        nxt = tsg[(size_t)sb0 * tseg_stride(R) + 1u];
    }
    uint32_t A[kDcPlanes];
#pragma unroll
    for (int k = 0; k < (int)kDcPlanes; k++) A[k] = 0u;
    // TID: this wave's tile in the transposed copy (a wave past the rows reads none of it: Qt = 0)
    const uint32_t tile = l >> 6, ntiles = (nloc + 63u) >> 6;
    const uint4* __restrict__ tq = nullptr;
    if constexpr (TID) tq = a.dc_tid + (tile < ntiles ? a.dc_toff[tile] : 0ull);
    dma(sb0, 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint32_t b = sb0; b <= sb1; b++) {
        const uint32_t buf = NB == 2u ? (b - sb0) & 1u : 0u;
        if (NB == 2u && b < sb1) dma(b + 1u, buf ^ 1u);
        const uint32_t blo = b << bl;
        const uint32_t lo = max(blo, a.dc_s0) - blo, hi = min(blo + bsz, a.dc_s1) - blo, span = hi - lo;
        const bool chk = lo != 0u || hi != bsz;   // S covers block b in part: every id tested
        const uint8_t* __restrict__ sl = slb + buf * kDcSliceBuf;
        // real ids [s0, s1), quads up to the padded end e (the next row's start)
        const uint32_t s0 = raw & kTsegPos, e = nxt & kTsegPos, s1 = e - (raw & 7u);
        const uint32_t pad = chk ? 0u : (raw & 7u);
        if (in && b < sb1) {   // the next block's entries, in flight with this block's ids
            raw = tsg[(size_t)(b + 1u) * tseg_stride(R)];
            nxt = tsg[(size_t)(b + 1u) * tseg_stride(R) + 1u];
        }
        // (one round of kDcLaneQ quads for a C3 row's ~66 ids per block)
        if constexpr (TID) {
            const uint32_t qr = (e - s0) >> 3, Qt = dc_wave_max(qr);   // (a lane past the rows: qr = 0)
            uint32_t first = 0;
            if (chk) {
                dc_tid_segment<true, Q>(A, np, tq, Qt, qr, (int)(s1 - s0), sl, lo, span, lane, first);
            } else {
                dc_tid_segment<false, Q>(A, np, tq, Qt, qr, (int)(s1 - s0), sl, lo, span, lane, first);
                if (__ballot(pad != 0u)) {   // the layout's padding (copies of the first id): out again
                    const uint32_t ohf = pad ? 1u << sl[first] : 0u;
                    dc_planes_sub(A, np, ohf, pad);
                }
            }
            tq += 64u * Qt;
        } else if (chk) {
            dc_lane_segment<true, Q>(A, np, gc, s0, s1, e, sl, lo, span);
        } else {
            dc_lane_segment<false, Q>(A, np, gc, s0, s1, e, sl, lo, span);
            if (__ballot(pad != 0u)) {   // the padding (copies of the segment's first id) counted: out again
                const uint32_t ohf = pad ? 1u << sl[gc[s0]] : 0u;
                dc_planes_sub(A, np, ohf, pad);
            }
        }
        // NB 1 (a single slice buffer): every wave is done with block b's slice before block b + 1's
        // lands in it (the other workgroup on the CU counts meanwhile)
        if (NB == 1u && b < sb1) {
            __syncthreads();
            dma(b + 1u, 0u);
        }
        // block b + 1's slice has landed and every wave is done with block b's (the next DMA's target)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const uint32_t fw = dc_fullw(a.nCol, 0u);
    uint32_t mw = 0;
#pragma unroll
    for (int k = 0; k < (int)kDcPlanes; k++) mw |= A[k];
    mw &= fw;
    if (in) {
        a.dc_mask[(size_t)l * NW] = mw;
        dc_lane_write(a, A, l);
    }
    // the wave's 64 rows are one open word (tasks start at multiples of 64 rows)
    const unsigned long long ob = __ballot(in && mw != fw);
    if (lane == 0u && in) {
        const size_t wi = (size_t)(l >> 6) * NW;
        const unsigned long long o = atomicExch(&a.dc_open[wi], ob);
        dc_osum_note(a, wi, o, ob);
    }
}

// A fresh colouring's update as its own launch (the host's dc_prep, before the colouring's first
// sweep; nCol <= 32): workgroup k < n1 copies C_t into the other buffer on local rows [16384 k,
// 16384 (k + 1)) -- the copy a rebuild sweep's update makes -- and workgroup n1 + k rebuilds the
// counts of rows [BS k, BS (k + 1)) by dc_rebuild_lanes. A kernel of its own, so the lane
// rebuild's registers (its planes, Q quads per lane in flight) are not the dense sweep's: inside the sweep
// (a rebuild after list overflows) the update keeps the chunk rebuild. dc_ctl_fresh_kernel then
// marks the update done (mode 0, empty lists) and counts the rebuild.
template <int NW, uint32_t BS, uint32_t Q, bool TID, uint32_t NB>
__global__ __launch_bounds__(BS) void dc_rebuild_kernel(SweepArgs a, uint32_t n1) {
    extern __shared__ uint4 dc_lds[];
    const uint32_t t = a.st->t;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;   // C_t
    uint8_t* __restrict__ Y = (t & 1) ? a.colors0 : a.colors1;
    if (blockIdx.x < n1) {
        const size_t b0 = (size_t)a.v_begin + (size_t)blockIdx.x * kDcCopyRows, b1 = min((size_t)a.v_end, b0 + kDcCopyRows);
        const size_t q0 = (b0 + 15) & ~(size_t)15, q1 = (b1 & ~(size_t)15) > q0 ? (b1 & ~(size_t)15) : q0;
        for (size_t i = q0 + 16u * threadIdx.x; i < q1; i += 16u * blockDim.x)
            *reinterpret_cast<uint4*>(Y + i) = *reinterpret_cast<const uint4*>(C + i);
        for (size_t i = b0 + threadIdx.x; i < (q0 < b1 ? q0 : b1); i += blockDim.x) Y[i] = C[i];
        for (size_t i = (q1 > b0 ? q1 : b0) + threadIdx.x; i < b1; i += blockDim.x) Y[i] = C[i];
        return;
    }
    dc_rebuild_lanes<NW, Q, TID, NB>(a, C, blockIdx.x - n1, reinterpret_cast<uint32_t*>(dc_lds));
}
__global__ void dc_ctl_fresh_kernel(uint32_t* __restrict__ k) {
    k[kDcMode] = 0u;
    for (uint32_t p = 0; p < 2u; p++) k[kDcLen + p] = k[kDcOvf + p] = k[kDcChgLen + p] = k[kDcChgOvf + p] = 0u;
    k[kDcTask] = k[kDcDone] = 0u;
    reinterpret_cast<unsigned long long*>(k + kDcStat)[1] += 1ull;   // rebuilds
}

template <int NW>
__device__ __forceinline__ void dc_update_tasks(const SweepArgs& a, uint32_t t, uint32_t* lds, const DcCtl& w) {
    __shared__ uint32_t sh_k;
    const uint32_t p = t & 1u;
    const uint32_t mode = w.mode, copy = mode | w.ovf[p];
    const uint32_t m = min(w.chg[p], a.dc_chg_cap), len = min(w.len[p], a.dc_cap);
    const uint32_t nloc = a.v_end - a.v_begin, bl = a.block_log2;
    const uint32_t bl0 = a.v_begin >> bl, nbl = ((a.v_end - 1u) >> bl) - bl0 + 1u;
    const uint32_t nmov_w = mode ? 0u : len * nbl;   // len <= |S| / 8 + 1 when incremental: no overflow
    const uint32_t n1 = copy ? (nloc + kDcCopyRows - 1u) / kDcCopyRows : (m + blockDim.x - 1u) / blockDim.x;
    const uint32_t R = a.grp_rows, Rc = a.dc_rbrows, cpg = Rc ? (R + Rc - 1u) / Rc : 0u;   // chunks per group
    const uint32_t n2 = mode ? (Rc ? a.ngroups * cpg : (nloc + kDcRebuildRows - 1u) / kDcRebuildRows)
                             : (nmov_w + (blockDim.x >> 6) - 1u) / (blockDim.x >> 6);   // a wave task per wave
    const uint32_t T = n1 + n2;
    if (T == 0u) return;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;   // C_t
    uint8_t* __restrict__ Y = (t & 1) ? a.colors0 : a.colors1;         // C_t-1, becomes C_t+1
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t* h = lds + 256u * wv;
    uint32_t mine = 0;
    for (;;) {
        if (threadIdx.x == 0) sh_k = atomicAdd(&a.dc_ctl[kDcTask], 1u);
        __syncthreads();
        const uint32_t k = sh_k;
        __syncthreads();   // every thread has read sh_k before thread 0 claims again
        if (k >= T) break;
        mine++;
        if (k < n1 && copy) {
            const size_t b0 = (size_t)a.v_begin + (size_t)k * kDcCopyRows, b1 = min((size_t)a.v_end, b0 + kDcCopyRows);
            const size_t q0 = (b0 + 15) & ~(size_t)15, q1 = (b1 & ~(size_t)15) > q0 ? (b1 & ~(size_t)15) : q0;
            for (size_t i = q0 + 16u * threadIdx.x; i < q1; i += 16u * blockDim.x)
                *reinterpret_cast<uint4*>(Y + i) = *reinterpret_cast<const uint4*>(C + i);
            for (size_t i = b0 + threadIdx.x; i < (q0 < b1 ? q0 : b1); i += blockDim.x) Y[i] = C[i];
            for (size_t i = (q1 > b0 ? q1 : b0) + threadIdx.x; i < b1; i += blockDim.x) Y[i] = C[i];
        } else if (k < n1) {
            const uint32_t i = k * blockDim.x + threadIdx.x;
            if (i < m) {
                const uint32_t u = a.dc_chg[(size_t)p * a.dc_chg_cap + i];
                Y[u] = C[u];
            }
        } else if (mode && Rc) {   // the streaming rebuild of one chunk of a group's rows
            const uint32_t k2 = k - n1, gg = k2 / cpg, r0 = (k2 - gg * cpg) * Rc;
            const uint32_t grow = min(R, nloc - gg * R);   // rows of group gg
            if (r0 < grow) dc_rebuild_chunk<NW>(a, C, gg, r0, min(Rc, grow - r0), lds);
        } else if (mode) {
            const uint32_t b0 = a.dc_s0 >> bl, b1 = (a.dc_s1 - 1u) >> bl, sw = a.dc_s1 - a.dc_s0;
            const uint32_t r0 = (k - n1) * kDcRebuildRows;
            for (uint32_t l = r0 + wv; l < min(r0 + kDcRebuildRows, nloc); l += blockDim.x >> 6) {
                for (uint32_t i = lane; i < a.dc_cw; i += 64u) h[i] = 0;
                dc_lds_wait();
                // 8 column blocks per round, 8 lanes each, 8 ids per lane in flight: one chain of
                // three dependent loads (segment bounds, ids, colours) per 8 blocks, not per block
                const uint32_t grp = lane >> 3, gl = lane & 7u;
                for (uint32_t bb = b0; bb <= b1; bb += 8u) {
                    const uint32_t b = bb + grp;
                    uint32_t s0 = 0, s1 = 0;
                    const uint16_t* gc = nullptr;
                    if (b <= b1) dc_segment(a, l, b, s0, s1, gc);
                    const uint32_t base = b << bl;
                    for (uint32_t q = s0 + gl; __ballot(q < s1); q += 64u) {
                        uint32_t id[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) id[k] = q + 8u * k < s1 ? (uint32_t)gc[q + 8u * k] : 0xFFFFFFFFu;
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const uint32_t u = base | id[k];
                            if (id[k] != 0xFFFFFFFFu && u - a.dc_s0 < sw) atomicAdd(&h[C[u]], 1u);
                        }
                    }
                }
                dc_lds_wait();
                uint32_t* cr = a.dc_cnt + (size_t)l * a.dc_cw;
                for (uint32_t i = lane; i < a.dc_cw; i += 64u) cr[i] = h[i];
                uint32_t* mk = a.dc_mask + (size_t)l * NW;
                const size_t ow0 = (size_t)(l >> 6) * NW;
                unsigned long long* ow = a.dc_open + ow0;
                const unsigned long long obit = 1ull << (l & 63u);
                for (uint32_t c0 = 0; c0 < 32u * NW; c0 += 64u) {
                    const uint32_t c = c0 + lane;
                    const uint64_t bm = __ballot(c < a.nCol && h[c] != 0u);
                    if (lane == 0) {
                        for (uint32_t i = c0 >> 5; i < min((c0 >> 5) + 2u, (uint32_t)NW); i++) {
                            const uint32_t mw = (uint32_t)(bm >> (32u * (i - (c0 >> 5)))), fw = dc_fullw(a.nCol, i);
                            mk[i] = mw;
                            if ((mw & fw) != fw) {
                                const unsigned long long o = atomicOr(&ow[i], obit);
                                dc_osum_note(a, ow0 + i, o, o | obit);
                            } else {
                                const unsigned long long o = atomicAnd(&ow[i], ~obit);
                                dc_osum_note(a, ow0 + i, o, o & ~obit);
                            }
                        }
                    }
                }
                dc_lds_wait();   // every lane's reads of h are done before the next row clears it
            }
        } else {
            const uint32_t task = (k - n1) * (blockDim.x >> 6) + wv;
            if (task < nmov_w) {
                const uint32_t i = task / nbl, b = bl0 + (task - i * nbl);
                const uint32_t* e = a.dc_list + 2u * ((size_t)p * a.dc_cap + i);   // (u, ca << 16 | cb)
                const uint32_t u = e[0], ab = e[1];
                const uint32_t ca = ab >> 16, cb = ab & 0xFFFFu;
                uint32_t s0, s1;
                const uint16_t* gc;
                dc_segment(a, u - a.v_begin, b, s0, s1, gc);
                const uint32_t base = b << bl;
                for (uint32_t q = s0 + lane; q < s1; q += 64u) {
                    const uint32_t lw = (base | (uint32_t)gc[q]) - a.v_begin;
                    if (lw < nloc) dc_move<NW>(a, lw, ca, cb);
                }
            }
        }
        // every wave drains its own stores (copies, rebuilt counts / masks) before the barrier:
        // thread 0's agent release below writes back what has reached L2, so the stores of the
        // other 15 waves must be complete first (MI355X_MICROARCH.md, "Valid forms": producer)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // the task's stores are complete before the next claim / the release
    }
    if (threadIdx.x == 0 && mine) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        atomicAdd(&a.dc_ctl[kDcDone], mine);
    }
    if (threadIdx.x < 64u) {   // wave 0 waits for every task (a wave-uniform spin loop; the others at the barrier)
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&a.dc_ctl[kDcDone], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT)) < T)
            __builtin_amdgcn_s_sleep(4);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// Rows of this wave whose dense mask is not full (`open`): each in turn, the whole wave scans its
// segments in the column blocks not inside S (colours of C_t from the replica), OR-ing into its
// mask until it is full or the blocks run out; lane j's mask comes back full. Out of line (rare:
// C3 ~0.005 % of rows) and with everything passed by value -- a reference to the kernel's
// SweepArgs would copy the whole struct to scratch in every lane.
// Lane j's 64-bit value (wave-uniform result).
__device__ __forceinline__ unsigned long long dc_lane64(unsigned long long x, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), j);
    return ((unsigned long long)hi << 32) | lo;
}

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
    // kDcScanBlocks column blocks per round, 16 lanes each (segment start/end, then up to 8 ids per
    // lane in flight, then their colours): one chain of three dependent loads covers the blocks a
    // missing colour is almost always found in, instead of one chain per block
    constexpr uint32_t kDcScanBlocks = 4;
    const uint32_t grp = (uint32_t)lane >> 4, gl = (uint32_t)lane & 15u;
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
        for (uint32_t b0 = 0; b0 < d.nb; b0 += kDcScanBlocks) {
            const uint32_t b = b0 + grp, lo = b << d.bl;
            const bool act = b < d.nb && !(lo >= d.s0 && lo + (1u << d.bl) <= d.s1);   // inside S: counted
            if (!__ballot(act)) continue;
            uint32_t s0 = 0, s1 = 0;
            if (act) {
                const uint32_t* ts = d.tseg + ((size_t)g * d.nb + b) * tseg_stride(d.R);
                const uint32_t raw = ts[r];
                s0 = raw & kTsegPos;
                s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
            }
            uint32_t m[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) m[i] = 0;
            for (uint32_t k = s0 + gl; __ballot(k < s1); k += 128u) {
                uint32_t id[8];
#pragma unroll
                for (int q = 0; q < 8; q++) id[q] = k + 16u * q < s1 ? (uint32_t)gc[k + 16u * q] : 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (id[q] != 0xFFFFFFFFu) set_color_bit<NW>(m, C[lo | id[q]]);
            }
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

// Sweep t's evaluation: persistent, one 1024-thread workgroup per CU. Lane j of a wave holds 16
// consecutive rows (kDcLaneRows), so a wave step covers a span of 1024 rows: one 16-byte colour
// load and one open word per lane. Wave w of the grid takes spans w, w + W, w + 2 W, ... (W = all
// waves), the next span's loads in flight while this one is evaluated. A row that is not open has
// the full mask: it holds its own colour and no free colour -- fill_p's case (i) -- so with the
// closed-form walk (SweepArgs::ewalk) it keeps its colour exactly when u in [E[cv], S[cv])
// (evaluate_lane's shortcut). Kept rows are only counted (Cviol; the update already holds C_t in
// the buffer written); any other row -- open, taboo, changing, or the walk's rare cases -- goes
// through evaluate_lane, one row position j of the lanes at a time, open rows first completing
// their mask (dc_open_scan). u_v of row l is x_t 16807^(v_begin + l + 1).
// The workgroup's staged appends (DcStage, evaluate_lane) into the global lists, all threads: a
// stage that never filled is copied behind one reservation per list; one that overflowed (its
// holes are ~0u) entry by entry. Returns whether anything was appended (the workgroup releases).
__device__ __forceinline__ bool dc_stage_flush(const SweepArgs& a, DevState* st, DcStage& stg, uint32_t t) {
    __shared__ uint32_t base[3];
    const uint32_t q = (t + 1u) & 1u;
    const uint32_t caps[3] = {kDcStageChg, kDcStageS, kDcStageEv};
    const uint32_t n0 = stg.n[0], n1 = stg.n[1], n2 = stg.n[2];
    if ((n0 | n1 | n2) == 0u) return false;
    if (threadIdx.x == 0) {
        base[0] = (n0 && n0 <= caps[0]) ? atomicAdd(&a.dc_ctl[kDcChgLen + q], n0) : 0u;
        base[1] = (n1 && n1 <= caps[1]) ? atomicAdd(&a.dc_ctl[kDcLen + q], n1) : 0u;
        base[2] = (n2 && n2 <= caps[2]) ? atomicAdd(&st->ev_count, n2) : 0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < min(n0, caps[0]); i += blockDim.x) {
        const uint32_t v = stg.chg[i];
        if (v == ~0u) continue;
        const uint32_t j = n0 <= caps[0] ? base[0] + i : atomicAdd(&a.dc_ctl[kDcChgLen + q], 1u);
        if (j < a.dc_chg_cap) a.dc_chg[(size_t)q * a.dc_chg_cap + j] = v;
        else a.dc_ctl[kDcChgOvf + q] = 1u;
    }
    for (uint32_t i = threadIdx.x; i < min(n1, caps[1]); i += blockDim.x) {
        const uint32_t v = stg.s[2u * i];
        if (v == ~0u) continue;
        const uint32_t j = n1 <= caps[1] ? base[1] + i : atomicAdd(&a.dc_ctl[kDcLen + q], 1u);
        if (j < a.dc_cap) {
            uint32_t* e = a.dc_list + 2u * ((size_t)q * a.dc_cap + j);
            e[0] = v;
            e[1] = stg.s[2u * i + 1u];
        } else {
            a.dc_ctl[kDcOvf + q] = 1u;
        }
    }
    for (uint32_t i = threadIdx.x; i < min(n2, caps[2]); i += blockDim.x) {
        const uint32_t v = stg.ev[i];
        if (v == ~0u) continue;
        const uint32_t j = n2 <= caps[2] ? base[2] + i : atomicAdd(&st->ev_count, 1u);
        if (j < a.ev_cap) a.events[j] = v;
        else atomicOr(&st->err, kDevErrEvents);
    }
    return true;
}

// x 16807 mod (2^31 - 1) for a minstd state x < 2^31: the product is below 2^46, one fold and one
// conditional subtraction (minstd_mulmod's general form takes two folds of a 64-bit product).
__device__ __forceinline__ uint32_t dc_mul16807(uint32_t x) {
    const uint32_t lo = x * kMinstdA, hi = __umulhi(x, kMinstdA);
    uint32_t r = (lo & kMinstdM) + ((hi << 1) | (lo >> 31));
    return r >= kMinstdM ? r - kMinstdM : r;
}
// The smallest minstd state x in [1, 2^31 - 1) with minstd_canonical(x) >= f (2^31 - 1 if none):
// canonical is non-decreasing in x, so u >= f <=> x >= this, exactly (a binary search over states).
__device__ __forceinline__ uint32_t dc_canonical_at_least(float f) {
    uint32_t lo = 1u, hi = kMinstdM;   // answer in [lo, hi]; hi = none
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (minstd_canonical(mid) >= f) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}

constexpr uint32_t kDcLaneRows = 16;
constexpr uint32_t kDcSpan = 64u * kDcLaneRows;
// The per-launch tables of a dense sweep (LDS): fill_p's closed-form own-colour walk {E[c], S[c]}
// and its keep interval [E, S) of u as minstd states, [x_lo, x_hi) (nullptr without ewalk).
struct DcTabs {
    const float2* ew;
    const uint2* xkeep;
};
__device__ __forceinline__ DcTabs dc_tabs_load(const SweepArgs& a, float2* ewl, uint2* xkeep) {
    if (a.ewalk) {
        for (uint32_t i = threadIdx.x; i < a.nCol; i += blockDim.x) {
            const float2 e = a.ewalk[i];
            ewl[i] = e;
            xkeep[i] = make_uint2(dc_canonical_at_least(e.x), dc_canonical_at_least(e.y));
        }
        return DcTabs{ewl, xkeep};
    }
    return DcTabs{nullptr, nullptr};
}

// One whole dense sweep by this workgroup as one of the grid's (every workgroup of the grid runs
// it for the same sweep): the update tasks, its spans of the evaluation, the arrival; the last
// workgroup to arrive commits. s4 = {t, done, x_t, err} as this workgroup read them. Returns
// whether this workgroup committed. (dc_eval_kernel: one per launch; dc_multi_kernel: its full
// sweeps, dense_sparse.h.) The caller has synchronised the workgroup after building `tb`.
template <int NW>
__device__ __forceinline__ bool dc_full_body(const SweepArgs& a, uint4 s4, DcTabs tb, uint32_t* dyn) {
    __shared__ TailShared sh;
    __shared__ DcCtl sh_ctl;
    DevState* __restrict__ st = a.st;
    if (threadIdx.x == 0) {
        sh.wg_viol = 0;
        sh.wg_ev = 0;
        sh.wg_last = 0;
        sh.viol = 0;
        dc_ctl_load(a, sh_ctl);
    }
    const uint32_t t = s4.x;
    const uint32_t x_t = s4.z;
    const uint32_t err0 = s4.w;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;
    uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;
    const uint32_t nloc = a.v_end - a.v_begin;
    uint8_t* const vf = a.vflags ? a.vflags + (size_t)(t & 1u) * nloc : nullptr;
    const float2* ew = tb.ew;
    const uint2* xkeep = tb.xkeep;
    uint32_t fullw[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) fullw[i] = dc_fullw(a.nCol, (uint32_t)i);
    __syncthreads();
    uint4* const dc_lds = reinterpret_cast<uint4*>(dyn);
    dc_update_tasks<NW>(a, t, reinterpret_cast<uint32_t*>(dc_lds), sh_ctl);
    // the list appends' stage (dc_lds is free between the update's histograms and the commit)
    __shared__ DcStage stg;
    {
        uint32_t* w = reinterpret_cast<uint32_t*>(dc_lds);
        for (uint32_t i = threadIdx.x; i < kDcStageChg + 2u * kDcStageS + kDcStageEv; i += blockDim.x) w[i] = ~0u;
        if (threadIdx.x == 0) {
            stg.n[0] = stg.n[1] = stg.n[2] = 0;
            stg.chg = w;
            stg.s = w + kDcStageChg;
            stg.ev = w + kDcStageChg + 2u * kDcStageS;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const uint32_t nwaves = blockDim.x >> 6;
    const uint32_t gw = blockIdx.x * nwaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), GW = gridDim.x * nwaves;
    const uint32_t nspan = (nloc + kDcSpan - 1u) / kDcSpan;
    const bool al16 = (a.v_begin & 15u) == 0u;   // 16-byte colour loads (else byte loads)
    uint32_t wave_viol = 0, wave_ev = 0, wave_open = 0, kept = 0;
    // 16807^16 (a row block of a lane), 16807^(16 lane), 16807^(1024 W) (a wave's next span)
    uint32_t a16 = kMinstdA;
#pragma unroll
    for (int i = 0; i < 4; i++) a16 = minstd_mulmod(a16, a16);
    uint32_t lp16 = 1u;
    for (uint32_t e = (uint32_t)lane, b = a16; e; e >>= 1, b = minstd_mulmod(b, b))
        if (e & 1u) lp16 = minstd_mulmod(lp16, b);
    uint32_t aspan = a.dc_apow;   // 16807^(64 W)
#pragma unroll
    for (int i = 0; i < 4; i++) aspan = minstd_mulmod(aspan, aspan);
    uint32_t xs = gw < nspan ? minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)a.v_begin + (uint64_t)kDcSpan * gw + 1ull)) : 0u;
    xs = __builtin_amdgcn_readfirstlane(xs);   // wave-uniform: the span powers run on the scalar unit
    // lane's rows of span S: l0 = S kDcSpan + 16 lane; colours as four words, open bits as 16 bits
#define DC_LOAD(CW, OPW, S)                                                                         \
    {                                                                                               \
        const uint32_t l0 = (S) * kDcSpan + kDcLaneRows * (uint32_t)lane;                           \
        const bool in = (S) < nspan && l0 < nloc;                                                   \
        const uint32_t nv = in ? min(kDcLaneRows, nloc - l0) : 0u;                                  \
        if (al16 && nv == kDcLaneRows) {                                                            \
            const uint4 q = *reinterpret_cast<const uint4*>(C + a.v_begin + l0);                    \
            CW[0] = q.x; CW[1] = q.y; CW[2] = q.z; CW[3] = q.w;                                     \
        } else {                                                                                    \
            CW[0] = CW[1] = CW[2] = CW[3] = 0u;                                                     \
            for (uint32_t j = 0; j < nv; j++) CW[j >> 2] |= (uint32_t)C[a.v_begin + l0 + j] << (8u * (j & 3u)); \
        }                                                                                           \
        unsigned long long o = 0;                                                                   \
        if (in) {                                                                                   \
            _Pragma("unroll") for (int i = 0; i < NW; i++) o |= a.dc_open[(size_t)(l0 >> 6) * NW + i]; \
        }                                                                                           \
        OPW = (uint32_t)(o >> (l0 & 63u)) & 0xFFFFu;                                                \
    }
#define DC_EVAL(CW, OPW, S)                                                                         \
    {                                                                                               \
        const uint32_t l0 = (S) * kDcSpan + kDcLaneRows * (uint32_t)lane;                           \
        const uint32_t nv = l0 < nloc ? min(kDcLaneRows, nloc - l0) : 0u;                           \
        const uint32_t vmask = (1u << nv) - 1u;                                                     \
        uint32_t tabw[kDcLaneRows];                                                                 \
        if (a.taboo != nullptr) {                                                                   \
            _Pragma("unroll") for (uint32_t j = 0; j < kDcLaneRows; j++)                            \
                tabw[j] = j < nv ? a.taboo[l0 + j] : 0u;                                            \
        }                                                                                           \
        const uint32_t xl = minstd_mulmod(xs, lp16);                                                \
        uint32_t keepm = 0;                                                                         \
        if (ew != nullptr) {                                                                        \
            uint32_t x = xl;                                                                        \
            _Pragma("unroll") for (uint32_t j = 0; j < kDcLaneRows; j++) {                          \
                if (j) x = dc_mul16807(x);                                                          \
                const uint32_t cv = (CW[j >> 2] >> (8u * (j & 3u))) & 0xFFu;                        \
                const uint2 xk = xkeep[cv];   /* u >= E[cv] && S[cv] > u, as states */              \
                bool k = x >= xk.x && x < xk.y;                                                     \
                if (a.taboo != nullptr) k = k && tabw[j] == 0u;                                     \
                keepm |= (k ? 1u : 0u) << j;                                                        \
            }                                                                                       \
            keepm &= vmask & ~(OPW);                                                                \
            kept += (uint32_t)__popc(keepm);                                                        \
            if (keepm != 0u && (vf != nullptr || a.taboo != nullptr)) {                             \
                for (uint32_t j = 0; j < kDcLaneRows; j++) {                                        \
                    if (!((keepm >> j) & 1u)) continue;                                             \
                    if (vf != nullptr) vf[l0 + j] = 1u;                                             \
                    if (a.taboo != nullptr) a.taboo[l0 + j] = a.tabooIteration;                     \
                }                                                                                   \
            }                                                                                       \
        }                                                                                           \
        const uint32_t need = vmask & ~keepm;                                                       \
        if (__ballot(need != 0u)) {                                                                 \
            for (uint32_t j = 0; j < kDcLaneRows; j++) {                                            \
                const bool nd = ((need >> j) & 1u) != 0u;                                           \
                if (!__ballot(nd)) continue;                                                        \
                const uint32_t l = l0 + j;                                                          \
                const uint32_t cv = nd ? (uint32_t)C[a.v_begin + l] : 0u;                           \
                const uint32_t tab = (nd && a.taboo != nullptr) ? a.taboo[l] : 0u;                  \
                const bool opn = nd && ((OPW >> j) & 1u) != 0u;                                     \
                DcMask<NW> m, fw;                                                                   \
                _Pragma("unroll") for (int i = 0; i < NW; i++) {                                    \
                    m.w[i] = opn ? a.dc_mask[(size_t)l * NW + i] : fullw[i];                        \
                    fw.w[i] = fullw[i];                                                             \
                }                                                                                   \
                const uint64_t ob = __ballot(opn);                                                  \
                if (ob) {                                                                           \
                    wave_open += (uint32_t)__popcll(ob);                                            \
                    const DcScan ds{a.tseg, a.gbase, a.tcol, a.grp_rows, a.nblocks, a.block_log2, a.dc_s0, a.dc_s1}; \
                    m = dc_open_scan<NW>(ds, C, l, opn, m, fw, lane);                               \
                }                                                                                   \
                uint32_t acc[NW];                                                                   \
                _Pragma("unroll") for (int i = 0; i < NW; i++) acc[i] = m.w[i];                     \
                wave_viol += evaluate_lane<NW>(a, st, Cs, nd, l, acc, lane, wave_ev, vf, cv, tab,   \
                                               minstd_mulmod(xl, kMinstdLanePow[j]), ew, &stg);     \
            }                                                                                       \
        }                                                                                           \
        xs = minstd_mulmod(xs, aspan);                                                              \
    }
    uint32_t cA[4], cB[4], oA, oB;
    uint32_t sp = gw;
    DC_LOAD(cA, oA, sp)
    while (sp < nspan) {
        DC_LOAD(cB, oB, sp + GW)
        DC_EVAL(cA, oA, sp)
        sp += GW;
        if (sp >= nspan) break;
        DC_LOAD(cA, oA, sp + GW)
        DC_EVAL(cB, oB, sp)
        sp += GW;
    }
#undef DC_LOAD
#undef DC_EVAL
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o, 64);
    wave_viol += kept;   // every kept row is a violator: its own colour is in the full mask
    if (wave_open) {   // statistics; the commit reads the word (this workgroup releases)
        if (lane == 0) atomicAdd(&a.dc_ctl[kDcOpen], wave_open);
        wave_ev = 1u;
    }
    __syncthreads();   // every wave's stage entries are in
    if (dc_stage_flush(a, st, stg, t)) wave_ev = 1u;
    __syncthreads();   // ewl's and the stage's last readers are done before the commit may reuse LDS
    sweep_tail(a, st, sh, wave_viol, wave_ev, lane, reinterpret_cast<uint32_t*>(dc_lds), a.lds_sort_cap, t, err0);
    return sh.wg_last != 0u;
}

template <int NW>
__global__ __launch_bounds__(1024) void dc_eval_kernel(SweepArgs a) {
    extern __shared__ uint4 dc_lds[];
    __shared__ float2 ewl[256];
    __shared__ uint2 xkeep[256];
    const uint4 s4 = *reinterpret_cast<const uint4*>(a.st);   // {t, done, x_t, err}: one load
    if (a.check_done && s4.y) return;
    const DcTabs tb = dc_tabs_load(a, ewl, xkeep);
    (void)dc_full_body<NW>(a, s4, tb, reinterpret_cast<uint32_t*>(dc_lds));
}

template <int NW>
void launch_dc(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    dc_eval_kernel<NW><<<g, b, lds, s>>>(a);
}
template <int NW>
hipError_t allow_lds_dc(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&dc_eval_kernel<NW>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
