// mcmc_colorer_amd/csrc/wide_tiled.h -- the wide sweep (nCol > 256, uint16 colours) over the tiled
// layout, for graphs that have no CSR: the build's generated G(n, p) at C3 size, where the
// reference's default colour count nCol = maxDeg (main.cu:162; about 10 500 at C3) applies and a
// CSR (4e11 B of uint32 ids) cannot exist beside the 2.2e11 B layout on one device. Included by
// mcmc_sweep.hip inside namespace mcmc, after sweep_wide.h.
//
// One wave per row, persistent (rows w, w + W, ... for the grid's W waves). The row's occupancy
// mask (count_free_colors, coloringMCMC_CPU.cpp:362-383: nCol bits) is built in the wave's own LDS
// words by scanning its segments of every column block of the layout (16-bit block-local ids; 4
// blocks per round, 16 lanes and 8 ids per lane in flight), the neighbours' colours gathered from
// the uint16 replica of C_t. Then, per the row's own colour and taboo counter:
//   taboo        the colour stays, the counter drops (:496-501);
//   violator     fill_p case (ii) or (i) and the exact CDF walk over the mask (walk_finish_wave:
//                word prefix counts, walk_mask_pre -- the wide sweep's violator walk);
//   otherwise    case (iii): own colour hi, others eps -- walk_own_tab over the eps prefix table.
// CDF overflows are appended to the event list; the stand-alone commit (commit_kernel<uint16_t>)
// replays them in ascending vertex order against glibc (:517-520) and runs the loop control.
// Every arc is read every sweep (the scan cannot stop early: a row without its own colour must
// see every neighbour), so a sweep moves the whole layout (2 B per arc) plus one 2-byte colour
// gather per arc from the replica (20 MB at C3: MALL-resident) -- exact, not fast: the dense and
// persistent sweeps of nCol <= 256 do not apply to masks of 10 000 colours.

// Waves per workgroup (8, or fewer when one wave's mask + prefix counts -- 2 NWW + 1 words -- make
// 8 of them exceed 144 KiB) and workgroups per CU: 24 waves per CU (the kernel's ~74 VGPRs allow 6
// per SIMD), as the LDS allows. Many waves in flight: a row's scan is a chain of dependent loads.
inline uint32_t wide_tiled_waves(uint32_t nCol) {
    const uint32_t nww = (nCol + 31u) >> 5;
    const uint32_t per = 4u * (2u * nww + 1u);
    uint32_t w = 8;
    while (w > 1 && (size_t)w * per > 144u * 1024u) w >>= 1;
    return w;
}
inline uint32_t wide_tiled_wgs_per_cu(uint32_t nCol) {
    const uint32_t W = wide_tiled_waves(nCol), per = 4u * (2u * ((nCol + 31u) >> 5) + 1u);
    return std::max<uint32_t>(1u, std::min<uint32_t>(24u / W, (uint32_t)((160u * 1024u) / ((size_t)W * per))));
}

__global__ __launch_bounds__(512) void wide_tiled_kernel(SweepArgs a) {
    extern __shared__ uint32_t wt_lds[];
    __shared__ uint32_t sh_viol;
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (threadIdx.x == 0) sh_viol = 0;
    __syncthreads();
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin, NWW = (a.nCol + 31u) >> 5;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t* const mask = wt_lds + (size_t)wave * (2u * NWW + 1u);
    uint32_t* const pre = mask + NWW;
    const uint32_t R = a.grp_rows, nb = a.nblocks, bl = a.block_log2;
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    uint32_t wave_viol = 0, nrows = 0;
    // Block rotation: a row's mask is an OR, so its blocks may be scanned in any cyclic order. Each
    // row starts at the block a common clock points to (one block per tick, the tick measured on
    // the previous sweep), so all waves gather from a narrow window of colour slices at any time --
    // one XCD's L2 holds it, where the 2 B x n replica (20 MB at C3) does not fit.
    const unsigned long long tick = a.wt_tick != nullptr ? *a.wt_tick : 0ull;
    const unsigned long long t_begin = wall_clock64();
    for (uint32_t l = blockIdx.x * nwv + wave; l < nloc; l += gridDim.x * nwv) {
        const uint32_t v = a.v_begin + l;
        for (uint32_t i = lane; i < NWW; i += 64u) mask[i] = 0u;
        wave_lds_sync();
        const uint32_t g = l / R, r = l - g * R;
        const uint16_t* __restrict__ gc = a.tcol + a.gbase[g];
        uint64_t deg = 0;
        const uint32_t bs = tick ? (uint32_t)((wall_clock64() / tick) % nb) : 0u;
        nrows++;
        for (uint32_t b0 = 0; b0 < nb; b0 += 4u) {
            const uint32_t bi = b0 + grp;
            const uint32_t b = bi + bs < nb ? bi + bs : bi + bs - nb;
            uint32_t s0 = 0, s1 = 0;
            if (bi < nb) {
                const uint32_t* ts = a.tseg + ((size_t)g * nb + b) * tseg_stride(R);
                const uint32_t raw = ts[r];
                s0 = raw & kTsegPos;
                s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
            }
            if (gl == 0 && s1 > s0) deg += s1 - s0;
            const uint32_t lo = b << bl;
            for (uint32_t k = s0 + gl; __ballot(k < s1); k += 128u) {
                uint32_t c[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const uint32_t kk = k + 16u * q;
                    c[q] = kk < s1 ? (uint32_t)C[lo | gc[kk]] : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (c[q] != 0xFFFFFFFFu) atomicOr(&mask[c[q] >> 5], 1u << (c[q] & 31u));
            }
        }
        for (int o = 32; o > 0; o >>= 1) deg += __shfl_xor(deg, o, 64);
        wave_lds_sync();
        const uint32_t cv = C[v];
        const uint32_t tab = a.taboo != nullptr ? a.taboo[l] : 0u;
        const uint32_t viol = (mask[cv >> 5] >> (cv & 31u)) & 1u;
        wave_viol += viol;
        if (a.vflags != nullptr && lane == 0) a.vflags[(size_t)(t & 1u) * nloc + l] = (uint8_t)viol;   // tail cut
        // u_v: engine draw K_t + v + 1 (coloringMCMC_CPU.cpp:139)
        const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)v + 1ull));
        if (tab > 0) {   // :496-501
            if (lane == 0) {
                Cs[v] = (uint16_t)cv;
                a.taboo[l] = tab - 1u;
            }
        } else if (viol) {   // case (ii) / (i): the walk over the mask (writes Cs, taboo, the event)
            walk_finish_wave<false>(a, v, t, cv, x, (uint32_t)min(deg, (uint64_t)0xFFFFFFFFu), Cs, mask, pre, nullptr, nullptr,
                             lane);
        } else if (lane == 0) {   // case (iii)
            const uint32_t nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, minstd_canonical(x));
            const bool event = nc == a.nCol;
            Cs[v] = (uint16_t)(event ? cv : nc);
            if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
            if (event) {
                const uint32_t idx = atomicAdd(&st->ev_count, 1u);
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, 1u);
            }
        }
        wave_lds_sync();   // the walk's LDS reads are done before the next row clears the mask
    }
    if (lane == 0 && wave_viol) atomicAdd(&sh_viol, wave_viol);
    if (a.wt_tick != nullptr && blockIdx.x == 0 && threadIdx.x == 0 && nrows > 0) {   // next sweep's tick
        const unsigned long long d = (wall_clock64() - t_begin) / ((unsigned long long)nrows * nb);
        *a.wt_tick = d > 0 ? d : 1ull;
    }
    __syncthreads();
    if (threadIdx.x == 0 && sh_viol) atomicAdd(&st->viol, (unsigned long long)sh_viol);
}

void launch_wide_tiled(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    wide_tiled_kernel<<<g, b, lds, s>>>(a);
}
