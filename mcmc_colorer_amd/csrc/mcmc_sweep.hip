// mcmc_colorer_amd/csrc/mcmc_sweep.hip -- the MCMC colour-resampling sweep for gfx950.
//
// Replaces the reference's per-sweep kernel chain (graph_coloring/coloringMCMC_main.cu:160-269:
// conflictCounter + sumReduction twice, a host histogram round trip, genDynamicDistribution,
// selectStarColoringBalanceDynamic) with ONE fused kernel per sweep plus a one-workgroup commit
// kernel, and implements the --mcmccpu semantics bit-exactly:
//
//   sweep_kernel   one neighbour scan per vertex builds the occupancy mask of the colours of N(v)
//                  (count_free_colors, coloringMCMC_CPU.cpp:362-383); viol_v = own colour
//                  occupied (violation_count, :329-351); p(c) in fp32 (fill_p, :393-481);
//                  u_v = minstd draw K_t + v + 1 by skip-ahead (:139); CDF walk with strict >
//                  (extract_new_color, :493-528); Cstar, taboo; Cviol_t by ballot/popcount;
//                  CDF overflows appended to an event list.
//   commit_kernel  loop control of run() (:136, :264-269): records Cviol_t, stops on
//                  Cviol_t <= z or the maxRip cap, otherwise replays overflow events in ascending
//                  vertex order against the glibc rand() window (`rand() % (nCol-1)`, :518),
//                  advances the minstd position by n and flips the colour buffers.
//
// The loop is device-resident: both kernels read the sweep index and RNG position from DevState,
// so a batch of (sweep, commit) pairs is captured once into a hipGraph and replayed until the
// commit kernel raises `done`. No host synchronisation inside a batch.
//
// Compiled with -ffp-contract=off: fill_p's products and quotients must round exactly as the
// reference's SSE code (no FMA), and fp32 division stays IEEE-correct (hipcc default).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "cdf_walk.h"
#include "mcmc_common.h"
#include "rng.h"
#include "xorwow.h"

namespace mcmc {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// ----------------------------------------------------------------------------------------------
// Device-resident loop state (one per context).
constexpr uint32_t kDevErrEvents = 1u, kDevErrWatchdog = 2u;   // DevState::err bits
struct DevState {
    uint32_t t;                 // sweep index == ColoringMCMC_CPU::iter
    uint32_t done;              // loop finished (set by commit)
    uint32_t x_t;               // minstd state after K0 + t*n draws
    uint32_t err;               // kDevErrEvents: event list overflow; kDevErrWatchdog: a persistent
                                // launch's phase did not complete in time (workgroups not resident)
    unsigned long long viol;    // sum of viol_v over the swept rows (Cviol_t)
    uint32_t ev_count;          // overflow events this sweep
    uint32_t arrive;            // workgroups finished with the running sweep (fused commit)
    unsigned long long arrive_viol;   // packed fused arrival: [63:48] workgroups arrived,
                                      // [47:32] workgroups that appended events, [31:0] Cviol
    uint32_t glibc_head;        // ring head of the glibc window
    uint32_t glibc_ring[31];
    uint32_t init_rejections;
    unsigned long long glibc_draws;
    unsigned long long finalViol;
    uint32_t iter;
    uint32_t maxIterReached;
    uint32_t lx;                // discrete log of x_t base 16807 (rng.h minstd_dlog): x_t = 16807^lx
};

struct SweepArgs {
    const uint64_t* row_off;    // local rows: row_off[v - v_begin], length (v_end - v_begin) + 1
    const uint64_t* row_off_g;  // the whole graph's offsets (row_off_g[v], any v): the wide sweep's
                                // partitioned incremental counts read other ranks' rows
    const uint32_t* col_idx;    // global vertex ids
    uint8_t* colors0;           // full-length colour replicas (C_t lives in colors[t & 1])
    uint8_t* colors1;
    uint32_t* taboo;            // local rows, nullptr when tabooIteration == 0
    uint32_t* events;           // overflow event list (global vertex ids)
    uint32_t* evdraw;           // the events' rand() draws (commit scratch, ev_cap entries)
    DevState* st;
    unsigned long long* traj;   // per-sweep Cviol, traj_cap entries
    uint32_t traj_cap;
    uint32_t ev_cap;
    uint32_t n, v_begin, v_end;
    uint32_t nCol, tabooIteration, maxRip, z;
    uint32_t tile;              // vertices per wave-tile (<= 64)
    const uint32_t* wave_start; // arc-balanced static partition: wave w sweeps local rows
                                // [wave_start[w], wave_start[w+1])
    uint32_t aN;                // 16807^n mod (2^31-1): minstd advance per sweep
    float eps, hi;              // epsilon and 1 - (nCol-1)*epsilon (fill_p, :406)
    float emax;                 // wide: E[nCol - 1], the largest eps prefix (walk_own_tab_e fast path)
    const uint16_t* ftab;       // wide: F(u) = first k with E[k] > u, for u = i 2^-31 < emax, i < ftab_n
    uint32_t ftab_n;
    int check_done;             // device-resident loop: exit immediately once done
    int fused;                  // last-arriving workgroup: 1 = runs the commit (single-context loop),
                                //                          2 = packs this rank's footer (partitioned)
    uint32_t world;
    uint32_t lds_sort_cap;      // words of the sweep kernel's dynamic LDS reusable by the commit sort
    int olist_on;               // tiled early exit: the LDS holds an R-entry open-row list (listed pairs)
    // tiled early exit, tail queue (tq_dense > 0): a group's blocks [0, tq_dense) run as pairs; its
    // rows still open then wait in this workgroup's queue (global) and finish block by block after
    // the workgroup's last group, rows of all its groups together (tile_tail)
    uint32_t tq_dense;
    uint32_t tq_cap;            // queue entries per workgroup and queue
    uint32_t* tq_l;             // [grid][2][tq_cap][3] local row, its u_v minstd state, own colour | taboo << 8
    uint32_t* tq_m;             // [grid][2][tq_cap][NW] their occupancy masks
    uint32_t eown_off;          // tiled early exit: LDS byte offset of the evaluated group's own colours (0: none)
    // the own-colour walk in closed form (fill_p cases (i)/(iii)): ewalk[c] = {E[c], fl(E[c] + hi)} with
    // E[c] the c-fold fp32 sum of eps; nullptr where the host found the form inexact (ewalk_table)
    const float2* ewalk;
    uint32_t ewalk_off;         // tiled: LDS byte offset of its copy (0: none)
    const uint32_t* seg;        // blocked: per-(block, local row) segment offsets, (nb+1) x nloc
    uint32_t nblocks;           // blocked: column blocks of 2^block_log2 vertices
    uint32_t block_log2;        // blocked: log2 of the column block (17: 128 KiB of uint8 colours)
    uint32_t chunk_rows;        // blocked: rows whose masks a workgroup keeps in LDS at once
    // tiled layout (variant 3): rows in groups of grp_rows; per group, arcs block-major, 16-bit
    // block-local ids, every (row, block) segment padded to a multiple of 8 ids
    const uint16_t* tcol;
    const uint64_t* gbase;      // [ngroups + 1] group start in tcol (ids)
    const uint32_t* tseg;       // [ngroups][nblocks][grp_rows + 1] segment start relative to gbase
    uint32_t grp_rows, ngroups;
    uint32_t sub_log2;          // lanes per row segment = 2^sub_log2
    uint32_t slice_bytes;       // tiled: colour bytes a pair's slice can hold (resident: the replica)
    uint32_t seg_buf_bytes;     // tiled: LDS bytes of one segment-table buffer (1 KiB multiple)
    unsigned long long* phase_ts;   // diagnostics (MCMC_PHASE_DUMP): per-workgroup phase timestamps
    unsigned long long* pair_trace; // diagnostics (MCMC_PAIR_TRACE): per workgroup and pair, kPairTraceRec words
    // partitioned runs: colour replicas stay in vertex order; every rank's footer (kFooterWords:
    // local Cviol, event count, flags, sorted events) sits in slot `rank` of the footer buffer of
    // the next-colour parity (sweep t: foot[(t + 1) & 1], like colors[(t + 1) & 1])
    uint32_t* foot0;
    uint32_t* foot1;
    uint32_t rank;
    // tail cutting enabled (mcmc_set_tailcut_repair): sweep t stores the violation flags of C_t at
    // vflags[(t & 1) * nloc + l] -- the tail cut's first pass needs those of the previous sweep
    uint8_t* vflags;
    // reference-GPU-semantics mode (REF instantiations of the tiled sweep, refmode.hip)
    uint32_t* xw0;              // XORWOW states of sweep parity 0 / 1: SoA {v0..v4, d} x nloc
    uint32_t* xw1;
    uint32_t* hist;             // [2][hist_words] colour histograms of C_t by parity (C_t[v] <= nCol)
    uint32_t hist_words;        // kHistWords (uint8 REF), nCol + 1 rounded up (REF wide, ref_wide.h)
    float ref_hi;               // 1 - (nCol - 1) * eps (coloringMCMC_balance.cu:132)
    uint32_t* rw_cnt;           // REF wide: [4] list lengths (ref_wide.h kRw*)
    uint32_t* rw_lists;         // REF wide: [4][n] listed violators / long rows
    float* ptab;                // REF wide: p of every colour for the running sweep (genDynamicDistribution)
    uint32_t own_buf_bytes;     // streaming REF: LDS bytes of one own-colour buffer
    // wide sweep (nCol > 256, uint16 replicas; sweep_wide.h)
    uint64_t arc_begin, arc_count;   // the local rows' arcs: col_idx[arc_begin, arc_begin + arc_count)
    const uint32_t* chunk_row;  // [nchunks + 1] first local row of every 256-arc chunk
    uint32_t nchunks;
    uint8_t* wflag;             // [nloc] viol flags of the running sweep (cleared by the evaluation)
    uint8_t* wfp0;              // wide LDS scan: [n] colour fingerprints (low byte) of colors0 / colors1
    uint8_t* wfp1;
    int fp_live;                // 1: the sweep's writers keep the next colouring's fingerprints (no wide_fp_kernel)
    uint32_t* wlist;            // [2][nloc] violating, untaboo'd vertices (global ids), split-walk slot
    uint32_t* wcount;           // [4]: violators, -, extra split-walk tasks, slots taken (sweep_wide.h)
    uint32_t* gmask;            // wide: [kSplitMax][kWideMaskWords] occupancy of split walks (zero between sweeps)
    uint32_t* gdone;            // wide: [3][kSplitMax] tasks counted per split walk (zero between sweeps), list index, xbase
    uint32_t split_arcs;        // wide: arcs per task of a split walk
    uint32_t walk_light;        // wide: a violator of at most this many arcs is walked by one wave
    uint32_t walk_tie;          // wide: tie binades by word functions (walk_mask_pre tie_scan; MCMC_WALK_TIE=1)
    int bench;                  // throughput mode (mcmc_bench_*): no convergence stop
    // tiled sweep: stop scanning a row once its occupancy mask holds every colour (count_free_colors
    // cannot change any more: the sweep's results are unchanged); 0 = scan every arc (A/B runs)
    int early;
    uint32_t drain_rows;        // tiled early exit: a group with at most this many rows left drains them (<= 256)
    // tiled early exit: a group's next pair (its next block) is staged at the END of the current
    // pair's scan, and only while some row is still open (rows expected to fill inside a block: C2)
    int late_stage;
    unsigned long long* scan_stats;   // diagnostics (MCMC_SCAN_STATS): [0] quads loaded, [1] pairs staged,
                                      // [2] quads whose ids were gathered (the scan needed them)
    const float* etab;          // wide: E[k] = k-fold fp32 sum of eps, k = 0..nCol (walk_own_tab)
    uint32_t* evblk;            // wide: per evaluation workgroup, its overflow events ascending [nblk][kEvSlot]
    uint32_t* evcnt;            // wide: their number per workgroup [nblk] (written every sweep)
    uint32_t evnblk;            // wide: evaluation workgroups
    const uint32_t* evpow;      // wide: [evnblk][4] 16807^(v + 1) of each evaluation wave's first vertex
    const uint32_t* gpow;       // tiled: [ngroups][16] 16807^(v_begin + g R + 64 w + 1) (u_v of wave w's first row)
    uint32_t apow_grid, apow_tile;   // tiled: 16807^(gridDim R), 16807^(64 * 16)
    uint32_t a256;              // 16807^256 mod (2^31 - 1)
    // wide: XCD-slab edge layout of the violation scan (sweep_wide.h, get_xslab); xs_ent == nullptr
    // -> the CSR arc scan
    const uint32_t* xs_ent;     // [xs_chunk0[8] * 256] entries (row delta << cbits | slab-local column)
    const uint32_t* xs_base;    // [xs_chunk0[8]] first local row of every chunk
    const uint32_t* xs_chunk0;  // [nslabs + 1] first chunk of every slab
    const uint32_t* xs_pieces;  // LDS mode: [npieces][3] {slab, c0, c1} grouped by workgroup
    const uint32_t* xs_wgp;     // LDS mode: [workgroups + 1] first piece of every workgroup
    uint32_t xs_mode;           // 0: L2 slabs (wide_xscan_kernel), 1: LDS tiles (wide_tscan_kernel)
    uint32_t xs_S, xs_cbits;    // slab width (vertices), bits of the slab-local column
    uint32_t xs_nwg;            // LDS mode: workgroups of the scan launch
    uint32_t xs_sym;            // 1: one entry per local edge, flags both ends; 0: every arc, flags its row
    // partitioned delta exchange (native driver, multi.hip): this rank's delta slots of parity 0 / 1
    // ([0] pairs appended, [1] 0, then (v, c) pairs); dcap > 0: the sweep appends (delta mode)
    uint32_t* dlt0;
    uint32_t* dlt1;
    uint32_t dcap;
    const uint32_t* dall0;      // commit: every rank's slots of parity 0 / 1 (world x kDeltaWords)
    const uint32_t* dall1;
    int part_delta;             // commit: 1 delta mode (remote changes arrive as pairs, applied to both
                                //   replicas), 0 full mode, -1 full-mode resumption of a paused sweep
    // wide sweep, incremental violation counts (sweep_wide.h, wide_inc_*; a whole-graph context over a
    // symmetric CSR without repeated arcs, LDS tile scan): nullptr = every sweep's tile scan flags.
    // The writers of sweep t list the rows they change (C_t -> C_t+1) in lists of parity q = (t+1) & 1,
    // each in its own slot (no shared counter: a device-scope atomic on one word serialises at ~90
    // per us): evaluation workgroup eb in eslot[q][eb], walk workgroup b in wslot[q][b], the commit in
    // cchg[q]; rows above inc_hub_arcs arcs in hub[q] (rare; one atomic each). A slot holds its count and
    // the rows' arcs in its first two words. The evaluation also lists the violators of C_t it saw
    // (vslot[p][eb], p = t & 1): the next sweep's flag pass starts from them.
    uint32_t* inc;              // [kIncWords] control words
    uint32_t* inc_vcnt;         // [nloc] same-colour arcs of every row in C_t
    uint32_t* inc_hub;          // [2][inc_lcap] changed rows above inc_hub_arcs arcs (global ids)
    uint32_t* inc_tch;          // [2][nloc] rows whose count left 0 in sweep t's delta pass
    uint32_t* inc_eslot;        // [2][evnblk][2 + inc_slot] evaluation workgroups' changed rows
    uint32_t* inc_vslot;        // [2][evnblk][2 + inc_slot] evaluation workgroups' violators of C_t
    uint32_t* inc_wslot;        // [2][kWalkBlocks][2 + inc_wslot_n] walk workgroups' changed rows
    uint32_t* inc_cchg;         // [2][2 + inc_ccap] the commit's changed rows (a slot; global ids)
    uint32_t* inc_dense;        // [2][inc_lcap] every changed row but the hubs (global ids), gathered by
                                //   the commit: this rank's, the event replay's, other ranks' (delta mode)
    uint32_t inc_lcap;          // entries of those lists: n (changed rows of a sweep are distinct vertices)
    uint32_t inc_ccap;          // entries of the commit's slot inc_cchg (the replayed events of every rank: n)
    uint32_t* inc_hdr;          // [2][evnblk + kWalkBlocks][2] the slots' headers again, side by side (the
                                //   commit reads them all: one workgroup's loads, ~64 GB/s per CU)
    uint32_t inc_slot, inc_wslot_n;   // rows per evaluation / walk slot (past it: the next sweep recounts)
    uint32_t inc_hub_arcs;      // a changed row above this many arcs is a hub (MCMC_WIDE_INC_HUB)
    unsigned long long inc_thresh;    // the next sweep is incremental while its changed rows' arcs stay <= this
    // dense-count sweep (dense_counts.h; tiled contexts): per local row the counts of the colours of
    // its neighbours in the dense column range [dc_s0, dc_s1) and their occupancy bits
    uint32_t* dc_ctl;           // kDcWords control words (nullptr: the tiled scan sweeps)
    uint32_t* dc_cnt;           // [nloc][dc_cw] uint32 counts
    uint32_t* dc_mask;          // [nloc][NW] occupancy of the counts
    uint32_t* dc_list;          // [2][dc_cap] (v, old colour << 16 | new colour): the vertices of S
                                //   whose colour changed, by parity (t + 1) & 1
    uint32_t* dc_chg;           // [2][dc_chg_cap] every local vertex whose colour changed (restore list)
    unsigned long long* dc_open;   // [ntiles][NW] bit j of word (tile, i): row 64 tile + j's mask word i not full
    uint32_t dc_s0, dc_s1, dc_cw, dc_cap, dc_max, dc_chg_cap;
    uint32_t dc_rbrows;         // rows per chunk of the streaming count rebuild (0: a wave per row)
    uint32_t dc_rbl;            // 1: the lane rebuild (dense_counts.h dc_rebuild_lanes; nCol <= 32)
    uint32_t dc_planes;         // its bit planes per count (counts < 2^dc_planes; 4..16)
    const uint4* dc_tid;        // the lane rebuild's copy of S's ids, tile-transposed (dense_counts.h), or nullptr
    const uint64_t* dc_toff;    // [ceil(nloc / 64)] tile t's first quad in dc_tid
    uint32_t dc_poll;           // persistent dense sweep: s_sleep(4) rounds between a helper's polls (MCMC_DC_POLL)
    uint32_t dc_commit_restore;  // restore lists up to this long are applied by the commit
    uint32_t dc_apow;           // 16807^(64 x the evaluation's waves): u_v advance per tile
    // open summary (dense_counts.h dc_osum_note): word 0's low half = open words that are nonzero;
    // then one bit per open word (its index (row >> 6) NW + mask word), set while it is nonzero
    unsigned long long* dc_osum;
    // the persistent dense sweep's candidate window (dense_sparse.h): every minstd state w whose draw
    // may move a closed row, with its discrete log: {L(w), w}, dl_n entries
    const uint2* dl_tab;
    uint32_t dl_n;
    unsigned long long* solo_ts;    // diagnostics (MCMC_SOLO_TRACE): the leader's stamps, [sweep of the launch][8]
    unsigned long long* wt_tick;    // wide tiled sweep: clock ticks per block step of the last sweep (0: none yet)
    uint32_t* wt_ctl;           // wide tiled sweep, incremental counts (wide_tiled.h): kWtWords control words
    uint32_t* wt_vcnt;          // [nloc] neighbours of the row's own colour in C_t
    uint32_t* wt_deg;           // [nloc] the row's arcs (counted by the full sweep)
    uint32_t* wt_list;          // [2][nloc] violators of the running sweep, then rows changed by it
    uint8_t* wt_chg;            // [nloc / 8 + 2] rows changed by the last sweep, a bit each (8-row groups of global v)
    uint32_t wt_rc;             // a full sweep = wt_recount_kernel + the incremental kernels (wide_tiled.h)
    uint32_t nmodN;             // n mod (2^31 - 2): the advance of DevState::lx per sweep
};
// control words of the incremental wide sweep (SweepArgs::inc)
constexpr uint32_t kIncMode = 0;     // the running sweep: 1 full (the tile scan recounts), 0 incremental
constexpr uint32_t kIncOvf = 1;      // [2] a slot overflowed (by parity q): the next sweep recounts
constexpr uint32_t kIncTch = 3;      // [2] counts that left 0, by parity of t
constexpr uint32_t kIncTchOvf = 5;   // [2] the touched list overflowed (the flag pass visits every row)
constexpr uint32_t kIncHubN = 7;     // [2] changed hubs, by parity q
constexpr uint32_t kIncDenseN = 9;   // [2] rows in the dense list, by parity q
constexpr uint32_t kIncStat = 16;    // u64 [4]: incremental sweeps, full sweeps, changed rows, their arcs
constexpr uint32_t kIncWords = 24;
#ifndef MCMC_WALK_BLOCKS
#define MCMC_WALK_BLOCKS 1024   // walk workgroups of the wide evaluation launch (sweep_wide.h kWalkBlocks)
#endif
constexpr uint32_t kIncWalkSlots = MCMC_WALK_BLOCKS;   // one changed-row slot per walk workgroup

// control words of the dense-count sweep (SweepArgs::dc_ctl; dense_counts.h)
constexpr uint32_t kDcMode = 0;    // the running sweep's update: 1 rebuild every count, 0 incremental
constexpr uint32_t kDcLen = 1;     // [2] vertices of S listed for the next sweep's update, by parity (t + 1) & 1
constexpr uint32_t kDcOvf = 3;     // [2] that list overflowed: the next sweep rebuilds
constexpr uint32_t kDcOpen = 5;    // rows of the running sweep whose dense mask was not full
constexpr uint32_t kDcStat = 8;    // u64 [4]: incremental sweeps, rebuilds, listed vertices, open rows
constexpr uint32_t kDcChgLen = 16; // [2] local vertices on the restore list, by parity (t + 1) & 1
constexpr uint32_t kDcChgOvf = 18; // [2] that list overflowed: the next update copies every local row
constexpr uint32_t kDcCommitRestore = 8192;   // restore lists up to this long: applied by the commit
                                               // (at most half the list's capacity)
constexpr uint32_t kDcTask = 20;   // the running sweep's update tasks claimed (dense_counts.h dc_update_tasks)
constexpr uint32_t kDcDone = 21;   // and completed
constexpr uint32_t kDcStat2 = 22;  // u32 [2]: rows on the restore lists (saturating), restore-list overflows
// the persistent dense sweep (dense_sparse.h dc_multi_kernel); the leader resets them before it returns
constexpr uint32_t kDcGen = 24;    // the leader's posted phase: seq << 2 | kind (1 full sweep, 2 exit)
constexpr uint32_t kDcAck = 25;    // helpers that saw the exit
constexpr uint32_t kDcCommitted = 26;   // full sweeps committed in this launch
constexpr uint32_t kDcSoloStat = 28;    // u64: sweeps the leader ran alone (solo), statistics
constexpr uint32_t kDcSoloEval = 30;    // u64: rows those sweeps evaluated (candidates + open rows)
constexpr uint32_t kDcMvDone = 32;      // the persistent sweep's move phases: workgroup tasks completed
constexpr uint32_t kDcMvN = 33;         // the posted move phase: vertices of S moved
constexpr uint32_t kDcMvList = 34;      // and their (v, a << 16 | b), 16 pairs at most
constexpr uint32_t kDcWords = 72;
constexpr uint32_t kDcEvalLds = 64u * 1024u;   // the dense sweep's LDS scratch: stage, commit sort buffer
constexpr uint32_t kDcRebuildLds = 2u * kDcEvalLds;   // + the streaming rebuild's colour slice (dc_eval_kernel's dynamic LDS)


// The commit's bookkeeping of sweep t (thread 0, after the event replay listed its vertices of S):
// statistics, list t & 1 (read by this sweep's update) emptied for sweep t + 1's writers, and the
// mode of sweep t + 1's update -- a rebuild when list (t + 1) & 1 overflowed or holds more
// vertices than an incremental update pays for (dc_max).
// The dense sweep's control words the commit reads (thread 0, loaded together).
struct DcCommitWords {
    uint32_t chg, chg_ovf, len, ovf, open, mode;
};
__device__ __forceinline__ DcCommitWords dc_commit_load(const SweepArgs& a, uint32_t q) {
    const uint32_t* k = a.dc_ctl;
    DcCommitWords w;
    w.chg = __hip_atomic_load(&k[kDcChgLen + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.chg_ovf = __hip_atomic_load(&k[kDcChgOvf + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.len = __hip_atomic_load(&k[kDcLen + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.ovf = __hip_atomic_load(&k[kDcOvf + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.open = __hip_atomic_load(&k[kDcOpen], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w.mode = k[kDcMode];
    return w;
}
__device__ __forceinline__ void dc_commit(const SweepArgs& a, uint32_t t, const DcCommitWords& w) {
    uint32_t* k = a.dc_ctl;
    const uint32_t p = t & 1u;
    unsigned long long* s = reinterpret_cast<unsigned long long*>(k + kDcStat);
    s[0] += w.mode ? 0ull : 1ull;
    s[1] += w.mode ? 1ull : 0ull;
    s[2] += min(w.len, a.dc_cap);
    s[3] += w.open;
    k[kDcOpen] = 0;
    k[kDcLen + p] = 0;
    k[kDcOvf + p] = 0;
    k[kDcChgLen + p] = 0;
    k[kDcChgOvf + p] = 0;
    k[kDcTask] = 0;
    k[kDcDone] = 0;
    k[kDcMode] = (w.ovf || w.len > a.dc_max) ? 1u : 0u;
}

// Vertex v changed colour (ca -> cb) in the sweep whose lists have parity q, one thread: onto the
// restore list when local (the next update copies it into the buffer that sweep overwrites), and
// onto the count list when in S.
__device__ __forceinline__ void dc_list_change(const SweepArgs& a, uint32_t q, uint32_t v, uint32_t ca, uint32_t cb,
                                               bool restore = true) {
    if (restore && v - a.v_begin < a.v_end - a.v_begin) {
        const uint32_t j = atomicAdd(&a.dc_ctl[kDcChgLen + q], 1u);
        if (j < a.dc_chg_cap) a.dc_chg[(size_t)q * a.dc_chg_cap + j] = v;
        else a.dc_ctl[kDcChgOvf + q] = 1u;
    }
    if (v - a.dc_s0 < a.dc_s1 - a.dc_s0) {
        const uint32_t j = atomicAdd(&a.dc_ctl[kDcLen + q], 1u);
        if (j < a.dc_cap) {
            uint32_t* e = a.dc_list + 2u * ((size_t)q * a.dc_cap + j);
            e[0] = v;
            e[1] = (ca << 16) | cb;
        } else {
            a.dc_ctl[kDcOvf + q] = 1u;
        }
    }
}

// Row l (deg arcs) changes colour in sweep t: into slot `slot` (count in slot[0], arcs in slot[1],
// bumped by the caller's LDS counters), or the hub list. Returns deg.
__device__ __forceinline__ uint32_t inc_list_deg(const SweepArgs& a, uint32_t l, uint32_t t, uint32_t* slot,
                                                 uint32_t cap, uint32_t* lcount, uint32_t deg) {
    const uint32_t q = (t + 1u) & 1u;
    if (deg > a.inc_hub_arcs) {
        a.inc_hub[(size_t)q * a.inc_lcap + atomicAdd(&a.inc[kIncHubN + q], 1u)] = a.v_begin + l;
    } else {
        const uint32_t k = atomicAdd(lcount, 1u);   // LDS
        if (k < cap) slot[2 + k] = l;
        else a.inc[kIncOvf + q] = 1u;
    }
    return deg;
}
__device__ __forceinline__ uint32_t inc_list(const SweepArgs& a, uint32_t l, uint32_t t, uint32_t* slot,
                                             uint32_t cap, uint32_t* lcount) {
    return inc_list_deg(a, l, t, slot, cap, lcount, (uint32_t)(a.row_off[l + 1] - a.row_off[l]));
}
// The same for vertex v by its global id (the event replay: any rank's vertex). Slot entries of this
// kind hold global ids (the commit's own slot, inc_cchg).
__device__ __forceinline__ uint32_t inc_list_global(const SweepArgs& a, uint32_t v, uint32_t t, uint32_t* slot,
                                                    uint32_t cap, uint32_t* lcount) {
    const uint32_t q = (t + 1u) & 1u, deg = (uint32_t)(a.row_off_g[v + 1] - a.row_off_g[v]);
    if (deg > a.inc_hub_arcs) {
        a.inc_hub[(size_t)q * a.inc_lcap + atomicAdd(&a.inc[kIncHubN + q], 1u)] = v;
    } else {
        const uint32_t k = atomicAdd(lcount, 1u);   // LDS
        if (k < cap) slot[2 + k] = v;
        else a.inc[kIncOvf + q] = 1u;
    }
    return deg;
}

constexpr uint32_t kTabooMax24 = (1u << 24) - 1u;   // tail-queue entries pack the taboo counter in 24 bits
constexpr uint32_t kDeltaWords = 4096;  // MCMC delta slot per rank: head + (v, c) pairs (16 KiB)
constexpr uint32_t kDeltaHead = 2;
constexpr uint32_t kDeltaPairs = (kDeltaWords - kDeltaHead) / 2;

// The commit's end of sweep t (all its threads): its own slot's header, the rows and arcs every
// writer listed, the statistics, and the choice for sweep t + 1 -- a full recount after a slot
// overflowed or when the changed rows carry more than inc_thresh arcs (each changed arc costs two
// random colour reads; the tile scan streams half an entry per arc), else incremental.
__device__ void inc_commit(const SweepArgs& a, uint32_t t, const uint32_t* cc) {
    __shared__ unsigned long long red[2][32];
    __shared__ unsigned long long pre[8];   // control words, loaded side by side (not one chain on thread 0)
    __shared__ uint32_t wtot[32];
    const uint32_t q = (t + 1u) & 1u;
    if (threadIdx.x < 7u) {
        const uint32_t i = threadIdx.x;
        pre[i] = i == 0 ? a.inc[kIncMode] : i == 1 ? a.inc[kIncOvf + q] : i == 2 ? a.inc[kIncHubN + q]
                        : reinterpret_cast<const unsigned long long*>(a.inc + kIncStat)[i - 3u];
    }
    // every slot's rows gathered into one dense list (the next sweep's delta pass takes one row per
    // wave): contiguous slot ranges per thread, their counts scanned over the workgroup
    const uint32_t es = 2u + a.inc_slot, ws = 2u + a.inc_wslot_n, nsl = a.evnblk + kIncWalkSlots;
    auto slot = [&](uint32_t i, uint32_t& cap) -> const uint32_t* {
        cap = i < a.evnblk ? a.inc_slot : a.inc_wslot_n;
        return i < a.evnblk ? a.inc_eslot + ((size_t)q * a.evnblk + i) * es
                            : a.inc_wslot + ((size_t)q * kIncWalkSlots + (i - a.evnblk)) * ws;
    };
    const uint32_t per = (nsl + blockDim.x - 1u) / blockDim.x;
    const uint32_t s0 = min(threadIdx.x * per, nsl), s1 = min(s0 + per, nsl);
    uint32_t mine = 0;
    unsigned long long arcs = 0;
    const uint32_t* hd = a.inc_hdr + (size_t)q * nsl * 2u;
    for (uint32_t i = s0; i < s1; i++) {
        uint32_t cap;
        (void)slot(i, cap);
        mine += min(hd[2u * i], cap);
        arcs += hd[2u * i + 1u];
    }
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t inc = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    for (int o = 32; o > 0; o >>= 1) arcs += __shfl_xor(arcs, o, 64);
    if (lane == 63u) wtot[wave] = inc;
    if (lane == 0) red[1][wave] = arcs;
    __syncthreads();
    uint32_t off = inc - mine, T = 0;
    for (uint32_t w = 0; w < nwv; w++) {
        if (w < wave) off += wtot[w];
        T += wtot[w];
    }
    uint32_t* dn = a.inc_dense + (size_t)q * a.inc_lcap;
    for (uint32_t i = s0; i < s1; i++) {
        uint32_t cap;
        const uint32_t* sl = slot(i, cap);
        const uint32_t c = min(sl[0], cap);
        for (uint32_t k = 0; k < c; k++) dn[off + k] = a.v_begin + sl[2 + k];   // (slots: local rows)
        off += c;
    }
    const uint32_t* cl = a.inc_cchg + (size_t)q * (2u + a.inc_ccap);   // the event replay's rows after them
    for (uint32_t k = threadIdx.x; k < cc[0]; k += blockDim.x) dn[T + k] = cl[2 + k];
    // a partitioned delta-mode commit: the other ranks' changed vertices (their delta slots) after
    // those -- their rows' arcs into this rank's rows move its counts, and the next sweep copies
    // their colours into its output buffer (part_commit_kernel wrote them into C_t+1's only)
    __shared__ uint32_t s_rem;
    __shared__ unsigned long long s_rarcs;
    if (threadIdx.x == 0) {
        s_rem = 0;
        s_rarcs = 0;
    }
    __syncthreads();
    if (a.world > 1 && a.part_delta > 0) {
        const uint32_t* dall = (t & 1) ? a.dall0 : a.dall1;   // sweep t's slots (next-colour parity)
        for (uint32_t r = 0; r < a.world; r++) {
            if (r == a.rank) continue;
            const uint32_t* d = dall + (size_t)r * kDeltaWords;
            const uint32_t nr = min(d[0], kDeltaPairs);
            for (uint32_t i = threadIdx.x; i < nr; i += blockDim.x) {
                const uint32_t v = d[kDeltaHead + 2u * i];
                const uint32_t deg = (uint32_t)(a.row_off_g[v + 1] - a.row_off_g[v]);
                if (deg > a.inc_hub_arcs) a.inc_hub[(size_t)q * a.inc_lcap + atomicAdd(&a.inc[kIncHubN + q], 1u)] = v;
                else dn[T + cc[0] + atomicAdd(&s_rem, 1u)] = v;
                atomicAdd(&s_rarcs, (unsigned long long)deg);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < nwv; w++) arcs += red[1][w];
        arcs += s_rarcs;
        a.inc[kIncDenseN + q] = T + cc[0] + s_rem;
        const unsigned long long rows = (unsigned long long)T + cc[0] + pre[2];
        arcs += cc[1];
        unsigned long long* s = reinterpret_cast<unsigned long long*>(a.inc + kIncStat);
        s[0] = pre[3] + (pre[0] ? 0ull : 1ull);
        s[1] = pre[4] + (pre[0] ? 1ull : 0ull);
        s[2] = pre[5] + rows;
        s[3] = pre[6] + arcs;
        // a full-mode exchange tells no rank which of the others' vertices changed: a recount
        const bool blind = a.world > 1 && a.part_delta <= 0;
        a.inc[kIncMode] = (pre[1] || arcs > a.inc_thresh || blind) ? 1u : 0u;
    }
}
constexpr uint32_t kPairTraceMax = 256;   // pairs traced per workgroup (MCMC_PAIR_TRACE)
constexpr uint32_t kPairTraceRec = 8;     // {start, scan end min, scan end max, eval end, barrier end, info, 0, 0}
constexpr uint32_t kHistWords = 260;   // colours 0..255 (a colour may equal nCol <= 255)

// Phase timestamps of the last sweep, 8 slots per workgroup (wall_clock64, 100 MHz): 0 start,
// 1 first scan begins, 2 scans done, 3 evaluation done, 4 tail done (last workgroup: commit done).
#define MCMC_PHASE(a, k)                                                                  \
    do {                                                                                  \
        if ((a).phase_ts && threadIdx.x == 0) (a).phase_ts[blockIdx.x * 8u + (k)] = wall_clock64(); \
    } while (0)

__constant__ uint32_t kMinstdLanePow[64];   // 16807^j mod (2^31-1), j = 0..63
__constant__ uint32_t kMinstdPow2[64];      // 16807^(2^i) mod (2^31-1), i = 0..63
constexpr uint32_t kGlibcTabK = 4096;       // glibc draws per table block (commit_accept)
__device__ uint32_t kGlibcTab[31 * kGlibcTabK];   // [i][k]: coefficient i of x^(k+31) mod (x^31 - x^28 - 1)

// 16807^e mod (2^31-1) from the squares table: one mulmod per set bit of e.
__device__ __forceinline__ uint32_t minstd_pow_tab(uint64_t e) {
    uint32_t r = 1;
    for (int i = 0; e; i++, e >>= 1)
        if (e & 1) r = minstd_mulmod(r, kMinstdPow2[i]);
    return r;
}
// The same for an exponent every lane of the wave shares: a scalar loop (scalar table loads), where
// a per-lane exponent is a chain of ~22 dependent vector loads and mulmods.
__device__ __forceinline__ uint32_t minstd_pow_tab_wave(uint64_t e) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)e);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(e >> 32));
    return minstd_pow_tab(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int lane) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, lane);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

template <int NW>
__device__ __forceinline__ void set_color_bit(uint32_t (&m)[NW], uint32_t c) {
    if (NW == 1) {
        m[0] |= 1u << c;
    } else {
        const uint32_t w = c >> 5, bit = 1u << (c & 31);
#pragma unroll
        for (int i = 0; i < NW; i++) m[i] |= (w == (uint32_t)i) ? bit : 0u;
    }
}

template <int NW>
__device__ __forceinline__ uint32_t get_color_bit(const uint32_t (&m)[NW], uint32_t c) {
    if (NW == 1) return (m[0] >> c) & 1u;
    uint32_t r = 0;
    const uint32_t w = c >> 5;
#pragma unroll
    for (int i = 0; i < NW; i++) r |= (w == (uint32_t)i) ? ((m[i] >> (c & 31)) & 1u) : 0u;
    return r;
}

// OR over the 64 lanes into a wave-uniform value: quad swaps and row rotations (DPP, VALU
// latency) reduce each row of 16 lanes, four readlanes and scalar ORs finish.
__device__ __forceinline__ uint32_t wave_or_uniform(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false);   // row_ror:4
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);   // row_ror:8
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) | (uint32_t)__builtin_amdgcn_readlane((int)x, 16) |
           (uint32_t)__builtin_amdgcn_readlane((int)x, 32) | (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}

template <int NW>
__device__ __forceinline__ void wave_or(uint32_t (&m)[NW]) {
#pragma unroll
    for (int i = 0; i < NW; i++) {
        uint32_t x = m[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x |= __shfl_xor(x, off, 64);
        m[i] = x;
    }
}

// ----------------------------------------------------------------------------------------------
// Commit: loop control + ordered glibc replay. One workgroup.
constexpr int kCommitThreads = 256;
constexpr uint32_t kLdsSortCap = 8192;
constexpr uint32_t kRankSortMax = 1024;   // commit: rank-sort event lists up to this length
constexpr uint32_t kEvSlot = 32;          // wide evaluation: events a workgroup keeps in order

__device__ void bitonic_sort_block(uint32_t* s, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const bool up = (i & k) == 0;
                    const uint32_t x = s[i], y = s[ixj];
                    if ((x > y) == up) { s[i] = y; s[ixj] = x; }
                }
            }
            __syncthreads();
        }
    }
}

// Applies the accepted sweep: replays E sorted events, advances the RNG, flips buffers.
// `ev` holds the events (global ids, any order) and is sorted in place (via LDS when small).
// CT: the colour replica's element type (uint8_t; uint16_t for the wide sweep, nCol > 256).
// Diagnostics (MCMC_PHASE_DUMP): commit phase stamps in the phase buffer's last 8 slots.
#define MCMC_COMMIT_PHASE(a, k)                                                                       \
    do {                                                                                              \
        if ((a).phase_ts && threadIdx.x == 0) (a).phase_ts[8u * 4095u + (k)] = wall_clock64();       \
    } while (0)

template <typename CT = uint8_t>
__device__ __forceinline__ void commit_accept(const SweepArgs& a, uint32_t t, uint32_t* ev, uint32_t E, uint32_t* lds,
                              uint32_t lds_cap, bool sorted = false) {
    DevState* st = a.st;
    __shared__ uint32_t inc_cc[2];   // incremental counts: rows the event replay changed, their arcs
    if (threadIdx.x == 0) inc_cc[0] = inc_cc[1] = 0;   // (the barriers below order it)
    MCMC_COMMIT_PHASE(a, 1);
    const CT* C = reinterpret_cast<const CT*>((t & 1) ? a.colors1 : a.colors0);
    CT* Cs = reinterpret_cast<CT*>((t & 1) ? a.colors0 : a.colors1);
    if (E > 0) {
        // Ascending vertex order. Events are distinct vertices, so a short list is ranked directly
        // (each event counts the smaller ids: all threads, LDS broadcast reads, 16 B at a time when
        // aligned); longer ones take the bitonic sort. The top 64 words of `lds` hold the glibc window.
        uint32_t* gw = lds + lds_cap - 64u;
        lds_cap -= 64u;
        const uint32_t E4 = (E + 3u) & ~3u;
        uint32_t* s;
        uint32_t* draws = a.evdraw;
        if (sorted) {   // already ascending (the wide evaluation's per-workgroup lists, in LDS)
            s = ev;
            if (ev == lds && 2u * E4 <= lds_cap) draws = lds + E4;
        } else if (E <= kRankSortMax && 2u * E4 <= lds_cap) {
            for (uint32_t i = threadIdx.x; i < E4; i += blockDim.x) lds[i] = (i < E) ? ev[i] : 0xFFFFFFFFu;
            __syncthreads();
            s = lds + E4;
            const bool al16 = (reinterpret_cast<uintptr_t>(lds) & 15u) == 0;
            for (uint32_t i = threadIdx.x; i < E; i += blockDim.x) {
                const uint32_t v = lds[i];
                uint32_t r = 0;
                if (al16) {
                    const uint4* l4 = reinterpret_cast<const uint4*>(lds);
#pragma unroll 8
                    for (uint32_t j = 0; j < E4 / 4u; j++) {
                        const uint4 q = l4[j];
                        r += (q.x < v ? 1u : 0u) + (q.y < v ? 1u : 0u) + (q.z < v ? 1u : 0u) + (q.w < v ? 1u : 0u);
                    }
                } else {
#pragma unroll 4
                    for (uint32_t j = 0; j < E4; j++) r += (lds[j] < v) ? 1u : 0u;
                }
                s[r] = v;
            }
            __syncthreads();
            draws = lds;   // the unsorted copy is dead: the draws go there
        } else {
            uint32_t P = 1;
            while (P < E) P <<= 1;
            s = (P <= lds_cap) ? lds : ev;
            if (s == ev) {
                for (uint32_t i = E + threadIdx.x; i < P; i += blockDim.x) s[i] = 0xFFFFFFFFu;
            } else {
                for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) s[i] = (i < E) ? ev[i] : 0xFFFFFFFFu;
            }
            __syncthreads();
            bitonic_sort_block(s, P);
        }
        MCMC_COMMIT_PHASE(a, 2);
        // The events' rand() draws in ascending vertex order. TYPE_3 is linear over Z/2^32: draw k
        // after the window w (oldest first) is r = sum_i T[i][k] w[i], T = x^(k+31) mod
        // (x^31 - x^28 - 1) (kGlibcTab, ensure_constants) -- every draw of a block of up to
        // kGlibcTabK at once, then the window moves to the block's last 31 raw draws.
        if (threadIdx.x < 31) gw[threadIdx.x] = st->glibc_ring[(st->glibc_head + threadIdx.x) % 31u];
        __syncthreads();
        for (uint32_t b = 0; b < E; b += kGlibcTabK) {
            const uint32_t nb = min(kGlibcTabK, E - b);
            for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
                uint32_t acc = 0;
#pragma unroll
                for (int i = 0; i < 31; i++) acc += kGlibcTab[i * kGlibcTabK + k] * gw[i];
                draws[b + k] = acc >> 1;
                if (k + 31u >= nb) gw[32u + k + 31u - nb] = acc;   // gw[32 + j]: raw draw nb - 31 + j
            }
            __syncthreads();
            uint32_t nw = 0;
            if (threadIdx.x < 31) {   // the window after the block: (w[nb..30], draws) or its last 31 draws
                const uint32_t j = threadIdx.x;
                nw = (nb < 31u && j < 31u - nb) ? gw[nb + j] : gw[32u + j];
            }
            __syncthreads();
            if (threadIdx.x < 31) gw[threadIdx.x] = nw;
            __syncthreads();
        }
        if (threadIdx.x < 31) st->glibc_ring[threadIdx.x] = gw[threadIdx.x];
        if (threadIdx.x == 0) st->glibc_head = 0;
        __threadfence_block();
        __syncthreads();
        MCMC_COMMIT_PHASE(a, 3);
        for (uint32_t i = threadIdx.x; i < E; i += blockDim.x) {
            const uint32_t v = s[i];
            const uint32_t c = draws[i] % (a.nCol - 1u);   // rand() % (nCol - 1), :518
            const uint32_t old = (uint32_t)C[v];
            Cs[v] = (CT)c;
            // delta mode: both replicas carry C_t+1 on the remote rows (part_commit_kernel)
            // (the wide sweep's incremental counts need C_t there: its next sweep copies the change)
            if (a.part_delta > 0 && a.inc == nullptr && (v < a.v_begin || v >= a.v_end)) const_cast<CT*>(C)[v] = (CT)c;
            if (a.fp_live) ((t & 1) ? a.wfp0 : a.wfp1)[v] = (uint8_t)c;
            if (a.taboo != nullptr && v >= a.v_begin && v < a.v_end)
                a.taboo[v - a.v_begin] = (c == old) ? a.tabooIteration : 0u;
            if (a.inc != nullptr && c != old)   // (any rank's vertex: global ids)
                atomicAdd(&inc_cc[1], inc_list_global(a, v, t, a.inc_cchg + (size_t)((t + 1u) & 1u) * (2u + a.inc_ccap),
                                                      a.inc_ccap, &inc_cc[0]));
            if (a.dc_list != nullptr && c != old) {
                // dense-count sweep: the count list when v is in S; a local v's new colour also
                // goes into the C_t buffer now (nothing reads C_t after the evaluation), so the
                // next sweep needs no restore of it
                dc_list_change(a, (t + 1u) & 1u, v, old, c, false);
                if (v - a.v_begin < a.v_end - a.v_begin) const_cast<CT*>(C)[v] = (CT)c;
            }
        }
        __syncthreads();
    }
    MCMC_COMMIT_PHASE(a, 4);
    if (a.dc_ctl != nullptr) {
        __syncthreads();   // the replay's list appends are in
        // a short restore list is applied here, C_t+1 into the C_t buffer (the one sweep t + 1
        // writes), so that sweep's update has nothing to do when no vertex of S moved
        const uint32_t q = (t + 1u) & 1u;
        __shared__ DcCommitWords dcw;
        if (threadIdx.x == 0) dcw = dc_commit_load(a, q);
        __syncthreads();
        const uint32_t m = dcw.chg, ovf = dcw.chg_ovf;
        if (threadIdx.x == 0) {
            const uint32_t r = a.dc_ctl[kDcStat2] + min(m, a.dc_chg_cap);
            a.dc_ctl[kDcStat2] = r < a.dc_ctl[kDcStat2] ? ~0u : r;
            a.dc_ctl[kDcStat2 + 1] += ovf ? 1u : 0u;
        }
        if (m != 0u && ovf == 0u && m <= a.dc_commit_restore) {
            CT* B = const_cast<CT*>(C);
            for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
                const uint32_t u = a.dc_chg[(size_t)q * a.dc_chg_cap + i];
                B[u] = Cs[u];
            }
            __syncthreads();
            if (threadIdx.x == 0) a.dc_ctl[kDcChgLen + q] = 0;
        }
        if (threadIdx.x == 0) dc_commit(a, t, dcw);
    }
    if (a.inc != nullptr) {
        __syncthreads();   // inc_cc complete
        inc_commit(a, t, inc_cc);
    }
    if (threadIdx.x == 0) {
        st->glibc_draws += E;
        st->x_t = minstd_mulmod(st->x_t, a.aN);
        const uint32_t lx = st->lx + a.nmodN;   // (both < 2^31 - 2: no wrap of 32 bits)
        st->lx = lx >= kMinstdN ? lx - kMinstdN : lx;
        st->t = t + 1;
        st->viol = 0;
        st->ev_count = 0;
        st->arrive = 0;
        st->arrive_viol = 0;
    }
}

// Loop control of run() (coloringMCMC_CPU.cpp:136, :259-269): records Cviol_t, stops on the cap or
// on Cviol_t <= z, otherwise accepts the sweep. All threads of one workgroup call it with the same
// state values; thread 0 writes the state.
template <typename CT = uint8_t>
__device__ __forceinline__ void commit_control(const SweepArgs& a, uint32_t t, unsigned long long viol, uint32_t E, uint32_t err,
                               uint32_t* lds, uint32_t lds_cap, uint32_t* ev = nullptr, bool sorted = false) {
    DevState* st = a.st;
    if (threadIdx.x == 0 && t < a.traj_cap) a.traj[t] = viol;
    const bool stop_cap = t == a.maxRip + 1;     // iter > maxiter after sweep maxRip
    const bool stop_conv = !a.bench && viol <= a.z;   // while (Cviol > z)
    if (stop_cap || stop_conv) {
        if (threadIdx.x == 0) {
            st->done = 1;
            st->iter = t;
            st->maxIterReached = stop_cap;
            st->finalViol = viol;
            st->arrive = 0;
            st->arrive_viol = 0;
        }
        return;
    }
    if (E > a.ev_cap || err) {
        if (threadIdx.x == 0) { st->err |= kDevErrEvents; st->done = 1; st->iter = t; }
        return;
    }
    commit_accept<CT>(a, t, ev ? ev : a.events, E, lds, lds_cap, sorted);
}

// The wide evaluation's per-workgroup event lists (each ascending, workgroups in vertex order)
// after the Eg events of the global list (walk events, list overflows). Eg == 0 and room in LDS:
// concatenated in order into lds (*out = lds, sorted); else appended to a.events (*out =
// a.events, unsorted). Returns the total. All threads call it.
__device__ uint32_t wide_block_events(const SweepArgs& a, uint32_t Eg, uint32_t* lds, uint32_t cap,
                                      uint32_t** out, bool* sorted) {
    __shared__ uint32_t wtot[17];
    const uint32_t nb = a.evnblk;
    const uint32_t per = (nb + blockDim.x - 1u) / blockDim.x;
    const uint32_t b0 = min(threadIdx.x * per, nb), b1 = min(b0 + per, nb);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += a.evcnt[b];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t inc = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) wtot[wave] = inc;
    __syncthreads();
    uint32_t off = inc - sum, tot = 0;
    for (uint32_t w = 0; w < nw; w++) {
        if (w < wave) off += wtot[w];
        tot += wtot[w];
    }
    const bool inl = Eg == 0 && tot <= cap;
    uint32_t* dst = inl ? lds : a.events + Eg;
    const uint32_t lim = inl ? cap : (a.ev_cap > Eg ? a.ev_cap - Eg : 0u);
    for (uint32_t b = b0; b < b1; b++) {
        const uint32_t c = a.evcnt[b];
        for (uint32_t i = 0; i < c; i++)
            if (off + i < lim) dst[off + i] = a.evblk[(size_t)b * kEvSlot + i];
        off += c;
    }
    __threadfence_block();
    __syncthreads();
    *out = inl ? lds : a.events;
    *sorted = inl;
    return Eg + tot;
}

// Loop control of the reference's GPU run() (coloringMCMC_main.cu:160-269), fused into the last
// workgroup of sweep t: `ecnt` = C_t's arcs (v, w) with w > v and equal colours, summed over the
// rows by the scan -- the conflictCounter kernel + calcConflicts (coloringMCMC_utils.cu:103-119,
// 184-198). Iteration rip = t + 1 counts C_t and stops at <= z; after maxRip
// iterations (maxRip sweeps) the loop ends without that test, and this sweep is the count-only
// pass whose count is the last sweep's "nuovi conflitti" (:229). Accepting flips the parity of
// the colours, XORWOW states and histograms, and clears the histogram sweep t+1 accumulates into.
// copy_from (REF wide): the histogram sweep t+1 accumulates into starts as this copy, not zeroed.
__device__ void commit_control_ref(const SweepArgs& a, uint32_t t, unsigned long long ecnt,
                                   const uint32_t* copy_from = nullptr) {
    DevState* st = a.st;
    const unsigned long long c = ecnt;
    if (threadIdx.x == 0 && t < a.traj_cap) a.traj[t] = c;
    const uint32_t cap = a.maxRip > 0 ? a.maxRip : 1u;   // do { ... } while (rip < maxRip): >= 1 sweep
    if (t == cap || (!a.bench && c <= a.z)) {   // throughput mode: no convergence stop
        if (threadIdx.x == 0) {
            const uint32_t rip = (t == cap) ? cap : t + 1u;
            st->done = 1;
            st->iter = rip;
            st->maxIterReached = rip == a.maxRip;   // :294-295
            st->finalViol = c;
            st->arrive_viol = 0;
        }
        return;
    }
    uint32_t* h = a.hist + (t & 1u) * a.hist_words;
    for (uint32_t i = threadIdx.x; i < a.hist_words; i += blockDim.x) h[i] = copy_from ? copy_from[i] : 0u;
    if (threadIdx.x == 0) {
        st->t = t + 1;
        st->arrive_viol = 0;
    }
}

// The wide sweep's commit when it is the common case -- at most NT events (the evaluation
// workgroups' ordered lists, plus the walks' global list sorted in LDS), no error, no stop -- as
// three dependent round trips instead of ~10. A single workgroup pulls ~64 GB/s, so what it loads
// is kept small and side by side: (1) the state words, the glibc ring, its evaluation workgroups'
// event counts, both parities' compact slot headers, the incremental control words; (2) the
// events' lists, the draw coefficients of the events present, the slots' rows; (3) the event
// colours' own loads; then the stores. Same results as commit_control + commit_accept +
// inc_commit (the generic path below runs otherwise, nothing written before the choice). Returns
// false to fall back.
constexpr uint32_t kPreBlk = 2, kPreSlots = 3;
using CT_U16 = uint16_t;
template <int NT>
__device__ bool wide_commit_fast(const SweepArgs& a) {
    __shared__ uint32_t s_ev[NT];          // the events, ascending
    __shared__ uint32_t s_raw[NT];         // their raw glibc draws
    __shared__ uint32_t s_ring[32], s_gw[32];
    __shared__ uint32_t s_w[NT / 64], s_w2[NT / 64];
    __shared__ uint32_t s_hdr[8];
    __shared__ unsigned long long s_q[8], s_arcs[NT / 64];
    __shared__ uint32_t s_cc[3];           // the replay's changed rows: listed, their arcs, hubs
    DevState* st = a.st;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, nwv = NT / 64u;
    const bool inc = a.inc != nullptr;
    const uint32_t nb = a.evnblk, nsl = inc ? nb + kIncWalkSlots : 0u;
    if (nb > NT * kPreBlk || nsl > NT * kPreSlots) return false;
    // ---- (1) every independent load: state words, the glibc ring, draw tid's 31 coefficients,
    // this thread's evaluation workgroups' event counts, both parities' slot headers ----
    uint32_t hv = 0;
    unsigned long long hq = 0;
    if (tid < 6u)
        hv = tid == 0 ? st->done : tid == 1 ? st->t : tid == 2 ? st->err : tid == 3 ? st->ev_count
           : tid == 4 ? st->glibc_head : st->x_t;
    if (tid < 2u) hq = tid == 0 ? st->viol : st->glibc_draws;
    const uint32_t ring = tid < 31u ? st->glibc_ring[tid] : 0u;
    const uint32_t b0 = min(tid * kPreBlk, nb), b1 = min(b0 + kPreBlk, nb);
    uint32_t bc[kPreBlk];
#pragma unroll
    for (uint32_t j = 0; j < kPreBlk; j++) bc[j] = b0 + j < b1 ? a.evcnt[b0 + j] : 0u;
    const uint32_t s0 = min(tid * kPreSlots, nsl), s1 = min(s0 + kPreSlots, nsl);
    uint32_t sc[2][kPreSlots], sa[2][kPreSlots];
#pragma unroll
    for (uint32_t p = 0; p < 2; p++)
#pragma unroll
        for (uint32_t j = 0; j < kPreSlots; j++) {
            const uint32_t i = s0 + j;
            sc[p][j] = i < s1 ? min(a.inc_hdr[((size_t)p * nsl + i) * 2u], i < nb ? a.inc_slot : a.inc_wslot_n) : 0u;
            sa[p][j] = i < s1 ? a.inc_hdr[((size_t)p * nsl + i) * 2u + 1u] : 0u;
        }
    uint32_t cw[5] = {0, 0, 0, 0, 0};   // mode, ovf[0..1], hubN[0..1]
    if (inc && tid == 0) {
        cw[0] = a.inc[kIncMode];
        cw[1] = a.inc[kIncOvf];
        cw[2] = a.inc[kIncOvf + 1];
        cw[3] = a.inc[kIncHubN];
        cw[4] = a.inc[kIncHubN + 1];
    }
    unsigned long long stq = 0;
    if (inc && tid < 4u) stq = reinterpret_cast<const unsigned long long*>(a.inc + kIncStat)[tid];
    if (tid < 8u) {
        s_hdr[tid] = hv;
        s_q[tid] = hq;
    }
    if (tid < 32u) s_ring[tid] = ring;
    if (tid == 0) s_cc[0] = s_cc[1] = s_cc[2] = 0;
    // ---- (2) orders: the events (per-workgroup counts) and the changed rows (slot counts) ----
    uint32_t me = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPreBlk; j++) me += bc[j];
    uint32_t ie = me;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(ie, o, 64);
        if (lane >= (uint32_t)o) ie += y;
    }
    if (lane == 63u) s_w[wave] = ie;
    __syncthreads();
    const uint32_t done = s_hdr[0], t = s_hdr[1], err = s_hdr[2], Eg = s_hdr[3], head = s_hdr[4], x_t = s_hdr[5];
    const unsigned long long viol = s_q[0], draws0 = s_q[1];
    if (done) return true;
    uint32_t off = ie - me, E = 0;
    for (uint32_t w = 0; w < nwv; w++) {
        if (w < wave) off += s_w[w];
        E += s_w[w];
    }
    const bool stop = t == a.maxRip + 1 || (!a.bench && viol <= a.z);
    const uint32_t Eb = E;   // the evaluation workgroups' events; the walks' (unsorted) follow them
    E += Eg;
    if (err != 0 || E > NT || E > a.ev_cap || stop) return false;   // the generic path
    uint32_t tab[31];   // draw tid's coefficients (tid < E): r = sum_i T[i][tid] w[i] (commit_accept)
#pragma unroll
    for (int i = 0; i < 31; i++) tab[i] = tid < E ? kGlibcTab[i * kGlibcTabK + tid] : 0u;
    const uint32_t q = (t + 1u) & 1u;
    uint32_t sm = 0;
    unsigned long long arcs = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPreSlots; j++) {
        sm += q ? sc[1][j] : sc[0][j];
        arcs += q ? sa[1][j] : sa[0][j];
    }
    uint32_t is = sm;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(is, o, 64);
        if (lane >= (uint32_t)o) is += y;
    }
    for (int o = 32; o > 0; o >>= 1) arcs += __shfl_xor(arcs, o, 64);
    if (lane == 63u) s_w2[wave] = is;
    if (lane == 0) s_arcs[wave] = arcs;
#pragma unroll
    for (uint32_t j = 0; j < kPreBlk; j++) {   // this thread's workgroups' events, in order
        const uint32_t b = b0 + j;
        if (b >= b1) break;
        for (uint32_t k = 0; k < bc[j]; k++) s_ev[off + k] = a.evblk[(size_t)b * kEvSlot + k];
        off += bc[j];
    }
    if (tid < Eg) s_ev[Eb + tid] = a.events[tid];
    if (tid == 0 && t < a.traj_cap) a.traj[t] = viol;
    if (tid < 31u) s_gw[tid] = s_ring[(head + tid) % 31u];
    __syncthreads();
    if (Eg != 0) {   // walk events: the whole list into ascending order (distinct vertices; LDS bitonic)
        uint32_t P = 1;
        while (P < E) P <<= 1;
        for (uint32_t k = E + tid; k < P; k += NT) s_ev[k] = 0xFFFFFFFFu;
        __syncthreads();
        bitonic_sort_block(s_ev, P);
    }
    uint32_t soff = is - sm, T = 0;
    for (uint32_t w = 0; w < nwv; w++) {
        if (w < wave) soff += s_w2[w];
        T += s_w2[w];
    }

    uint32_t* dn = inc ? a.inc_dense + (size_t)q * a.inc_lcap : nullptr;
    // ---- (3) the events' glibc draws and colours; the slots' rows into the dense list ----
    const CT_U16* C = reinterpret_cast<const CT_U16*>((t & 1) ? a.colors1 : a.colors0);
    CT_U16* Cs = reinterpret_cast<CT_U16*>((t & 1) ? a.colors0 : a.colors1);
    uint32_t v = 0, c = 0, oc = 0;
    uint64_t r0 = 0, r1 = 0;
    if (tid < E) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 31; i++) acc += tab[i] * s_gw[i];
        s_raw[tid] = acc;
        v = s_ev[tid];
        c = (acc >> 1) % (a.nCol - 1u);   // rand() % (nCol - 1), :518
        oc = C[v];
        if (inc) {
            r0 = a.row_off[v - a.v_begin];
            r1 = a.row_off[v - a.v_begin + 1];
        }
    }
    if (inc) {
        const uint32_t es = 2u + a.inc_slot, ws = 2u + a.inc_wslot_n;
#pragma unroll
        for (uint32_t j = 0; j < kPreSlots; j++) {
            const uint32_t i = s0 + j;
            if (i >= s1) break;
            const uint32_t n = q ? sc[1][j] : sc[0][j];
            const uint32_t* sl = i < nb ? a.inc_eslot + ((size_t)q * nb + i) * es
                                        : a.inc_wslot + ((size_t)q * kIncWalkSlots + (i - nb)) * ws;
            for (uint32_t k = 0; k < n; k++) dn[soff + k] = a.v_begin + sl[2 + k];
            soff += n;
        }
    }
    __syncthreads();   // s_raw complete
    uint32_t nwin = 0;
    if (tid < 31u) nwin = (E < 31u && tid < 31u - E) ? s_gw[E + tid] : s_raw[E + tid - 31u];
    if (tid < E) {
        Cs[v] = (CT_U16)c;
        if (a.fp_live) ((t & 1) ? a.wfp0 : a.wfp1)[v] = (uint8_t)c;
        if (a.taboo != nullptr) a.taboo[v - a.v_begin] = (c == oc) ? a.tabooIteration : 0u;
        if (inc && c != oc) {   // the replay's changed rows go straight after the slots' in the dense list
            const uint32_t deg = (uint32_t)(r1 - r0);
            if (deg > a.inc_hub_arcs) {
                a.inc_hub[(size_t)q * a.inc_lcap + atomicAdd(&a.inc[kIncHubN + q], 1u)] = v;
                atomicAdd(&s_cc[2], 1u);
            } else {
                dn[T + atomicAdd(&s_cc[0], 1u)] = v;
            }
            atomicAdd(&s_cc[1], deg);
        }
    }
    if (tid < 31u) st->glibc_ring[tid] = nwin;
    if (tid == 0) {
        st->glibc_head = 0;
        st->glibc_draws = draws0 + E;
        st->x_t = minstd_mulmod(x_t, a.aN);
        {
            const uint32_t lx = st->lx + a.nmodN;
            st->lx = lx >= kMinstdN ? lx - kMinstdN : lx;
        }
        st->t = t + 1;
        st->viol = 0;
        st->ev_count = 0;
        st->arrive = 0;
        st->arrive_viol = 0;
    }
    if (!inc) return true;
    // ---- (4) the next sweep's mode and the statistics ----
    if (tid < 4u) s_q[tid] = stq;
    __syncthreads();
    if (tid == 0) {
        unsigned long long ar = s_cc[1];
        for (uint32_t w = 0; w < nwv; w++) ar += s_arcs[w];
        a.inc[kIncDenseN + q] = T + s_cc[0];
        const unsigned long long rows = (unsigned long long)T + s_cc[0] + s_cc[2] + (q ? cw[4] : cw[3]);
        unsigned long long* sst = reinterpret_cast<unsigned long long*>(a.inc + kIncStat);
        sst[0] = s_q[0] + (cw[0] ? 0ull : 1ull);
        sst[1] = s_q[1] + (cw[0] ? 1ull : 0ull);
        sst[2] = s_q[2] + rows;
        sst[3] = s_q[3] + ar;
        a.inc[kIncMode] = ((q ? cw[2] : cw[1]) || ar > a.inc_thresh) ? 1u : 0u;
    }
    return true;
}

// Stand-alone commit (the wide sweep; MCMC_FUSED_COMMIT=0 A/B builds): same control, own launch.
// NT threads: the wide sweep's hundreds of events per sweep rank-sort faster on 1024.
template <typename CT, int NT = kCommitThreads>
__global__ __launch_bounds__(NT) void commit_kernel(SweepArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsSortCap];
    __shared__ uint32_t sh_done, sh_t, sh_E, sh_err;
    __shared__ unsigned long long sh_viol;
    DevState* st = a.st;
    MCMC_COMMIT_PHASE(a, 0);
    if (a.wcount && threadIdx.x < 4) a.wcount[threadIdx.x] = 0;   // the walk list, for the next sweep
    if constexpr (sizeof(CT) == 2 && NT == 1024) {
        if (a.evcnt != nullptr && !a.phase_ts && wide_commit_fast<NT>(a)) return;
    }
    if (threadIdx.x == 0) {
        sh_done = st->done;
        sh_t = st->t;
        sh_viol = st->viol;
        sh_E = st->ev_count;
        sh_err = st->err;
    }
    __syncthreads();
    if (sh_done) return;
    uint32_t E = sh_E;
    uint32_t* ev = nullptr;
    bool sorted = false;
    if (a.evcnt) E = wide_block_events(a, sh_E, lds, kLdsSortCap - 64u, &ev, &sorted);
    commit_control<CT>(a, sh_t, sh_viol, E, sh_err, lds, kLdsSortCap, ev, sorted);
    MCMC_COMMIT_PHASE(a, 5);
    if (a.phase_ts && threadIdx.x == 0) a.phase_ts[8u * 4095u + 6] = sh_E;
}

// ---- vertex-partitioned sweep: footer exchange ------------------------------------------------
constexpr uint32_t kFooterWords = 1024;                 // MCMC_FOOTER_WORDS
constexpr uint32_t kFooterEvents = kFooterWords - 4;
constexpr uint32_t kMaxWorld = 64;                       // ranks of a partitioned run
constexpr uint64_t kTrajCapMax = 1u << 20;               // trajectory entries kept (throughput runs lift maxRip)
constexpr uint32_t kPartAlign = 64;                      // inner partition bounds: multiples of 64 rows
constexpr double kPartRowWeight = 16.0;                  // arc-balanced plans: a row costs deg + 16

// Footer flags (word 3): bit 0 fatal (the local list overflowed ev_cap, or a device error), bit 1
// the sorted list did not fit the footer -- the commit then pauses for the spill exchange
// (mcmc_part_spill_*), which takes every rank's full list from its `events` buffer.
constexpr uint32_t kFootFatal = 1u, kFootSpill = 2u;
// DevState::err bits: 1 fatal, 2 paused for a spill exchange (st->done is set meanwhile, so every
// kernel of the steps a driver enqueued before it noticed returns at once).
constexpr uint32_t kErrFatal = 1u, kErrSpill = 2u;
// bit 2: paused because some rank's delta slot overflowed (delta mode): the driver exchanges the
// sweep's colour ranges instead and resumes with a full-mode commit (multi.hip)
constexpr uint32_t kErrDelta = 4u;

__device__ __forceinline__ uint32_t* rank_footer(const SweepArgs& a, uint32_t t, uint32_t r) {
    return ((t & 1) ? a.foot0 : a.foot1) + (size_t)r * kFooterWords;   // next-colour parity
}

// Last workgroup of a partitioned sweep: sort this rank's overflow events and publish
// [Cviol_local, E, flags, events] for the exchange; reset the local accumulators. A list longer
// than the footer stays sorted in a.events for the spill exchange.
__device__ void pack_footer(const SweepArgs& a, uint32_t t, unsigned long long viol, uint32_t E, uint32_t err,
                            uint32_t* lds, uint32_t lds_cap, uint32_t* presorted = nullptr) {
    DevState* st = a.st;
    uint32_t* footer = rank_footer(a, t, a.rank);
    uint32_t* s = presorted ? presorted : a.events;
    if (!presorted && E > 0 && E <= a.ev_cap) {
        uint32_t P = 1;
        while (P < E) P <<= 1;
        s = (P <= lds_cap) ? lds : a.events;
        if (s == a.events) {
            for (uint32_t i = E + threadIdx.x; i < P; i += blockDim.x) s[i] = 0xFFFFFFFFu;
        } else {
            for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) s[i] = (i < E) ? a.events[i] : 0xFFFFFFFFu;
        }
        __syncthreads();
        bitonic_sort_block(s, P);
    }
    const bool fatal = E > a.ev_cap || err;
    if (E > kFooterEvents && !fatal && s != a.events) {   // keep the whole sorted list for the spill
        for (uint32_t i = threadIdx.x; i < E; i += blockDim.x) a.events[i] = s[i];
        __syncthreads();
    }
    const uint32_t En = min(E, kFooterEvents);
    for (uint32_t i = threadIdx.x; i < En; i += blockDim.x) footer[4 + i] = s[i];
    if (threadIdx.x == 0) {
        footer[0] = (uint32_t)viol;
        footer[1] = (uint32_t)(viol >> 32);
        footer[2] = E;
        footer[3] = (fatal ? kFootFatal : 0u) | (E > kFooterEvents ? kFootSpill : 0u);
        st->viol = 0;
        st->ev_count = 0;
        st->arrive = 0;
        st->arrive_viol = 0;
    }
}

// Every rank, after the exchange: global Cviol = sum of the footers, events = rank-ordered
// concatenation (ranks own ascending vertex ranges, so it is ascending), then the same commit as
// the single-context loop -- identical glibc replay on every replica. A list that did not fit a
// footer pauses the loop here (spill) unless the sweep stops anyway; spill = the full lists,
// gathered by the driver (rank r's at spill[r * stride], E_r from its footer).
template <typename CT>
__global__ __launch_bounds__(kCommitThreads) void part_commit_kernel(SweepArgs a, const uint32_t* spill,
                                                                     uint32_t stride) {
    __shared__ uint32_t lds[kLdsSortCap];
    __shared__ uint32_t sh_go, sh_t, sh_E, sh_err, sh_spill, sh_dovf;
    __shared__ unsigned long long sh_viol;
    __shared__ uint32_t sh_off[kMaxWorld + 1];
    __shared__ uint32_t sh_dn[kMaxWorld];
    DevState* st = a.st;
    if (threadIdx.x == 0) {
        const uint32_t t0 = st->t;
        // spill == nullptr and not resuming: the step's own commit (skipped once done); else the
        // resumption of a loop paused for this sweep's spill or delta-overflow exchange
        const bool resume = spill != nullptr || (a.part_delta < 0);
        sh_go = resume ? ((st->err & (kErrSpill | kErrDelta)) != 0u) : (st->done == 0u);
        sh_t = t0;
        unsigned long long v = 0;
        uint32_t E = 0, err = st->err & kErrFatal, sp = 0, dovf = 0;
        const uint32_t* dall = (t0 & 1) ? a.dall0 : a.dall1;   // next-colour parity, like the footers
        for (uint32_t r = 0; r < a.world; r++) {
            const uint32_t* f = rank_footer(a, t0, r);
            v += (unsigned long long)f[0] | ((unsigned long long)f[1] << 32);
            sh_off[r] = E;
            E += spill ? f[2] : min(f[2], kFooterEvents);
            err |= f[3] & kFootFatal;
            sp |= f[3] & kFootSpill;
            sh_dn[r] = 0;
            if (a.part_delta > 0) {
                const uint32_t k = dall[(size_t)r * kDeltaWords];
                dovf |= k > kDeltaPairs ? 1u : 0u;
                sh_dn[r] = min(k, kDeltaPairs);
            }
        }
        sh_off[a.world] = E;
        sh_viol = v;
        sh_E = E;
        sh_err = err;
        sh_spill = spill ? 0u : sp;
        sh_dovf = dovf;
        if (sh_go && resume) {
            st->done = 0;
            st->err &= ~(kErrSpill | kErrDelta);
        }
    }
    __syncthreads();
    if (!sh_go) return;
    const uint32_t t = sh_t;
    const bool stop = t == a.maxRip + 1 || (!a.bench && sh_viol <= a.z);
    if ((sh_spill || sh_dovf) && !stop && !sh_err) {   // pause: the driver gathers lists / colour ranges
        if (threadIdx.x == 0) {
            st->err |= (sh_spill ? kErrSpill : 0u) | (sh_dovf ? kErrDelta : 0u);
            st->done = 1;
        }
        return;
    }
    if (!stop && !sh_err && sh_E <= a.ev_cap) {
        for (uint32_t r = 0; r < a.world; r++) {
            const uint32_t* src = spill ? spill + (size_t)r * stride : rank_footer(a, t, r) + 4;
            const uint32_t Er = sh_off[r + 1] - sh_off[r];
            for (uint32_t i = threadIdx.x; i < Er; i += blockDim.x) a.events[sh_off[r] + i] = src[i];
        }
        if (a.part_delta > 0) {
            // the other ranks' changed vertices into both replicas: C_t+1 (this sweep's output)
            // and the C_t buffer, which sweep t+1 overwrites only on this rank's rows -- so after
            // every delta-mode commit both replicas hold C_t+1 outside the local range
            CT* B = reinterpret_cast<CT*>((t & 1) ? a.colors0 : a.colors1);
            CT* A = reinterpret_cast<CT*>((t & 1) ? a.colors1 : a.colors0);
            const uint32_t* dall = (t & 1) ? a.dall0 : a.dall1;
            for (uint32_t r = 0; r < a.world; r++) {
                if (r == a.rank) continue;
                const uint32_t* d = dall + (size_t)r * kDeltaWords + kDeltaHead;
                for (uint32_t i = threadIdx.x; i < sh_dn[r]; i += blockDim.x) {
                    const uint32_t v = d[2u * i];
                    const CT c = (CT)d[2u * i + 1u];
                    B[v] = c;
                    if (a.inc == nullptr) A[v] = c;   // (incremental counts: the next sweep copies it)
                }
            }
        }
        // this rank's slot for sweep t + 1 starts empty
        if (threadIdx.x == 0 && a.dlt0) ((t & 1) ? a.dlt1 : a.dlt0)[0] = 0u;
    }
    __syncthreads();
    commit_control<CT>(a, t, sh_viol, sh_E, sh_err, lds, kLdsSortCap);
}

// Delta mode needs both replicas equal outside this rank's rows: after a full-mode step (or at the
// start of a run) the next-colour buffer's remote part is set to the current colouring's.
template <typename CT>
__global__ __launch_bounds__(256) void part_sync_remote_kernel(SweepArgs a) {
    const DevState* st = a.st;
    if (st->done) return;
    const uint32_t t = st->t;
    const uint8_t* src = (t & 1) ? a.colors1 : a.colors0;   // C_t
    uint8_t* dst = (t & 1) ? a.colors0 : a.colors1;
    const size_t cb = sizeof(CT);
    const size_t r0[2] = {0, (size_t)a.v_end * cb};
    const size_t r1[2] = {(size_t)a.v_begin * cb, (size_t)a.n * cb};
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    for (int k = 0; k < 2; k++) {
        const size_t b0 = r0[k], b1 = r1[k];
        if (b1 <= b0) continue;
        const size_t q0 = (b0 + 15) & ~(size_t)15, q1 = (b1 & ~(size_t)15) > q0 ? (b1 & ~(size_t)15) : q0;
        for (size_t i = q0 + 16 * tid; i < q1; i += 16 * nth)
            *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
        for (size_t i = b0 + tid; i < (q0 < b1 ? q0 : b1); i += nth) dst[i] = src[i];
        for (size_t i = q1 + tid; i < b1; i += nth) dst[i] = src[i];
    }
}

// The wide sweep's partitioned footer (its kernels have no fused last-workgroup step): this
// rank's Cviol, sorted events and flags into its region of the next-colour buffer.
__global__ __launch_bounds__(kCommitThreads) void wide_footer_kernel(SweepArgs a) {
    __shared__ uint32_t lds[kLdsSortCap];
    __shared__ uint32_t sh_done, sh_t, sh_E, sh_err;
    __shared__ unsigned long long sh_viol;
    DevState* st = a.st;
    if (threadIdx.x < 4) a.wcount[threadIdx.x] = 0;   // the walk list, for the next sweep
    if (threadIdx.x == 0) {
        sh_done = st->done;
        sh_t = st->t;
        sh_viol = st->viol;
        sh_E = st->ev_count;
        sh_err = st->err;
    }
    __syncthreads();
    if (sh_done) return;
    uint32_t* ev = nullptr;
    bool sorted = false;
    const uint32_t E = wide_block_events(a, sh_E, lds, kLdsSortCap, &ev, &sorted);
    pack_footer(a, sh_t, sh_viol, E, sh_err, lds, kLdsSortCap, sorted ? ev : nullptr);
}

// ----------------------------------------------------------------------------------------------
// evaluate_core: the caller has loaded lane j's own colour cv and taboo counter tab and computed
// x = the minstd state after draw v + 1 of this sweep (x_t 16807^(v+1) mod 2^31-1).
// evaluate_lane: lane-wise form -- this lane evaluates local row l when `valid` (any rows per lane,
// not necessarily consecutive: the tail queue's entries); every lane of the wave calls it.
// ew (LDS, or nullptr): the closed-form own-colour walk (SweepArgs::ewalk) -- for fill_p's cases
// (i)/(iii) the CDF before colour c < cv is E[c+1], at cv it is S = fl(E[cv] + hi), and after it adding
// eps leaves S unchanged (checked on the host for every colour), so once u >= E[cv] the walk's answer
// is cv when S > u, else a CDF overflow; below E[cv] (probability ~E[cv], < 3e-6 at eps 1e-8) the
// step-by-step walk runs. Bit-identical to the loop.
// The dense sweep's per-workgroup staging of evaluate_lane's list appends (restore list, count
// list, overflow events) in LDS: a wave that appends pays an LDS atomic instead of a global round
// trip; the workgroup flushes once at its end (dc_stage_flush). Full stages fall back to the
// global appends.
constexpr uint32_t kDcStageChg = 4096, kDcStageS = 2048, kDcStageEv = 1024;
struct DcStage {
    uint32_t n[3];      // entries staged: restore list, count list (pairs), events
    uint32_t* chg;      // [kDcStageChg]
    uint32_t* s;        // [2 kDcStageS]
    uint32_t* ev;       // [kDcStageEv]
};
// lane 0 reserves `cnt` entries of stage list i (cap entries); returns the base or ~0u when full
__device__ __forceinline__ uint32_t dc_stage_reserve(uint32_t* n, uint32_t cnt, uint32_t cap, int lane) {
    uint32_t b = 0;
    if (lane == 0) {
        b = atomicAdd(n, cnt);
        if (b + cnt > cap) b = ~0u;
    }
    return __shfl(b, 0, 64);
}

template <int NW>
__device__ __forceinline__ uint32_t evaluate_lane(const SweepArgs& a, DevState* __restrict__ st,
                                                  uint8_t* __restrict__ Cs, bool valid, uint32_t l,
                                                  const uint32_t (&acc)[NW], int lane, uint32_t& ev_flag,
                                                  uint8_t* __restrict__ vf, uint32_t cv, uint32_t tab, uint32_t x,
                                                  const float2* ew = nullptr, DcStage* stg = nullptr) {
    const uint32_t v = a.v_begin + l;
    uint32_t pop = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) pop += __popc(acc[i]);
    const bool viol = valid && get_color_bit<NW>(acc, cv);
    const uint32_t Zvcomp = a.nCol - pop;
    if (vf != nullptr && valid) vf[l] = viol;   // Cviols of C_t (coloringMCMC_CPU.cpp:152)
    const float u = minstd_canonical(x);

    // fill_p cases: (ii) viol with free colours -> occupied eps, free pf;
    //               (i)/(iii) otherwise      -> own colour hi, others eps.
    uint32_t sel[NW];
    float pA, pB;
    if (viol && Zvcomp > 0) {
#pragma unroll
        for (int i = 0; i < NW; i++) sel[i] = acc[i];
        pA = a.eps;
        pB = (1.0f - a.eps * (float)pop) / (float)Zvcomp;
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) sel[i] = 0;
        set_color_bit<NW>(sel, cv);
        pA = a.hi;
        pB = a.eps;
    }
    // extract_new_color: cdf += p[c]; break on cdf > u (strict).
    uint32_t newc = a.nCol;
    bool walked = false;
    if (ew != nullptr && valid && tab == 0 && !(viol && Zvcomp > 0)) {
        const float2 es = ew[cv];
        if (u >= es.x) {
            newc = (es.y > u) ? cv : a.nCol;
            walked = true;
        }
    }
    if (valid && tab == 0 && !walked) {
        float cdf = 0.0f;
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const uint32_t bits = sel[i];
            const uint32_t cmax = min(32u, a.nCol > (uint32_t)(32 * i) ? a.nCol - 32u * i : 0u);
            for (uint32_t cc = 0; cc < cmax && newc == a.nCol; cc++) {
                cdf += ((bits >> cc) & 1u) ? pA : pB;
                if (cdf > u) newc = 32u * i + cc;
            }
        }
    }
    const bool event = valid && tab == 0 && newc == a.nCol;
    if (valid) {
        if (tab > 0) {
            Cs[v] = (uint8_t)cv;
            a.taboo[l] = tab - 1;
        } else if (!event) {
            Cs[v] = (uint8_t)newc;
            if (a.taboo != nullptr) a.taboo[l] = (newc == cv) ? a.tabooIteration : 0u;
        } else {
            Cs[v] = (uint8_t)cv;   // placeholder, overwritten by the commit's glibc replay
        }
    }

    // partitioned delta exchange (a.dcap > 0): this rank's vertices whose colour changed, as (v, c)
    // pairs in its delta slot of the next-colour parity; overflow events are left out (every rank
    // replays them), so a slot lists exactly the other vertices where C_t+1 differs from C_t
    if (a.dcap) {
        const bool chg = valid && tab == 0 && !event && newc != cv;
        const uint64_t cb = __ballot(chg);
        if (cb) {
            uint32_t* dl = (Cs == a.colors1) ? a.dlt1 : a.dlt0;
            uint32_t based = 0;
            if (lane == 0) based = atomicAdd(dl, (uint32_t)__popcll(cb));
            based = __shfl(based, 0, 64);
            const uint32_t idx = based + (uint32_t)__popcll(cb & ((1ull << lane) - 1ull));
            if (chg && idx < a.dcap) {
                dl[kDeltaHead + 2u * idx] = v;
                dl[kDeltaHead + 2u * idx + 1u] = newc;
            }
        }
    }
    // dense-count sweep: the vertices whose colour changes (events aside: the commit's replay lists
    // those) -- every one on the restore list, those of S on the count list (pairs with both colours)
    if (a.dc_list != nullptr) {
        const bool dchg = valid && tab == 0 && !event && newc != cv;
        const uint64_t db = __ballot(dchg);
        const bool ins0 = dchg && v - a.dc_s0 < a.dc_s1 - a.dc_s0;
        const uint64_t sb0 = __ballot(ins0);
        bool staged = false;
        if (db && stg != nullptr) {
            const uint64_t below = (1ull << lane) - 1ull;
            const uint32_t bc = dc_stage_reserve(&stg->n[0], (uint32_t)__popcll(db), kDcStageChg, lane);
            const uint32_t bs = sb0 ? dc_stage_reserve(&stg->n[1], (uint32_t)__popcll(sb0), kDcStageS, lane) : 0u;
            if (bc != ~0u && bs != ~0u) {
                if (dchg) stg->chg[bc + (uint32_t)__popcll(db & below)] = v;
                if (ins0) {
                    const uint32_t j = bs + (uint32_t)__popcll(sb0 & below);
                    stg->s[2u * j] = v;
                    stg->s[2u * j + 1u] = (cv << 16) | newc;
                }
                staged = true;
            }   // else a full stage: this wave's entries go global; what it reserved stays ~0u
                // (the stage is pre-filled), a hole the flush skips
        }
        if (db && !staged) {
            const uint32_t q = (Cs == a.colors1) ? 1u : 0u;   // (t + 1) & 1
            const bool ins = ins0;
            const uint64_t sb = sb0;
            uint32_t bc = 0, bs = 0;
            if (lane == 0) {
                bc = atomicAdd(&a.dc_ctl[kDcChgLen + q], (uint32_t)__popcll(db));
                if (sb) bs = atomicAdd(&a.dc_ctl[kDcLen + q], (uint32_t)__popcll(sb));
            }
            bc = __shfl(bc, 0, 64);
            bs = __shfl(bs, 0, 64);
            const uint64_t below = (1ull << lane) - 1ull;
            if (dchg) {
                const uint32_t j = bc + (uint32_t)__popcll(db & below);
                if (j < a.dc_chg_cap) a.dc_chg[(size_t)q * a.dc_chg_cap + j] = v;
                else a.dc_ctl[kDcChgOvf + q] = 1u;
            }
            if (ins) {
                const uint32_t j = bs + (uint32_t)__popcll(sb & below);
                if (j < a.dc_cap) {
                    uint32_t* e = a.dc_list + 2u * ((size_t)q * a.dc_cap + j);
                    e[0] = v;
                    e[1] = (cv << 16) | newc;
                } else {
                    a.dc_ctl[kDcOvf + q] = 1u;
                }
            }
            ev_flag = 1u;   // the commit reads the lists' lengths: this workgroup releases (sweep_tail)
        }
    }

    const uint32_t nviol = (uint32_t)__popcll(__ballot(viol));
    uint64_t eb = __ballot(event);
    if (eb && stg != nullptr) {
        const uint32_t be = dc_stage_reserve(&stg->n[2], (uint32_t)__popcll(eb), kDcStageEv, lane);
        if (be != ~0u) {
            if (event) stg->ev[be + (uint32_t)__popcll(eb & ((1ull << lane) - 1ull))] = v;
            eb = 0;
        }
    }
    if (eb) {
        ev_flag = 1u;
        uint32_t basei = 0;
        if (lane == 0) basei = atomicAdd(&st->ev_count, (uint32_t)__popcll(eb));
        basei = __shfl(basei, 0, 64);
        if (event) {
            const uint32_t idx = basei + (uint32_t)__popcll(eb & ((1ull << lane) - 1ull));
            if (idx < a.ev_cap) a.events[idx] = v;
            else atomicOr(&st->err, kDevErrEvents);
        }
    }
    return nviol;
}

template <int NW>
__device__ __forceinline__ uint32_t evaluate_core(const SweepArgs& a, DevState* __restrict__ st,
                                                  uint8_t* __restrict__ Cs, uint32_t l0, uint32_t cnt,
                                                  const uint32_t (&acc)[NW], int lane, uint32_t& ev_flag,
                                                  uint8_t* __restrict__ vf, uint32_t cv, uint32_t tab, uint32_t x) {
    return evaluate_lane<NW>(a, st, Cs, (uint32_t)lane < cnt, l0 + lane, acc, lane, ev_flag, vf, cv, tab, x);
}

// Per-vertex evaluation of one tile, after the occupancy masks are built: lane j < cnt holds the
// mask of vertex v = v_begin + l0 + j in `acc`. viol, fill_p, u_v, the CDF walk, the writes, the
// Cviol ballot and the overflow-event append.
template <int NW>
__device__ __forceinline__ uint32_t evaluate_tile(const SweepArgs& a, DevState* __restrict__ st,
                                              const uint8_t* __restrict__ Cown, uint8_t* __restrict__ Cs,
                                              uint32_t x_t, uint32_t l0, uint32_t cnt, const uint32_t (&acc)[NW],
                                              int lane, uint32_t& ev_flag, uint8_t* __restrict__ vf) {
    const bool valid = (uint32_t)lane < cnt;
    const uint32_t l = l0 + lane;
    const uint32_t cv = valid ? (uint32_t)Cown[a.v_begin + l] : 0u;
    const uint32_t tab = (a.taboo != nullptr && valid) ? a.taboo[l] : 0u;
    // u_v: engine draw K_t + v + 1 (bulk draw in vertex order, coloringMCMC_CPU.cpp:139)
    const uint32_t base = minstd_pow_tab_wave((uint64_t)(a.v_begin + l0) + 1);
    const uint32_t x = minstd_mulmod(minstd_mulmod(x_t, base), kMinstdLanePow[lane]);
    return evaluate_core<NW>(a, st, Cs, l0, cnt, acc, lane, ev_flag, vf, cv, tab, x);
}

// ----------------------------------------------------------------------------------------------
// The fused sweep. Every wave owns a contiguous, arc-balanced range of rows (wave_start, computed
// once per context) and walks it in tiles of `tile` vertices. For each vertex of the tile the 64 lanes stream its CSR
// row in passes of 64 x 16 B x U (aligned dwordx4 loads of neighbour ids, the next pass issued
// before the current one is consumed), gather the neighbours' colours and OR them into the
// occupancy mask; a wave OR-reduction leaves vertex j's mask in lane j. Then evaluate_tile.
// LDSC: the whole colour replica (n bytes) is first staged in LDS so the byte gathers never pull
// cache lines through L1/L2 (1 persistent 1024-thread workgroup per CU).
#ifndef MCMC_PASS_U
#define MCMC_PASS_U 4
#endif
constexpr int kPassU = MCMC_PASS_U;          // dwordx4 loads per lane per pass
constexpr uint32_t kPassArcs = 256u * kPassU;

// Streams the CSR rows of one wave tile and leaves the occupancy mask of row j in lane j's `acc`.
// Lane j < cnt holds its row's arc range [rb, re) relative to `tcol` (a 16-B aligned, wave-uniform
// base). Rows are read in passes of 64 lanes x U dwordx4; the next pass is issued before the
// current one is consumed; loads are clamped instead of branched (countable vmcnt); every loaded
// word is a valid vertex id (rows are contiguous, the array tail is zero-padded), so all 4U colour
// gathers issue unmasked -- Cg[(w - gbase) & gmask] -- and a per-quad row mask gates the merge.
template <int NW>
__device__ __forceinline__ void scan_tile(const uint32_t* __restrict__ tcol, const uint8_t* __restrict__ Cg,
                                          uint32_t gbase, uint32_t gmask, uint32_t rb, uint32_t re,
                                          uint32_t cnt, int lane, uint32_t (&acc)[NW]) {
#pragma unroll
    for (int i = 0; i < NW; i++) acc[i] = 0;
    uint32_t j = 0, pbeg = 0, pend = 0;
    while (j < cnt) {   // first non-empty row
        pbeg = __builtin_amdgcn_readlane(rb, j);
        pend = __builtin_amdgcn_readlane(re, j);
        if (pend > pbeg) break;
        j++;
    }
    uint32_t pbase = pbeg & ~3u;
    uint4 cur[kPassU];
#pragma unroll
    for (int u = 0; u < kPassU; u++) {
        const uint32_t q = min(pbase + 256u * u + 4u * lane, (pend - 1u) & ~3u);
        cur[u] = *reinterpret_cast<const uint4*>(tcol + (j < cnt ? q : 0u));
    }
    uint32_t m[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) m[i] = 0;

    while (j < cnt) {
        // next pass (wave-uniform): same row, or the next non-empty row of the tile
        uint32_t nj = j, nbeg = pbeg, nend = pend, nbase = pbase + kPassArcs;
        const bool row_done = nbase >= pend;
        if (row_done) {
            nj = j + 1;
            while (nj < cnt) {
                nbeg = __builtin_amdgcn_readlane(rb, nj);
                nend = __builtin_amdgcn_readlane(re, nj);
                if (nend > nbeg) break;
                nj++;
            }
            nbase = nbeg & ~3u;
            if (nj >= cnt) { nbeg = pbeg; nend = pend; nbase = pbase; }   // nothing left: re-read (hits)
        }
        uint4 nxt[kPassU];
#pragma unroll
        for (int u = 0; u < kPassU; u++) {
            const uint32_t q = min(nbase + 256u * u + 4u * lane, (nend - 1u) & ~3u);
            nxt[u] = *reinterpret_cast<const uint4*>(tcol + q);
        }
        uint32_t qm[kPassU];
#pragma unroll
        for (int u = 0; u < kPassU; u++) {
            const int32_t q = (int32_t)(pbase + 256u * u + 4u * lane);
            const int32_t lo = min(max((int32_t)pbeg - q, 0), 4);
            const int32_t hi = min(max((int32_t)pend - q, 0), 4);
            qm[u] = (0xFu << lo) & ((1u << hi) - 1u);
        }
        uint32_t cg[4 * kPassU];
#pragma unroll
        for (int u = 0; u < kPassU; u++) {
            cg[4 * u + 0] = Cg[(cur[u].x - gbase) & gmask];
            cg[4 * u + 1] = Cg[(cur[u].y - gbase) & gmask];
            cg[4 * u + 2] = Cg[(cur[u].z - gbase) & gmask];
            cg[4 * u + 3] = Cg[(cur[u].w - gbase) & gmask];
        }
#pragma unroll
        for (int i = 0; i < 4 * kPassU; i++) {
            const uint32_t ok = (qm[i >> 2] >> (i & 3)) & 1u;
            if (NW == 1) {
                m[0] |= ok << cg[i];
            } else {
                const uint32_t c = cg[i];
                const uint32_t bit = ok << (c & 31);
#pragma unroll
                for (int w = 0; w < NW; w++) m[w] |= ((c >> 5) == (uint32_t)w) ? bit : 0u;
            }
        }
        if (row_done) {
#pragma unroll
            for (int i = 0; i < NW; i++) {
                const uint32_t r = wave_or_uniform(m[i]);
                acc[i] = ((uint32_t)lane == j) ? r : acc[i];
            }
#pragma unroll
            for (int i = 0; i < NW; i++) m[i] = 0;
        }
        j = nj;
        pbeg = nbeg;
        pend = nend;
        pbase = nbase;
#pragma unroll
        for (int u = 0; u < kPassU; u++) cur[u] = nxt[u];
    }
}

// Shared tail of every sweep kernel: Cviol per workgroup, then (fused) the last-arriving
// workgroup runs the commit (single context) or packs this rank's footer (partitioned).
// Fused protocol (MI355X_MICROARCH.md "Workgroup dispatch ... visibility"): every storing wave
// drains its stores, the workgroup meets, lane 0 publishes Cviol, releases at agent scope and
// arrives; the workgroup whose arrival is last acquires.
struct TailShared {
    uint32_t wg_viol, wg_ev, wg_last, t, E, err;
    uint32_t cursor[2];   // tiled: per-pair row cursor (double-buffered with the pair buffers)
    uint32_t nfull[3];    // tiled early exit: rows of the group whose mask filled up, per pair (mod 3)
    uint32_t dn[2];       // tiled sparse pairs / drain: rows listed (by pair-buffer parity)
    uint32_t st_quads, st_pairs, st_used;   // diagnostics (scan_stats): quads loaded, pairs staged, quads gathered
    uint32_t st_slices, st_qw, st_qr;       // colour slices staged, tail-queue entries written / read
    uint16_t dlist[256];  // tiled sparse pairs / drain: the group's rows whose masks are not full yet
    unsigned long long viol;
    unsigned long long tr[2][4];   // diagnostics (pair trace): scan end min / max over waves, eval end max,
                                   // the evaluation's barrier passed (max)
    uint32_t qn[2];       // tiled tail queue: entries of the two queues
};

// t0 / err0 (when t0 != ~0u): the sweep's t and the error word as every workgroup read them at its
// start; the error word changes during a sweep only where a workgroup appended overflow events, so
// a sweep without events commits with no state load after the arrival.
__device__ __forceinline__ void sweep_tail(const SweepArgs& a, DevState* st, TailShared& sh, uint32_t wave_viol,
                                           uint32_t wave_ev, int lane, uint32_t* lds, uint32_t cap,
                                           uint32_t t0 = ~0u, uint32_t err0 = 0u) {
    if (lane == 0) {
        if (wave_viol) atomicAdd(&sh.wg_viol, wave_viol);
        if (wave_ev) sh.wg_ev = 1u;
    }
    if (!a.fused) {
        __syncthreads();
        if (threadIdx.x == 0 && sh.wg_viol) atomicAdd(&st->viol, (unsigned long long)sh.wg_viol);
        return;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // One packed arrival: [63:48] +1 workgroup, [47:32] +1 if it appended overflow events,
        // [31:0] its Cviol. The events are the only plain stores the committing workgroup reads, so
        // only a workgroup that appended some releases (and the last one acquires only if the
        // packed count says any did): the per-workgroup release fence and second atomic of every
        // sweep are gone.
        const bool ev = sh.wg_ev != 0;
        if (ev) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned long long mine = (1ull << 48) | (ev ? (1ull << 32) : 0ull) | (unsigned long long)sh.wg_viol;
        const unsigned long long prev = atomicAdd(&st->arrive_viol, mine);
        sh.wg_last = ((prev >> 48) == gridDim.x - 1) ? 1u : 0u;
        if (sh.wg_last) {
            const unsigned long long tot = prev + mine;
            sh.viol = tot & 0xFFFFFFFFull;
            if ((tot >> 32) & 0xFFFFull) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                sh.E = __hip_atomic_load(&st->ev_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sh.err = __hip_atomic_load(&st->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                sh.E = 0;
                sh.err = t0 != ~0u ? err0 : __hip_atomic_load(&st->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            sh.t = t0 != ~0u ? t0 : st->t;
        }
    }
    __syncthreads();
    if (!sh.wg_last) return;
    if (a.fused == 1) commit_control(a, sh.t, sh.viol, sh.E, sh.err, lds, cap);
    else pack_footer(a, sh.t, sh.viol, sh.E, sh.err, lds, cap);
}

// REF tail: the packed arrival carries the workgroup's same-colour arc count in [47:0] (REF sweeps
// append no overflow events); the last workgroup runs the reference's loop control.
__device__ __forceinline__ void sweep_tail_ref(const SweepArgs& a, DevState* st, TailShared& sh,
                                               unsigned long long wave_cnt, int lane) {
    if (lane == 0 && wave_cnt) atomicAdd(&sh.viol, wave_cnt);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long mine = (1ull << 48) | sh.viol;
        const unsigned long long prev = atomicAdd(&st->arrive_viol, mine);
        sh.wg_last = ((prev >> 48) == gridDim.x - 1) ? 1u : 0u;
        if (sh.wg_last) {
            sh.viol = (prev + mine) & ((1ull << 48) - 1ull);
            sh.t = st->t;
        }
    }
    __syncthreads();
    if (!sh.wg_last) return;
    commit_control_ref(a, sh.t, sh.viol);
}

// The fused sweep (n fits LDS, or the L2-gather variant). Every wave owns a contiguous,
// arc-balanced range of rows (wave_start, computed once per context) and walks it in tiles.
// LDSC: the whole colour replica (n bytes) is first staged in LDS so the byte gathers never pull
// cache lines through L1/L2 (1 persistent 1024-thread workgroup per CU).
template <int NW, bool LDSC>
__global__ __launch_bounds__(1024) void sweep_kernel(SweepArgs a) {
    extern __shared__ uint4 sc_raw[];
    __shared__ TailShared sh;
    __shared__ uint32_t sort_static[LDSC ? 1 : 2048];
    DevState* __restrict__ st = a.st;
    if (a.check_done && st->done) return;
    if (threadIdx.x == 0) { sh.wg_viol = 0; sh.wg_ev = 0; }
    const uint32_t t = st->t;
    const uint32_t x_t = st->x_t;
    uint8_t* const vf = a.vflags ? a.vflags + (size_t)(t & 1u) * (a.v_end - a.v_begin) : nullptr;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;
    uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;
    const uint8_t* __restrict__ Cg = C;
    if (LDSC) {
        // stage the colour replica: 8 independent 16-B loads in flight per thread
        const uint32_t nq = (a.n + 15u) >> 4;
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(C);
        for (uint32_t i0 = threadIdx.x; i0 < nq; i0 += 8u * blockDim.x) {
            uint4 r[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t i = i0 + k * blockDim.x;
                r[k] = src[i < nq ? i : 0u];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t i = i0 + k * blockDim.x;
                sc_raw[i < nq ? i : 0u] = r[k];   // out-of-range lanes rewrite src[0] at 0: keeps the loads unconditional
            }
        }
        Cg = reinterpret_cast<const uint8_t*>(sc_raw);
    }
    __syncthreads();   // colours staged, sh initialised

    const int lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t wbeg = a.wave_start[gw], wend = a.wave_start[gw + 1];
    uint32_t wave_viol = 0, wave_ev = 0;   // Cviol of this wave's rows; overflow events appended

    for (uint32_t l0 = wbeg; l0 < wend; l0 += a.tile) {
        const uint32_t cnt = min(a.tile, wend - l0);
        uint64_t ob = 0, oe = 0;
        if ((uint32_t)lane < cnt) {
            ob = a.row_off[l0 + lane];
            oe = a.row_off[l0 + lane + 1];
        }
        const uint64_t tb = readlane64(ob, 0) & ~3ull;   // tile-relative 32-bit arc positions
        uint32_t acc[NW];
        scan_tile<NW>(a.col_idx + tb, Cg, 0u, 0xFFFFFFFFu, (uint32_t)(ob - tb), (uint32_t)(oe - tb), cnt, lane, acc);
        wave_viol += evaluate_tile<NW>(a, st, C, Cs, x_t, l0, cnt, acc, lane, wave_ev, vf);
    }
    sweep_tail(a, st, sh, wave_viol, wave_ev, lane, LDSC ? reinterpret_cast<uint32_t*>(sc_raw) : sort_static,
               LDSC ? a.lds_sort_cap : 2048u);
}

// Column-blocked sweep: for colour replicas larger than one workgroup's LDS (multi-GPU replicas,
// n >= 159 Ki). Column block b = vertices [b*B, (b+1)*B) (B = 2^17 uint8 colours = 128 KiB of
// LDS). Each workgroup owns an arc-balanced range of rows (wg_start) and takes it in chunks of R
// rows whose occupancy masks live in LDS; for every column block it stages that colour slice in
// LDS, and its waves pull 8-row tiles (LDS counter) and scan each row's block-b segment
// (seg[b][row], rows ascending) with scan_tile, OR-ing into the chunk masks. After the last block
// the chunk rows are evaluated exactly as in sweep_kernel.
constexpr uint32_t kBlockLog2Max = 17;

template <int NW>
__global__ __launch_bounds__(1024) void sweep_blocked_kernel(SweepArgs a) {
    extern __shared__ uint4 lds_raw[];
    __shared__ TailShared sh;
    __shared__ uint32_t tile_ctr;
    DevState* __restrict__ st = a.st;
    if (a.check_done && st->done) return;
    if (threadIdx.x == 0) { sh.wg_viol = 0; sh.wg_ev = 0; }
    const uint32_t t = st->t;
    const uint32_t x_t = st->x_t;
    uint8_t* const vf = a.vflags ? a.vflags + (size_t)(t & 1u) * (a.v_end - a.v_begin) : nullptr;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;
    uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;
    const uint32_t B = 1u << a.block_log2;
    uint8_t* sc = reinterpret_cast<uint8_t*>(lds_raw);
    uint32_t* smask = reinterpret_cast<uint32_t*>(sc + B);
    const int lane = threadIdx.x & 63;
    const uint32_t wid = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const uint32_t R = a.chunk_rows;
    const uint32_t nb = a.nblocks;
    const uint32_t nloc = a.v_end - a.v_begin;
    const uint32_t gbeg = a.wave_start[blockIdx.x], gend = a.wave_start[blockIdx.x + 1];
    uint32_t wave_viol = 0, wave_ev = 0;

    for (uint32_t c0 = gbeg; c0 < gend; c0 += R) {
        const uint32_t cn = min(R, gend - c0);
        for (uint32_t b = 0; b < nb; b++) {
            __syncthreads();   // previous block's scans (or the previous chunk's evaluation) are done
            if (b == 0)
                for (uint32_t i = threadIdx.x; i < cn * NW; i += blockDim.x) smask[i] = 0;
            // stage colour slice b (16-B chunks; the replica has >= 16 B of slack past n)
            const uint32_t lo = b << a.block_log2;
            const uint32_t bytes = min(B, ((a.n + 15u) & ~15u) - lo);
            const uint4* __restrict__ src = reinterpret_cast<const uint4*>(C + lo);
            for (uint32_t i0 = threadIdx.x; i0 < (bytes >> 4); i0 += 8u * blockDim.x) {
                uint4 r[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t i = i0 + k * blockDim.x;
                    r[k] = src[i < (bytes >> 4) ? i : 0u];
                }
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t i = i0 + k * blockDim.x;
                    lds_raw[i < (bytes >> 4) ? i : 0u] = r[k];
                }
            }
            if (threadIdx.x == 0) tile_ctr = 0;
            __syncthreads();
            const uint32_t* __restrict__ segb = a.seg + (size_t)b * nloc;
            const uint32_t* __restrict__ sege = a.seg + (size_t)(b + 1) * nloc;
            for (;;) {
                uint32_t tt = 0;
                if (lane == 0) tt = atomicAdd(&tile_ctr, 1u);
                tt = __builtin_amdgcn_readfirstlane(tt);
                const uint32_t r0 = tt * 8u;
                if (r0 >= cn) break;
                const uint32_t cnt = min(8u, cn - r0);
                const uint32_t l = c0 + r0 + (uint32_t)lane;
                uint64_t ob = 0, oe = 0;
                if ((uint32_t)lane < cnt) {
                    const uint64_t rs = a.row_off[l];
                    ob = rs + segb[l];
                    oe = rs + sege[l];
                }
                const uint64_t tb = readlane64(a.row_off[c0 + r0], 0) & ~3ull;
                uint32_t acc[NW];
                scan_tile<NW>(a.col_idx + tb, sc, lo, B - 1u, (uint32_t)(ob - tb), (uint32_t)(oe - tb),
                              cnt, lane, acc);
                if ((uint32_t)lane < cnt) {
#pragma unroll
                    for (int i = 0; i < NW; i++) smask[(r0 + lane) * NW + i] |= acc[i];
                }
            }
        }
        __syncthreads();   // all blocks scanned: evaluate the chunk
        for (uint32_t e0 = wid * 64u; e0 < cn; e0 += nwaves * 64u) {
            const uint32_t cnt = min(64u, cn - e0);
            uint32_t acc[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) acc[i] = ((uint32_t)lane < cnt) ? smask[(e0 + lane) * NW + i] : 0u;
            wave_viol += evaluate_tile<NW>(a, st, C, Cs, x_t, c0 + e0, cnt, acc, lane, wave_ev, vf);
        }
    }
    __syncthreads();   // the commit may reuse the colour-slice LDS for its sort
    sweep_tail(a, st, sh, wave_viol, wave_ev, lane, reinterpret_cast<uint32_t*>(lds_raw), B / 4u);
}

// Tiled sweep (variant 3). Group g = local rows [g*R, (g+1)*R); for every column block b the group's
// row segments are contiguous in `tcol` (16-bit block-local ids, each segment padded to whole
// quads of 8 ids), so a dwordx4 load is 8 valid ids of one row. Workgroups take groups
// round-robin. Resident mode (the whole colour replica fits LDS): the replica is staged once and
// block b is the LDS window at b*B; otherwise (2 workgroups/CU) the block's 64 KiB colour slice is
// staged per (group, block). Per block the waves split the group's rows; inside a wave, sub-groups
// of L = 2^sub_log2 lanes walk one row segment each, kTileU quads per lane per step, loads for the
// next step issued before the current step's LDS gathers; a finished segment is OR-reduced over
// its L lanes and OR-ed into the row's LDS mask. After the last block the rows are evaluated.
#ifndef MCMC_TILE_U
#define MCMC_TILE_U 4
#endif
constexpr uint32_t kTileU = MCMC_TILE_U;   // quads per lane per step of the tiled scan

template <int NW>
__device__ __forceinline__ void tile_gather(const uint8_t* __restrict__ sc, const uint4& v, bool ok,
                                            uint32_t (&m)[NW]) {
    // exec-masked: a slot past its segment (about half the slots on C3) issues no LDS reads
    if (ok) {
        const uint32_t w8[4] = {v.x, v.y, v.z, v.w};
        uint32_t cg[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            cg[2 * e] = sc[w8[e] & 0xFFFFu];
            cg[2 * e + 1] = sc[w8[e] >> 16];
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
            if (NW == 1) {
                m[0] |= 1u << cg[e];
            } else {
                const uint32_t c = cg[e];
                const uint32_t bit = 1u << (c & 31);
#pragma unroll
                for (int w = 0; w < NW; w++) m[w] |= ((c >> 5) == (uint32_t)w) ? bit : 0u;
            }
        }
    }
}

// REF scan: the occupancy masks plus the arcs the reference's conflictCounter counts
// (coloringMCMC_utils.cu:115): same colour as the row's (oc) and a larger id (vertex vrow, the
// pair's block starts at whi), not padding (the quad starts at id position q of the group, the
// row's real ids end at tend). cmode (pair-uniform): 0 the block lies below every row of the
// group (no arc counts), 1 above them all (no id test), 2 the diagonal block (id test). Padding
// fills the tail of a segment's last quad with copies of one id, so the count of the 8 ids is
// corrected by (pads) x [element 7 counts] instead of a position test per id.
template <int NW>
__device__ __forceinline__ void tile_gather_ref(const uint8_t* __restrict__ sc, const uint4& v, bool ok,
                                                uint32_t (&m)[NW], uint32_t oc, uint32_t q, uint32_t tend,
                                                uint32_t whi, uint32_t vrow, uint32_t cmode, uint32_t& ecnt) {
    if (ok) {
        const uint32_t w8[4] = {v.x, v.y, v.z, v.w};
        uint32_t id[8], cg[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            id[2 * e] = w8[e] & 0xFFFFu;
            id[2 * e + 1] = w8[e] >> 16;
        }
#pragma unroll
        for (int e = 0; e < 8; e++) cg[e] = sc[id[e]];
        if (cmode == 1) {
            uint32_t c = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) c += cg[e] == oc ? 1u : 0u;
            const uint32_t nv = tend - q;   // >= 1: a quad starts before its segment's real end
            ecnt += c - ((nv < 8u && cg[7] == oc) ? 8u - nv : 0u);
        } else if (cmode == 2) {
            uint32_t c = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) c += (cg[e] == oc && (whi | id[e]) > vrow) ? 1u : 0u;
            const uint32_t nv = tend - q;
            ecnt += c - ((nv < 8u && cg[7] == oc && (whi | id[7]) > vrow) ? 8u - nv : 0u);
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const uint32_t cc = cg[e];
            const uint32_t bit = 1u << (cc & 31);
#pragma unroll
            for (int w = 0; w < NW; w++) m[w] |= ((cc >> 5) == (uint32_t)w) ? bit : 0u;
        }
    }
}

// REF evaluation of one tile (selectStarColoringBalanceDynamic, coloringMCMC_balance.cu:79-143):
// lane j < cnt, vertex l0 + j, occupancy `acc`. Taboo'd: count down, keep the colour (the
// reference leaves the star slot unwritten; it holds the colour of two sweeps before, which equals
// the current one whenever a vertex is taboo'd). No free colour: keep, no draw. Otherwise one
// curand_uniform and the proposal walk: occupied own colour -> free colours p[i] + r with
// r = (sum over occupied of p - eps) / Zp, occupied eps; free own colour -> hi at the own colour,
// eps elsewhere; stop at threshold >= u or i = nCol. A colour >= nCol (initColoring at u = 1.0f)
// occupies nothing (the reference writes it into the next vertex's checker row: a data race).
// States: read at parity t & 1, written (advanced or not) at the other parity.
template <int NW>
__device__ __forceinline__ void evaluate_ref_tile(const SweepArgs& a, const uint8_t* __restrict__ Cown,
                                                  uint8_t* __restrict__ Cs, uint32_t t, uint32_t l0, uint32_t cnt,
                                                  const uint32_t (&acc)[NW], int lane, const float* __restrict__ p,
                                                  uint32_t* hist_lds) {
    if ((uint32_t)lane >= cnt) return;
    const uint32_t l = l0 + (uint32_t)lane, v = a.v_begin + l;
    const size_t nloc = a.v_end - a.v_begin;
    const uint32_t* __restrict__ X = (t & 1u) ? a.xw1 : a.xw0;
    uint32_t* __restrict__ Y = (t & 1u) ? a.xw0 : a.xw1;
    xw::State s;
#pragma unroll
    for (int k = 0; k < xw::kWords; k++) s.v[k] = X[k * nloc + l];
    s.d = X[xw::kWords * nloc + l];
    const uint32_t nodeCol = Cown[v];
    uint32_t star = nodeCol;
    const uint32_t tab = a.taboo ? a.taboo[l] : 0u;
    if (tab > 0) {
        a.taboo[l] = tab - 1u;
    } else {
        uint32_t occ[NW];
        uint32_t Zn = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const uint32_t lo = 32u * i;
            const uint32_t valid = a.nCol >= lo + 32u ? ~0u : (a.nCol > lo ? (1u << (a.nCol - lo)) - 1u : 0u);
            occ[i] = acc[i] & valid;
            Zn += __popc(occ[i]);
        }
        const uint32_t Zp = a.nCol - Zn;
        if (Zp != 0) {
            float reminder = 0.0f;
#pragma unroll
            for (int i = 0; i < NW; i++) {
                uint32_t bits = occ[i];
                while (bits) {
                    const uint32_t b = __builtin_ctz(bits);
                    bits &= bits - 1u;
                    reminder += p[32u * i + b] - a.eps;
                }
            }
            const float u = xw::uniform(xw::next(s));
            const bool own = nodeCol < a.nCol && get_color_bit<NW>(occ, nodeCol);
            const float r = reminder / (float)Zp;
            uint32_t i = 0;
            float thr = 0.0f;
            do {
                const float q = own ? (get_color_bit<NW>(occ, i) ? a.eps : p[i] + r) : (i == nodeCol ? a.ref_hi : a.eps);
                thr += q;
                i++;
            } while (thr < u && i < a.nCol);
            star = i - 1u;
            if (a.taboo) a.taboo[l] = (star == nodeCol) ? a.tabooIteration : 0u;
        }
    }
    Cs[v] = (uint8_t)star;
#pragma unroll
    for (int k = 0; k < xw::kWords; k++) Y[k * nloc + l] = s.v[k];
    Y[xw::kWords * nloc + l] = s.d;
    atomicAdd(&hist_lds[star], 1u);
}

// Streaming mode: the colour slice of a pair (2^block_log2 vertices, at most 2^16) per LDS buffer of
// max(2^block_log2, 16 KiB) bytes (the DMA lands whole wave-instructions: 16 waves x 1 KiB).
__host__ __device__ inline uint32_t tile_slice_buf(uint32_t block_log2) { return 1u << (block_log2 > 14u ? block_log2 : 14u); }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // register-promotable 16 B
typedef __attribute__((address_space(3))) uint8_t lds_u8;

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const lds_u8*)(p); }

// LDS-DMA (global_load_lds_dwordx4): 16 B per lane from `gsrc` to LDS `lds_dst + lane * 16` (`lds_dst`
// wave-uniform). Inline asm, so hipcc's own vmcnt bookkeeping ignores it (cdna_hip_programming.md
// "What hipcc does not do"): its completion is awaited by the counted wait at the pair boundary.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// DMA of pair (g, b) into LDS buffer `buf`: its segment-table row (tseg_stride(R) entries, 16-B
// pieces, 64 per wave-instruction) and, streaming, its colour slice (4096 pieces: 4 per lane).
template <bool RES>
__device__ __forceinline__ void tile_dma_pair(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t g,
                                              uint32_t b, uint32_t seg_lds, uint32_t slice_lds, uint32_t wid,
                                              uint32_t nwaves, int lane, bool slice = true) {
    const uint32_t TS = tseg_stride(a.grp_rows);
    const uint32_t np = TS / 4u;   // 16-B pieces of the table row
    const uint32_t* gs = a.tseg + ((size_t)g * a.nblocks + b) * TS;
    for (uint32_t w = wid; w * 64u < np; w += nwaves) {
        const uint32_t p = min(w * 64u + (uint32_t)lane, np - 1u);
        glds16(gs + 4u * p, __builtin_amdgcn_readfirstlane(seg_lds + w * 1024u));
    }
    if (!RES && slice) {
        const uint32_t lo = b << a.block_log2;
        const uint32_t nq16 = min(a.slice_bytes, ((a.n + 15u) & ~15u) - lo) >> 4;
        // the slice buffer (tile_slice_buf: 16-64 KiB): 1-4 wave-instructions per wave
        const uint32_t kn = tile_slice_buf(a.block_log2) / 1024u / nwaves;
        for (uint32_t k = 0; k < kn; k++) {
            const uint32_t piece = (k * nwaves + wid) * 64u;
            const uint32_t q = min(piece + (uint32_t)lane, nq16 - 1u);
            glds16(C + (lo + 16u * q), __builtin_amdgcn_readfirstlane(slice_lds + piece * 16u));
        }
    }
}

// DMA of column block b's colour slice alone (the tail queue's blocks; no segment table).
__device__ __forceinline__ void tile_dma_slice(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t b,
                                               uint32_t slice_lds, uint32_t wid, uint32_t nwaves, int lane) {
    const uint32_t lo = b << a.block_log2;
    const uint32_t nq16 = min(a.slice_bytes, ((a.n + 15u) & ~15u) - lo) >> 4;
    const uint32_t kn = tile_slice_buf(a.block_log2) / 1024u / nwaves;
    for (uint32_t k = 0; k < kn; k++) {
        const uint32_t piece = (k * nwaves + wid) * 64u;
        const uint32_t q = min(piece + (uint32_t)lane, nq16 - 1u);
        glds16(C + (lo + 16u * q), __builtin_amdgcn_readfirstlane(slice_lds + piece * 16u));
    }
}

// REF, streaming: DMA of group g's own colours (the rows' bytes, from the 16-byte boundary at or
// below the group's first vertex) into an own-colour buffer (a multiple of 1 KiB: every wave
// instruction lands 64 x 16 B).
__device__ __forceinline__ void tile_dma_own(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t g,
                                             uint32_t own_lds, uint32_t wid, uint32_t nwaves, int lane) {
    const uint32_t R = a.grp_rows, nloc = a.v_end - a.v_begin;
    const uint32_t v0 = a.v_begin + g * R, rows = min(R, nloc - g * R);
    const uint32_t base = v0 & ~15u;
    const uint32_t np = (v0 + rows - base + 15u) >> 4;
    for (uint32_t w = wid; w * 64u < np; w += nwaves) {
        const uint32_t q = min(w * 64u + (uint32_t)lane, np - 1u);
        glds16(C + base + 16u * q, __builtin_amdgcn_readfirstlane(own_lds + w * 1024u));
    }
}

// Buffer descriptor over group g's ids: loads at an offset past its end (idle lanes, slots past a
// segment) return 0 without a memory request -- a clamped address would still cost a request (C3:
// 8 lanes/segment 64 ms, 4 lanes 42 ms: the dummy loads were throughput, not free).
constexpr uint32_t kTileOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_group_rsrc(const SweepArgs& a, uint32_t g) {
    const uint64_t p = (uint64_t)(uintptr_t)(a.tcol + a.gbase[g]);
    const uint64_t bytes = 2ull * (a.gbase[g + 1] - a.gbase[g]);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)min<uint64_t>(bytes, 0xFFFFFFF0ull));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, (int)nb,
                                             0x00020000);
}
#ifndef MCMC_TILE_BUFLOAD
#define MCMC_TILE_BUFLOAD 0
#endif
#ifndef MCMC_TILE_NT
#define MCMC_TILE_NT 0
#endif
// One quad of ids at byte offset `byte_off` of the group. MCMC_TILE_BUFLOAD=1: buffer load, slots
// past the end return 0 without a request; 0 (default, measured faster on C3): a plain load
// clamped to the group base.
__device__ __forceinline__ uint4 tile_load(__amdgpu_buffer_rsrc_t r, const uint16_t* gbase_ptr, uint32_t byte_off) {
#if MCMC_TILE_BUFLOAD
    (void)gbase_ptr;
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
    return make_uint4(x.x, x.y, x.z, x.w);
#else
    (void)r;
    const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(gbase_ptr) +
                                                    (byte_off == kTileOOB ? 0u : byte_off));
#if MCMC_TILE_NT
    // ids are read once per sweep: non-temporal, so they do not push the pairs' colour slices
    // (re-staged by every group) and segment tables out of L2
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
#endif
}

// Segment bounds (ids from the group base) of this lane's first row in pair (g, b): sub-group
// (wave w, s) starts at row w * nsub + s; read from the global segment table. Branch-free (rows
// beyond the group read the empty range [s(rows), s(rows)) ), so the loads stay in flight.
__device__ __forceinline__ void tile_first_row(const SweepArgs& a, uint32_t g, uint32_t b, uint32_t nloc,
                                               uint32_t wid, uint32_t nwaves, uint32_t sub,
                                               uint32_t& s0, uint32_t& s1, uint32_t& pads) {
    const uint32_t R = a.grp_rows;
    const uint32_t rows = min(R, nloc - g * R);
    const uint32_t row = wid * (64u >> a.sub_log2) + sub;   // the sub-group's static first row
    const uint32_t* gs = a.tseg + ((size_t)g * a.nblocks + b) * tseg_stride(R);
    const uint32_t raw = gs[min(row, rows)];
    s0 = raw & kTsegPos;
    s1 = gs[min(row + 1, rows)] & kTsegPos;
    pads = raw & 7u;
}

// Pair boundary: this lane's LDS-DMA (issued before at least 6 ordinary vector-memory operations:
// the next pair's 2 first-row bounds and 4 first quads) has landed, this wave's LDS traffic is
// done, then a raw barrier -- the loads issued after the DMA stay in flight across it (a
// __syncthreads() would drain them).
#define MCMC_STR2(x) #x
#define MCMC_STR(x) MCMC_STR2(x)
#define MCMC_PAIR_VMCNT (2 + MCMC_TILE_U)   // the next pair's 2 first-row bounds + its kTileU first quads
#define MCMC_PAIR_BARRIER() \
    asm volatile("s_waitcnt vmcnt(" MCMC_STR(MCMC_PAIR_VMCNT) ") lgkmcnt(0)\n\ts_barrier" ::: "memory")
#define MCMC_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Drain (early exit): the group's rows whose masks are still not full (at most drain_rows, few once
// most rows filled up) finish every remaining column block in this pair, reading their segments'
// bounds and ids from the global layout and the neighbours' colours straight from the replica
// (L2/MALL) -- no more (table, slice) pairs are staged for them. Rounds of 4 blocks: a team of 4
// lanes per (row, block) segment gathers its quads; masks are OR-ed into smask; a round is
// followed by another only while a listed row is not full. All threads call it (uniform).
template <int NW>
__device__ __forceinline__ void drain_quad(const uint8_t* __restrict__ cb, const uint4& v, bool ok, uint32_t (&m)[NW]) {
    if (!ok) return;
    const uint32_t w8[4] = {v.x, v.y, v.z, v.w};
    uint32_t c[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        c[2 * e] = cb[w8[e] & 0xFFFFu];
        c[2 * e + 1] = cb[w8[e] >> 16];
    }
#pragma unroll
    for (int e = 0; e < 8; e++) set_color_bit<NW>(m, c[e]);
}

// The group's rows whose masks are not full yet, into `list` (at most `cap`; ascending inside each
// wave's 64-row chunk, chunks in arrival order); *count = sh.dn[par] (zeroed at the top of the
// previous pair). Ballot compaction, one LDS atomic per wave and chunk. All threads; a barrier follows.
template <int NW>
__device__ __forceinline__ void tile_open_rows(uint32_t rows, const uint32_t* smask, TailShared& sh,
                                               const uint32_t* fullw, uint32_t par, uint16_t* list, uint32_t cap) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r0 = threadIdx.x & ~63u; r0 < rows; r0 += blockDim.x) {
        const uint32_t r = r0 + lane;
        bool open = false;
        if (r < rows) {
            bool f = true;
#pragma unroll
            for (int i = 0; i < NW; i++) f = f && ((smask[r * NW + i] & fullw[i]) == fullw[i]);
            open = !f;
        }
        const uint64_t bm = __ballot(open);
        uint32_t base = 0;
        if (lane == 0 && bm) base = atomicAdd(&sh.dn[par], (uint32_t)__popcll(bm));
        base = __shfl(base, 0, 64);
        if (open) {
            const uint32_t k = base + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
            if (k < cap) list[k] = (uint16_t)r;
        }
    }
    __syncthreads();
}

template <int NW, bool DG>
__device__ __forceinline__ void tile_drain(const SweepArgs& a, const uint8_t* __restrict__ C, uint32_t g, uint32_t b,
                                           uint32_t na, uint32_t* smask, TailShared& sh, const uint32_t* fullw,
                                           int lane) {
    auto row_full = [&](uint32_t r) -> bool {
        bool f = true;
#pragma unroll
        for (int i = 0; i < NW; i++) f = f && ((smask[r * NW + i] & fullw[i]) == fullw[i]);
        return f;
    };
    const uint32_t R = a.grp_rows, TS = tseg_stride(R);
    const uint32_t team = threadIdx.x >> 2, tl = threadIdx.x & 3u, nteams = blockDim.x >> 2;
    const uint16_t* __restrict__ gids = a.tcol + a.gbase[g];
    for (uint32_t bb = b; bb < a.nblocks; bb += 4) {
        for (uint32_t it = team; it < na * 4u; it += nteams) {
            const uint32_t r = sh.dlist[it >> 2], blk = bb + (it & 3u);
            uint32_t m[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) m[i] = 0;
            if (blk < a.nblocks) {
                const uint32_t* ts = a.tseg + ((size_t)g * a.nblocks + blk) * TS;
                const uint32_t s0 = ts[r] & kTsegPos, s1 = ts[r + 1] & kTsegPos;
                const uint8_t* __restrict__ cb = C + ((size_t)blk << a.block_log2);
                // the segment's quads two per lane at once, then their gathers: one memory round
                // trip per two quads instead of per quad
                for (uint32_t q = s0 + 8u * tl; q < s1; q += 64u) {
                    const uint32_t q2 = q + 32u;
                    const uint4 v0 = *reinterpret_cast<const uint4*>(gids + q);
                    const uint4 v1 = *reinterpret_cast<const uint4*>(gids + (q2 < s1 ? q2 : q));
                    drain_quad<NW>(cb, v0, true, m);
                    drain_quad<NW>(cb, v1, q2 < s1, m);
                    if (DG && a.scan_stats) {   // drain quads: loaded and gathered alike
                        atomicAdd(&sh.st_quads, q2 < s1 ? 2u : 1u);
                        atomicAdd(&sh.st_used, q2 < s1 ? 2u : 1u);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < NW; i++) {
                uint32_t x = m[i];
                x |= __shfl_xor(x, 1, 64);
                x |= __shfl_xor(x, 2, 64);
                if (tl == 0 && x) atomicOr(&smask[r * NW + i], x);
            }
        }
        __syncthreads();
        bool open = false;   // every wave reads the same masks: a uniform decision
        for (uint32_t k = (uint32_t)lane; k < na; k += 64u) open = open || !row_full(sh.dlist[k]);
        if (__ballot(open) == 0ull) break;
    }
}

// ---- tail queue (phase B of the early-exit sweep) ---------------------------------------------
// After its last group a workgroup finishes the rows its groups left open after the dense blocks,
// block by block: block b's slice is staged ONCE, then the queue is streamed through it in chunks
// (entries: local row, its mask; per chunk the rows' segment bounds of block b are read into LDS),
// sub-groups claiming entries exactly as rows of a pair (one-ahead loads, ping-pong register sets).
// A row whose mask filled up, or whose blocks ran out, is evaluated (lane per entry, u_v by minstd
// skip-ahead); the others are queued for block b + 1. Rows of ~22 groups share every block: the
// per-group tail pairs (few open rows each: one exposed memory round trip after another, C3 pair 2
// 9.7 us for 737 rows, pair 3 4.8 us, the drain 8.9 us) become a few dense passes.
template <int NW, bool DG>
__device__ __forceinline__ void tail_scan(const SweepArgs& a, const uint8_t* __restrict__ sc,
                                          const uint64_t* E_base, const uint32_t* E_s0, const uint32_t* E_s1,
                                          uint32_t* E_m, uint32_t k, TailShared& sh, const uint32_t (&fullw)[NW],
                                          int lane) {
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t L = 1u << a.sub_log2, nsub = 64u >> a.sub_log2;
    const uint32_t sub = (uint32_t)lane >> a.sub_log2, li = (uint32_t)lane & (L - 1u);
    const uint32_t step = 8u * L * kTileU;
    const uint16_t* __restrict__ tc = a.tcol;
    auto is_full = [&](const uint32_t (&x)[NW]) -> bool {
        bool f = true;
#pragma unroll
        for (int i = 0; i < NW; i++) f = f && ((x[i] & fullw[i]) == fullw[i]);
        return f;
    };
    uint32_t e = wid * nsub + sub, pos = 0, end = 0;
    const uint16_t* rb = tc;
    uint32_t base[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) base[i] = 0;
    if (e < k) {
        pos = E_s0[e] + 8u * li;
        end = E_s1[e];
        rb = tc + E_base[e];
#pragma unroll
        for (int i = 0; i < NW; i++) base[i] = E_m[e * NW + i];
    }
    uint32_t claim = 0;
    if (li == 0) claim = atomicAdd(&sh.cursor[0], 1u);
    uint4 v0[kTileU], v1[kTileU];
#pragma unroll
    for (int u = 0; u < kTileU; u++) {
        const uint32_t pu = pos + 8u * L * u;
        const bool ld = e < k && pu < end;
        if ((DG && a.scan_stats) && ld) atomicAdd(&sh.st_quads, 1u);
        v0[u] = *reinterpret_cast<const uint4*>(ld ? rb + pu : tc);
    }
    uint32_t m[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) m[i] = 0;
    bool rowfull = false;
#define MCMC_TQ_STEP(CUR, NXT, CONT)                                                                    \
    {                                                                                                   \
        const bool act = e < k;                                                                         \
        uint32_t npos2 = pos + step, ne = e, nend2 = end;                                               \
        const uint16_t* nrb = rb;                                                                       \
        uint32_t nbase[NW];                                                                             \
        _Pragma("unroll") for (int i = 0; i < NW; i++) nbase[i] = base[i];                              \
        const bool fin = act && (npos2 - 8u * li >= end || rowfull);                                    \
        if (__ballot(fin)) {                                                                            \
            const uint32_t got = __shfl(claim, (int)(sub << a.sub_log2), 64);                           \
            if (fin) {                                                                                  \
                ne = got;                                                                               \
                if (ne < k) {                                                                           \
                    npos2 = E_s0[ne] + 8u * li;                                                         \
                    nend2 = E_s1[ne];                                                                   \
                    nrb = tc + E_base[ne];                                                              \
                    _Pragma("unroll") for (int i = 0; i < NW; i++) nbase[i] = E_m[ne * NW + i];         \
                }                                                                                       \
                if (li == 0) claim = atomicAdd(&sh.cursor[0], 1u);                                      \
            }                                                                                           \
        }                                                                                               \
        CONT = __ballot(ne < k) != 0;                                                                   \
        if (CONT) {                                                                                     \
            _Pragma("unroll") for (int u = 0; u < kTileU; u++) {                                        \
                const uint32_t pu = npos2 + 8u * L * u;                                                 \
                const bool ld = ne < k && pu < nend2;                                                   \
                if ((DG && a.scan_stats) && ld) atomicAdd(&sh.st_quads, 1u);                            \
                NXT[u] = *reinterpret_cast<const uint4*>(ld ? nrb + pu : tc);                           \
            }                                                                                           \
        }                                                                                               \
        _Pragma("unroll") for (int u = 0; u < kTileU; u++) {                                            \
            const bool ok = act && !rowfull && pos + 8u * L * u < end;                                  \
            tile_gather<NW>(sc, CUR[u], ok, m);                                                         \
            if (DG && a.scan_stats) {                                                                   \
                const uint64_t ub = __ballot(ok);                                                       \
                if (lane == 0 && ub) atomicAdd(&sh.st_used, (uint32_t)__popcll(ub));                    \
            }                                                                                           \
        }                                                                                               \
        const bool chk = act && !fin;                                                                   \
        if (__ballot(fin || chk)) {                                                                     \
            uint32_t red[NW];                                                                           \
            _Pragma("unroll") for (int i = 0; i < NW; i++) {                                            \
                uint32_t x = m[i];                                                                      \
                for (uint32_t off = 1; off < L; off <<= 1) x |= __shfl_xor(x, (int)off, 64);            \
                red[i] = x;                                                                             \
            }                                                                                           \
            if (fin) {                                                                                  \
                if (li == 0) {                                                                          \
                    _Pragma("unroll") for (int i = 0; i < NW; i++)                                      \
                        if (red[i]) atomicOr(&E_m[e * NW + i], red[i]);                                 \
                }                                                                                       \
                _Pragma("unroll") for (int i = 0; i < NW; i++) m[i] = 0;                                \
            } else if (chk) {                                                                           \
                uint32_t nm[NW];                                                                        \
                _Pragma("unroll") for (int i = 0; i < NW; i++) nm[i] = red[i] | base[i];                \
                rowfull = is_full(nm);                                                                  \
            }                                                                                           \
        }                                                                                               \
        if (fin) rowfull = false;                                                                       \
        _Pragma("unroll") for (int i = 0; i < NW; i++) base[i] = nbase[i];                              \
        e = ne;                                                                                         \
        pos = npos2;                                                                                    \
        end = nend2;                                                                                    \
        rb = nrb;                                                                                       \
    }
    if (__ballot(e < k)) {
        for (;;) {
            bool c0, c1;
            MCMC_TQ_STEP(v0, v1, c0)
            if (!c0) break;
            MCMC_TQ_STEP(v1, v0, c1)
            if (!c1) break;
        }
    }
#undef MCMC_TQ_STEP
}

template <int NW, bool DG>
__device__ __forceinline__ void tile_tail(const SweepArgs& a, DevState* __restrict__ st, const uint8_t* __restrict__ C,
                                       uint8_t* __restrict__ Cs, uint8_t* __restrict__ vf, uint8_t* lbase,
                                       uint32_t SB, TailShared& sh, const uint32_t (&fullw)[NW], uint32_t x_t,
                                       int lane, uint32_t& wave_viol, uint32_t& wave_ev, uint32_t kpair,
                                       const float2* ew) {
    const bool ptrace = DG && a.pair_trace != nullptr;
    auto stamp = [&](unsigned long long* rec, int k) {
        if (ptrace && threadIdx.x == 0) rec[k] = wall_clock64();
    };
    const uint32_t R = a.grp_rows, nb = a.nblocks, TS = tseg_stride(R);
    const uint32_t wid = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const uint32_t nsub = 64u >> a.sub_log2;
    auto is_full = [&](const uint32_t (&x)[NW]) -> bool {
        bool f = true;
#pragma unroll
        for (int i = 0; i < NW; i++) f = f && ((x[i] & fullw[i]) == fullw[i]);
        return f;
    };
    // chunk entries in slice buffer 1: base (8 B), s0, s1, row, u_v state, own colour | taboo << 8
    // (4 B each), mask (4 NW B)
    const uint32_t CH = min(2048u, (SB / (28u + 4u * NW)) & ~63u);
    uint64_t* E_base = reinterpret_cast<uint64_t*>(lbase + SB);
    uint32_t* E_s0 = reinterpret_cast<uint32_t*>(E_base + CH);
    uint32_t* E_s1 = E_s0 + CH;
    uint32_t* E_l = E_s1 + CH;
    uint32_t* E_x = E_l + CH;
    uint32_t* E_c = E_x + CH;
    uint32_t* E_m = E_c + CH;
    uint32_t* Q_l = a.tq_l + (size_t)blockIdx.x * 2u * a.tq_cap * 3u;
    uint32_t* Q_m = a.tq_m + (size_t)blockIdx.x * 2u * a.tq_cap * NW;
    const uint32_t lds0 = lds_addr(lbase);
    uint32_t qs = 0;
    for (uint32_t bb = a.tq_dense; bb < nb; bb++) {
        __syncthreads();
        const uint32_t qn = sh.qn[qs];
        if (qn == 0) break;
        __syncthreads();   // every wave has read qn
        if (threadIdx.x == 0) sh.qn[qs ^ 1u] = 0;
        unsigned long long* rec = (ptrace && kpair < kPairTraceMax)
                                      ? a.pair_trace + ((size_t)blockIdx.x * kPairTraceMax + kpair) * kPairTraceRec
                                      : nullptr;
        if (rec) stamp(rec, 0);
        tile_dma_slice(a, C, bb, lds0, wid, nwaves, lane);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // the slice landed
        if (rec) stamp(rec, 1);
        uint64_t t_load = 0, t_scan = 0, t_cls = 0;
        if ((DG && a.scan_stats) && threadIdx.x == 0) {
            sh.st_slices++;
            sh.st_qr += qn;
        }
        const uint32_t* Ql = Q_l + (size_t)qs * a.tq_cap * 3u;
        const uint32_t* Qm = Q_m + (size_t)qs * a.tq_cap * NW;
        uint32_t* Pl = Q_l + (size_t)(qs ^ 1u) * a.tq_cap * 3u;
        uint32_t* Pm = Q_m + (size_t)(qs ^ 1u) * a.tq_cap * NW;
        const bool lastb = bb + 1 == nb;
        for (uint32_t c0 = 0; c0 < qn; c0 += CH) {
            const uint32_t k = min(CH, qn - c0);
            for (uint32_t e = threadIdx.x; e < k; e += blockDim.x) {
                const uint32_t l = Ql[(size_t)(c0 + e) * 3u];
                E_x[e] = Ql[(size_t)(c0 + e) * 3u + 1u];
                E_c[e] = Ql[(size_t)(c0 + e) * 3u + 2u];
                const uint32_t g = l / R, r = l - g * R;
                const uint32_t* ts = a.tseg + ((size_t)g * nb + bb) * TS;
                E_base[e] = a.gbase[g];
                E_s0[e] = ts[r] & kTsegPos;
                E_s1[e] = ts[r + 1] & kTsegPos;
                E_l[e] = l;
#pragma unroll
                for (int i = 0; i < NW; i++) E_m[e * NW + i] = Qm[(size_t)(c0 + e) * NW + i];
            }
            if (threadIdx.x == 0) sh.cursor[0] = nwaves * nsub;
            const uint64_t w0 = ptrace ? wall_clock64() : 0;
            __syncthreads();
            const uint64_t w1 = ptrace ? wall_clock64() : 0;
            tail_scan<NW, DG>(a, lbase, E_base, E_s0, E_s1, E_m, k, sh, fullw, lane);
            __syncthreads();
            const uint64_t w2 = ptrace ? wall_clock64() : 0;
            t_load += w1 - w0;
            t_scan += w2 - w1;
            // full (or out of blocks): evaluate; else queue for block bb + 1
            for (uint32_t e0 = wid * 64u; e0 < k; e0 += nwaves * 64u) {
                const uint32_t e = e0 + (uint32_t)lane;
                const bool in = e < k;
                uint32_t acc[NW];
#pragma unroll
                for (int i = 0; i < NW; i++) acc[i] = in ? E_m[e * NW + i] : 0u;
                const uint32_t l = in ? E_l[e] : 0u;
                const bool done = in && (lastb || is_full(acc));
                const bool keep = in && !done;
                const uint64_t km = __ballot(keep);
                if (km) {
                    uint32_t qb = 0;
                    if (lane == 0) qb = atomicAdd(&sh.qn[qs ^ 1u], (uint32_t)__popcll(km));
                    if ((DG && a.scan_stats) && lane == 0) atomicAdd(&sh.st_qw, (uint32_t)__popcll(km));
                    qb = __shfl(qb, 0, 64);
                    if (keep) {
                        const uint32_t idx = qb + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
                        Pl[(size_t)idx * 3u] = l;
                        Pl[(size_t)idx * 3u + 1u] = E_x[e];
                        Pl[(size_t)idx * 3u + 2u] = E_c[e];
#pragma unroll
                        for (int i = 0; i < NW; i++) Pm[(size_t)idx * NW + i] = acc[i];
                    }
                }
                uint32_t cv = 0, tab = 0, x = 0;
                if (done) {   // everything from the entry: no global load in this loop
                    const uint32_t ct = E_c[e];
                    cv = ct & 0xFFu;
                    tab = ct >> 8;
                    x = E_x[e];
                }
                wave_viol += evaluate_lane<NW>(a, st, Cs, done, l, acc, lane, wave_ev, vf, cv, tab, x, ew);
            }
            __syncthreads();
            if (ptrace) t_cls += wall_clock64() - w2;
        }
        if (rec && threadIdx.x == 0) {   // tail block: slice staged, entry loads, scans, classify (durations)
            rec[2] = t_load;
            rec[3] = t_scan;
            rec[4] = t_cls;
            rec[5] = (unsigned long long)bb | ((unsigned long long)qn << 16) | (1ull << 39);
        }
        kpair++;
        qs ^= 1u;
    }
}

// RES: the whole replica is LDS-resident; otherwise the colour slice of each pair. One 1024-thread
// workgroup per CU (two smaller ones per CU were measured to split the CU's issue unevenly: the
// younger finished 30% later and the tail ran at half occupancy). A workgroup walks its
// (group, block) pairs in order. LDS: [replica | slice buffers 0, 1] [segment-table buffers 0, 1]
// [row masks]. While pair k is scanned from buffer k&1, pair k+1's table (and slice) arrive in
// buffer (k+1)&1 by LDS-DMA, and pair k+1's first quads are issued before the boundary barrier,
// so no pair starts from an empty memory pipeline (the register-landing design spent 38% of the
// C3 sweep at pair boundaries).
// REF: the reference-GPU-semantics sweep on the same pipeline -- the scan also counts the rows'
// same-colour arcs (own colours from the replica, or streamed per group into LDS), the evaluation
// is evaluate_ref_tile, the arrival carries the count (sweep_tail_ref).
// DG: the diagnostics instantiation (scan_stats counters, MCMC_PHASE_DUMP cycle accounting,
// kept out of the timed kernels' registers.
template <int NW, bool RES, bool REF, bool EX, bool DG = false>
__global__ __launch_bounds__(1024) void sweep_tiled_kernel(SweepArgs a) {
    extern __shared__ uint4 lds_raw[];
    __shared__ TailShared sh;
    DevState* __restrict__ st = a.st;
    // loads that depend on the launch alone go out beside the state words: the first pair's
    // first-row bounds and (u_v) this wave's first-row power
    const uint32_t wid0 = threadIdx.x >> 6;
    const uint32_t gclamp = min(blockIdx.x, a.ngroups ? a.ngroups - 1u : 0u);
    uint32_t fpos, fend, fpads;
    tile_first_row(a, gclamp, 0, a.v_end - a.v_begin, wid0, blockDim.x >> 6, (threadIdx.x & 63u) >> a.sub_log2,
                   fpos, fend, fpads);
    const uint32_t gp = (!REF && a.gpow != nullptr && blockIdx.x < a.ngroups) ? a.gpow[(size_t)blockIdx.x * 16u + wid0] : 0u;
    if (a.check_done && st->done) return;
    MCMC_PHASE(a, 0);
    if (threadIdx.x == 0) { sh.wg_viol = 0; sh.wg_ev = 0; sh.viol = 0; }
    const uint32_t t = st->t;
    const uint32_t x_t = st->x_t;
    const uint32_t err0 = st->err;
    uint8_t* const vf = a.vflags ? a.vflags + (size_t)(t & 1u) * (a.v_end - a.v_begin) : nullptr;
    const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;
    uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;
    uint8_t* lbase = reinterpret_cast<uint8_t*>(lds_raw);
    // the closed-form own-colour walk's table in LDS (landed by the first barrier below)
    const float2* ew = nullptr;
    if (!REF && a.ewalk_off && a.ewalk) {
        float2* ewl = reinterpret_cast<float2*>(lbase + a.ewalk_off);
        for (uint32_t i = threadIdx.x; i < a.nCol; i += blockDim.x) ewl[i] = a.ewalk[i];
        ew = ewl;
    }
    const uint32_t R = a.grp_rows, nb = a.nblocks;
    const uint32_t SB = RES ? a.slice_bytes : tile_slice_buf(a.block_log2);   // bytes per colour buffer
    uint8_t* seg_base = lbase + (RES ? SB : 2u * SB);
    const uint32_t SEGB = a.seg_buf_bytes;                              // bytes per table buffer
    uint32_t* smask = reinterpret_cast<uint32_t*>(seg_base + 2u * SEGB);
    // early exit, listed pairs: the group's open rows (R entries) after the masks (a.olist_on)
    uint16_t* olist = reinterpret_cast<uint16_t*>(smask + R * NW);
    // REF: [dynamic distribution p (256 floats)][new-colour histogram][2 own-colour buffers]
    float* p_lds = reinterpret_cast<float*>(seg_base + 2u * SEGB + ((R * NW * 4u + 15u) & ~15u));
    uint32_t* hist_lds = reinterpret_cast<uint32_t*>(p_lds + 256);
    uint8_t* own_base = reinterpret_cast<uint8_t*>(hist_lds + kHistWords);
    if (REF) {
        // genDynamicDistribution (coloringMCMC_utils.cu:64-70) from C_t's histogram
        const uint32_t* __restrict__ H = a.hist + (t & 1u) * a.hist_words;
        for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x) hist_lds[i] = 0;
        for (uint32_t c = threadIdx.x; c < a.nCol; c += blockDim.x)
            p_lds[c] = (1.0f - ((float)H[c] / (float)a.n)) / (float)(a.nCol - 1u);
    }
    uint32_t ecnt = 0;      // REF: same-colour arcs scanned by this lane
    uint32_t gpar = 0;      // REF streaming: own-colour buffer of the current group
    const int lane = threadIdx.x & 63;
    const uint32_t wid = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const uint32_t L = 1u << a.sub_log2, nsub = 64u >> a.sub_log2;
    const uint32_t sub = (uint32_t)lane >> a.sub_log2, li = (uint32_t)lane & (L - 1u);
    const uint32_t step = 8u * L * kTileU;
    const uint32_t nloc = a.v_end - a.v_begin;
    const uint32_t nbytes16 = (a.n + 15u) & ~15u;
    const uint32_t lds0 = lds_addr(lbase), seg_lds0 = lds_addr(seg_base);
    uint32_t wave_viol = 0, wave_ev = 0;
    const uint32_t lpow = REF ? 0u : kMinstdLanePow[lane];   // 16807^lane: read once, before any scan load
    const bool timing = DG && a.phase_ts != nullptr;
    const bool ptrace = DG && a.pair_trace != nullptr;
    unsigned long long tr_start = 0;
    uint64_t cyc_wait = 0, cyc_scan = 0, cyc_eval = 0, tmark = 0;

    uint32_t g = blockIdx.x, b = 0, buf = 0;
    // u_v (evaluation): xg = x_t 16807^(v_begin + g R + 64 wid + 1), the draw of this wave's first
    // evaluation row in group g; xsg advances it by one group of this workgroup, xsk by one tile
    uint32_t xg = 0, xsg = 0, xsk = 0;
    if (!REF && a.gpow != nullptr && nwaves == 16u) {   // host-computed (create_impl)
        xg = minstd_mulmod(x_t, gp);
        xsg = a.apow_grid;
        xsk = a.apow_tile;
    } else if (!REF) {
        xg = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)a.v_begin + (uint64_t)g * R + 64u * wid + 1u));
        xsg = minstd_pow_tab((uint64_t)gridDim.x * R);
        xsk = minstd_pow_tab(64u * (uint64_t)nwaves);
    }
    for (uint32_t i = threadIdx.x; i < R * NW; i += blockDim.x) smask[i] = 0;
    if (threadIdx.x == 0) {
        sh.cursor[0] = nwaves * nsub;
        sh.nfull[0] = sh.nfull[1] = sh.nfull[2] = 0;
        sh.dn[0] = sh.dn[1] = 0;
        sh.qn[0] = sh.qn[1] = 0;
    }
    // Early exit (not REF: its scan counts arcs): a row whose mask holds all nCol colours is done --
    // its later segments are skipped, and once every row of a group is done its remaining pairs are.
    const bool EXIT = EX && !REF && a.early;   // EX = false: the full-scan instantiation (no early-exit code)
    const bool TQ = EXIT && !RES && a.tq_dense != 0 && a.tq_dense < nb;   // the tail queue (tile_tail)
    // with the tail queue's two dense blocks, their slices stay in the two slice buffers for all of
    // phase A (every group's pairs read the same two slices): pairs stage their tables only
    const bool RS = TQ && a.tq_dense == 2u;
    uint32_t fullw[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint32_t lo = 32u * i;
        fullw[i] = a.nCol >= lo + 32u ? ~0u : (a.nCol > lo ? (1u << (a.nCol - lo)) - 1u : 0u);
    }
    auto is_full = [&](const uint32_t (&x)[NW]) -> bool {
        bool f = true;
#pragma unroll
        for (int i = 0; i < NW; i++) f = f && ((x[i] & fullw[i]) == fullw[i]);
        return f;
    };
    uint32_t nfull_run = 0, kpair = 0;   // rows of the current group known full; pair counter
    bool pstaged = true;                 // this pair's table and slice were staged (late staging skips some)
    if (threadIdx.x == 0) {
        sh.st_quads = sh.st_pairs = sh.st_used = sh.st_qw = sh.st_qr = 0;
        sh.st_slices = (RS && g < a.ngroups) ? 2u : 0u;   // the resident dense slices
    }
    if (g < a.ngroups) {
        tile_dma_pair<RES>(a, C, g, 0, seg_lds0, lds0, wid, nwaves, lane);
        if (RS) tile_dma_slice(a, C, 1, lds0 + SB, wid, nwaves, lane);   // block 1's slice, resident too
        if (REF && !RES) tile_dma_own(a, C, g, lds_addr(own_base), wid, nwaves, lane);
    }
    // the first pair's first quads (bounds loaded at the top), then the resident replica
    fpos += 8u * li;
    __amdgpu_buffer_rsrc_t gr = tile_group_rsrc(a, gclamp);
    const uint16_t* __restrict__ gcol = a.tcol + a.gbase[gclamp];
    uint4 v[kTileU];
    uint32_t nq0 = 0;   // scan_stats: quads of the first prefetch (counted after the barrier below)
#pragma unroll
    for (int u = 0; u < kTileU; u++) {
        const uint32_t pu = fpos + 8u * L * u;
        nq0 += pu < fend ? 1u : 0u;
        v[u] = tile_load(gr, gcol, pu < fend ? 2u * pu : kTileOOB);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the staging below the first quads
    if (RES) {
        constexpr int kResPer = 10;   // uint4 per thread: replica <= 160 KiB over 1024 threads
        u32x4 rr[kResPer];
        const uint32_t nq16 = nbytes16 >> 4;
#pragma unroll
        for (int k = 0; k < kResPer; k++) {
            const uint32_t i = threadIdx.x + k * blockDim.x;
            rr[k] = *reinterpret_cast<const u32x4*>(C + (16u * (i < nq16 ? i : 0u)));
        }
#pragma unroll
        for (int k = 0; k < kResPer; k++) {
            const uint32_t i = threadIdx.x + k * blockDim.x;
            reinterpret_cast<u32x4*>(lds_raw)[i < nq16 ? i : 0u] = rr[k];   // (src[0] again at 0)
        }
    }
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // DMA + staging landed
    MCMC_PHASE(a, 1);
    if ((DG && a.scan_stats) && nq0) atomicAdd(&sh.st_quads, nq0);

    while (g < a.ngroups) {
        if (timing) tmark = __builtin_readcyclecounter();
        if (ptrace && threadIdx.x == 0) {
            tr_start = wall_clock64();
            sh.tr[(kpair + 1u) & 1u][0] = ~0ull;
            sh.tr[(kpair + 1u) & 1u][1] = 0;
            sh.tr[(kpair + 1u) & 1u][2] = 0;
            sh.tr[(kpair + 1u) & 1u][3] = 0;
        }
        const uint32_t r0 = g * R;
        const uint32_t rows = min(R, nloc - r0);
        const uint32_t q = (rows + nwaves - 1) / nwaves;   // evaluation share per wave
        // early exit: rows that filled up in the previous pair (slot (k-1) % 3 is final: its pair
        // ended at the barrier); slot (k+1) % 3 was last read at the top of pair k-1 and is next
        // counted into in pair k+1, after this pair's barrier
        bool allfull = false, drain = false, sparse = false;
        if (EXIT) {
            nfull_run = (b == 0) ? 0u : nfull_run + sh.nfull[(kpair + 2u) % 3u];
            allfull = b > 0 && nfull_run >= rows;
            const uint32_t nopen = rows - min(nfull_run, rows);
            // few rows left: they finish every remaining block here (tile_drain), no more pairs
            drain = !allfull && b > 0 && nopen <= a.drain_rows && b + 1 < nb;
            // a listed pair: only the open rows are claimed (not every row of the group) -- few open
            // rows (the 256-entry list), or (a.olist_on) a tenth of the rows or more full: claiming
            // full rows broke the one-row-ahead load pipeline (every open row behind a full one
            // waited a whole memory round trip; C3 pair 2: 12.2 us with 737 of 1776 rows open)
            sparse = !allfull && !drain && b > 0 && (nopen <= 256u || (a.olist_on && 10u * nopen < 9u * rows));
            if (threadIdx.x == 0) {
                sh.nfull[(kpair + 1u) % 3u] = 0;
                sh.dn[buf ^ 1u] = 0;   // the next pair's list counter (its last use: the previous pair)
            }
        }
        // tail queue: the group's last dense pair -- its full rows are evaluated at its end, the open
        // ones queued for tile_tail
        const bool split = TQ && b + 1 == a.tq_dense && !allfull && !drain;
        uint32_t nlist = 0;
        uint16_t* dl = sh.dlist;
        if (drain || sparse) {
            const bool big = sparse && a.olist_on;   // the R-entry list (any number of open rows)
            dl = big ? olist : sh.dlist;
            tile_open_rows<NW>(rows, smask, sh, fullw, buf, dl, big ? R : 256u);
            nlist = min(sh.dn[buf], big ? R : 256u);
        }
        const uint32_t kslot = kpair % 3u;
        // the group's last pair: its last block, every row already full, or the drain
        const bool last = (b + 1 == nb) || allfull || drain || split;
        // the next pair's row cursor (its first nwaves * nsub rows are assigned statically)
        if (threadIdx.x == 0) sh.cursor[buf ^ 1u] = nwaves * nsub;
        // the next pair: its table (and slice) by DMA into the other buffers, its first-row bounds
        const uint32_t ng = last ? g + gridDim.x : g, nbn = last ? 0u : b + 1;
        const bool nvalid = ng < a.ngroups;
        // late staging: the group's next pair is staged after this pair's scan, and not at all once
        // every row is full (the next pair then reads neither buffer); its first-row bounds are read
        // after that DMA too, so the boundary's counted vmcnt still covers it
        const bool late = EXIT && a.late_stage && !last && nvalid && !RES;
        // the evaluated group's own colours by LDS-DMA now, so the evaluation at the pair's end finds
        // them landed (a register load there waited one loaded-HBM round trip, ~5 us per group)
        if (!REF && last && a.eown_off) tile_dma_own(a, C, g, lds0 + a.eown_off, wid, nwaves, lane);
        if (nvalid && !late) {
            tile_dma_pair<RES>(a, C, ng, nbn, seg_lds0 + (buf ^ 1u) * SEGB, lds0 + (buf ^ 1u) * SB, wid, nwaves, lane,
                               !RS);
            if (REF && !RES && nbn == 0)
                tile_dma_own(a, C, ng, lds_addr(own_base) + (gpar ^ 1u) * a.own_buf_bytes, wid, nwaves, lane);
        }
        const uint32_t pg = nvalid ? ng : g, pb = nvalid ? nbn : b;
        uint32_t npos = 0, nend = 0, npads = 0;
        if (!late) {
            tile_first_row(a, pg, pb, nloc, wid, nwaves, sub, npos, nend, npads);
            npos += 8u * li;
            if (!nvalid) nend = npos;   // no next pair: its "first quads" load nothing
        }
        const __amdgpu_buffer_rsrc_t ngr = tile_group_rsrc(a, pg);
        const uint16_t* __restrict__ ngcol = a.tcol + a.gbase[pg];
        const uint8_t* __restrict__ scb = RES ? lbase + (b << a.block_log2) : lbase + (RS ? (b & 1u) : buf) * SB;
        const uint32_t* __restrict__ sseg = reinterpret_cast<const uint32_t*>(seg_base + buf * SEGB);
        // sub-group state: current row, this lane's next quad, the row's end (ids from the group
        // base); the first step's quads are already in v. Rows after the first come from the pair's
        // LDS cursor, claimed one row ahead (dynamic balance across the waves: the static split
        // left 36% of the C3 sweep waiting at pair barriers for the slowest wave).
        uint32_t row = wid * nsub + sub, pos = fpos, end = fend;
        uint32_t tend = fend - fpads;                 // REF: the row's real ids end here
        const uint32_t whi = b << a.block_log2;       // REF: vertex id of the pair's block start
        const uint32_t vlo = a.v_begin + r0;
        const uint32_t cmode = (whi + (1u << a.block_log2) - 1u < vlo) ? 0u : (whi > vlo + rows - 1u) ? 1u : 2u;
        // REF: the own colour of a row of this group (0 past the group: such rows gather nothing)
        const uint8_t* ownp = RES ? lbase + a.v_begin + r0
                                  : own_base + gpar * a.own_buf_bytes + ((a.v_begin + r0) & 15u);
        auto own_of = [&](uint32_t r) -> uint32_t { return r < rows ? (uint32_t)ownp[r] : 0u; };
        uint32_t oc = REF ? own_of(row) : 0u;
        uint32_t claim = 0;
        if (li == 0 && !allfull) claim = atomicAdd(&sh.cursor[buf], 1u);
        uint32_t m[NW];
#pragma unroll
        for (int i = 0; i < NW; i++) m[i] = 0;
        // the row's mask from earlier blocks; a full one makes its segment empty
        uint32_t base[NW];
        bool rowfull = false;
#pragma unroll
        for (int i = 0; i < NW; i++) base[i] = 0;
        if (sparse) {
            // sparse pair: the open rows of the list, the first nwaves * nsub of them assigned to the
            // sub-groups (their first quads reloaded: the prefetched ones are the static rows'),
            // the rest claimed (the cursor starts past them)
            const uint32_t s = wid * nsub + sub;
            row = s < nlist ? (uint32_t)dl[s] : rows;
            if (row < rows) {
                const uint32_t sraw = sseg[row];
                pos = (sraw & kTsegPos) + 8u * li;
                end = sseg[row + 1] & kTsegPos;
#pragma unroll
                for (int i = 0; i < NW; i++) base[i] = smask[row * NW + i];
            }
#pragma unroll
            for (int u = 0; u < kTileU; u++) {
                const uint32_t pu = pos + 8u * L * u;
                if ((DG && a.scan_stats) && row < rows && pu < end) atomicAdd(&sh.st_quads, 1u);
                v[u] = tile_load(gr, gcol, (row < rows && pu < end) ? 2u * pu : kTileOOB);
            }
        } else if (EXIT && b > 0 && row < rows) {
#pragma unroll
            for (int i = 0; i < NW; i++) base[i] = smask[row * NW + i];
            if (is_full(base)) end = pos;
        }
        if ((DG && a.scan_stats) && threadIdx.x == 0 && pstaged) {
            sh.st_pairs++;
            if (!RS && !RES) sh.st_slices++;
        }
        bool nstaged = true;
        // One step: gathers of CUR (this step's quads), loads of the next step into NXT. Expanded
        // twice over ping-pong register sets (a `v = vn` copy at the back-edge made hipcc wait
        // vmcnt(0) before the copy: a one-step-deep pipeline). The wave's last step issues no
        // loads, so nothing is pending into either set when the loop ends; the gathers sit in both
        // branches so each path keeps an exact vmcnt.
#define MCMC_TILE_STEP(CUR, NXT, CONT)                                                                  \
    {                                                                                                   \
        const bool act = row < rows;                                                                    \
        uint32_t npos2 = pos + step, nrow = row, nend2 = end, noc = oc, ntend = tend;                   \
        uint32_t nbase[NW];                                                                             \
        _Pragma("unroll") for (int i = 0; i < NW; i++) nbase[i] = base[i];                              \
        /* the row's last step: its segment ends, or its mask filled up in the previous step */        \
        const bool fin = act && (npos2 - 8u * li >= end || rowfull);                                    \
        if (__ballot(fin)) {                                                                            \
            const uint32_t got = __shfl(claim, (int)(sub << a.sub_log2), 64);                           \
            if (fin) {                                                                                  \
                nrow = got;                                                                             \
                if (sparse) nrow = (got < nlist) ? (uint32_t)dl[got] : rows;                            \
                if (nrow < rows) {                                                                      \
                    const uint32_t sraw = sseg[nrow];                                                   \
                    npos2 = (sraw & kTsegPos) + 8u * li;                                                \
                    nend2 = sseg[nrow + 1] & kTsegPos;                                                  \
                    ntend = nend2 - (sraw & 7u);                                                        \
                    if (EXIT && b > 0) {                                                                \
                        _Pragma("unroll") for (int i = 0; i < NW; i++) nbase[i] = smask[nrow * NW + i]; \
                        if (is_full(nbase)) nend2 = npos2;   /* done in earlier blocks: empty segment */ \
                    }                                                                                   \
                }                                                                                       \
                if (REF) noc = own_of(nrow);                                                            \
                if (li == 0) claim = atomicAdd(&sh.cursor[buf], 1u);                                    \
            }                                                                                           \
        }                                                                                               \
        CONT = __ballot(nrow < rows) != 0;                                                              \
        if (CONT) {                                                                                     \
            _Pragma("unroll") for (int u = 0; u < kTileU; u++) {                                        \
                const uint32_t pu = npos2 + 8u * L * u;                                                 \
                const bool ld = nrow < rows && pu < nend2;                                              \
                if ((DG && a.scan_stats) && ld) atomicAdd(&sh.st_quads, 1u);                                    \
                NXT[u] = tile_load(gr, gcol, ld ? 2u * pu : kTileOOB);                                  \
            }                                                                                           \
            _Pragma("unroll") for (int u = 0; u < kTileU; u++)                                          \
                MCMC_TILE_GATHER(CUR[u], act && !rowfull && pos + 8u * L * u < end, pos + 8u * L * u);  \
        } else {                                                                                        \
            _Pragma("unroll") for (int u = 0; u < kTileU; u++)                                          \
                MCMC_TILE_GATHER(CUR[u], act && !rowfull && pos + 8u * L * u < end, pos + 8u * L * u);  \
        }                                                                                               \
        /* reduce over the sub-group: at a row's end (flush), and each step of a longer row when */  \
        /* early exit can stop it */                                                                   \
        const bool chk = EXIT && act && !fin;                                                           \
        if (__ballot(fin || chk)) {                                                                     \
            uint32_t red[NW];                                                                           \
            _Pragma("unroll") for (int i = 0; i < NW; i++) {                                            \
                uint32_t x = m[i];                                                                      \
                for (uint32_t off = 1; off < L; off <<= 1) x |= __shfl_xor(x, (int)off, 64);            \
                red[i] = x;                                                                             \
            }                                                                                           \
            if (fin) {                                                                                  \
                if (li == 0) {                                                                          \
                    _Pragma("unroll") for (int i = 0; i < NW; i++)                                      \
                        if (red[i]) atomicOr(&smask[row * NW + i], red[i]);                             \
                    if (EXIT) {                                                                         \
                        uint32_t nm[NW];                                                                \
                        _Pragma("unroll") for (int i = 0; i < NW; i++) nm[i] = red[i] | base[i];        \
                        if (is_full(nm) && !is_full(base)) atomicAdd(&sh.nfull[kslot], 1u);             \
                    }                                                                                   \
                }                                                                                       \
                _Pragma("unroll") for (int i = 0; i < NW; i++) m[i] = 0;                                \
            } else if (chk) {                                                                           \
                uint32_t nm[NW];                                                                        \
                _Pragma("unroll") for (int i = 0; i < NW; i++) nm[i] = red[i] | base[i];                \
                rowfull = is_full(nm);                                                                  \
            }                                                                                           \
        }                                                                                               \
        if (fin) rowfull = false;                                                                       \
        _Pragma("unroll") for (int i = 0; i < NW; i++) base[i] = nbase[i];                              \
        row = nrow;                                                                                     \
        pos = npos2;                                                                                    \
        end = nend2;                                                                                    \
        oc = noc;                                                                                       \
        tend = ntend;                                                                                   \
    }
#define MCMC_TILE_GATHER(Q, OK, QPOS)                                                                   \
    do {                                                                                                \
        if (REF) tile_gather_ref<NW>(scb, Q, OK, m, oc, QPOS, tend, whi, a.v_begin + r0 + row, cmode, ecnt); \
        else tile_gather<NW>(scb, Q, OK, m);                                                            \
        if (DG && a.scan_stats) {                                                                       \
            const uint64_t ub = __ballot(OK);                                                           \
            if (lane == 0 && ub) atomicAdd(&sh.st_used, (uint32_t)__popcll(ub));                        \
        }                                                                                               \
    } while (0)
        uint4 v1[kTileU];
        if (drain) {
            tile_drain<NW, DG>(a, C, g, b, nlist, smask, sh, fullw, lane);
        } else if (!allfull && __ballot(row < rows)) {
            for (;;) {
                bool c0, c1;
                MCMC_TILE_STEP(v, v1, c0)
                if (!c0) break;
                MCMC_TILE_STEP(v1, v, c1)
                if (!c1) break;
            }
        }
#undef MCMC_TILE_STEP
#undef MCMC_TILE_GATHER
        if (late) {
            // rows full so far (monotone: a count that reaches `rows` is final) -- every row full means
            // the next pair is all-full and reads neither buffer
            const uint32_t fnow = __builtin_amdgcn_readfirstlane(
                nfull_run + __hip_atomic_load(&sh.nfull[kslot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            const bool af = fnow >= rows;
            nstaged = !af;
            if (!af)
                tile_dma_pair<RES>(a, C, ng, nbn, seg_lds0 + (buf ^ 1u) * SEGB, lds0 + (buf ^ 1u) * SB, wid, nwaves,
                                   lane, !RS);
            tile_first_row(a, pg, pb, nloc, wid, nwaves, sub, npos, nend, npads);
            npos += 8u * li;
            if (af) nend = npos;
        }
        // the evaluation's own colours and taboo counters of this wave's first two tiles, loaded
        // BEFORE the next pair's first quads: vmcnt retires loads in order, so a load issued after
        // those quads would make the evaluation wait for their HBM round trip (C3: 6 us per group)
        const uint32_t tstride = nwaves * 64u;
        uint32_t cvA = 0, tabA = 0, cvB = 0, tabB = 0;
        const uint8_t* eown = lbase + a.eown_off + ((a.v_begin + r0) & 15u);   // a.eown_off: own colours in LDS
        if (!REF && last) {
            const uint32_t ea = wid * 64u + (uint32_t)lane, eb = ea + tstride;
            if (ea < rows) {
                if (!a.eown_off) cvA = C[a.v_begin + r0 + ea];
                if (a.taboo) tabA = a.taboo[r0 + ea];
            }
            if (eb < rows) {
                if (!a.eown_off) cvB = C[a.v_begin + r0 + eb];
                if (a.taboo) tabB = a.taboo[r0 + eb];
            }
        }
        // the next pair's first quads: in flight across the boundary (and the evaluation)
        gr = ngr;
        gcol = ngcol;
        fpos = npos;
        fend = nend;
        fpads = npads;
#pragma unroll
        for (int u = 0; u < kTileU; u++) {
            const uint32_t pu = fpos + 8u * L * u;
            if ((DG && a.scan_stats) && pu < fend) atomicAdd(&sh.st_quads, 1u);
            v[u] = tile_load(gr, gcol, pu < fend ? 2u * pu : kTileOOB);
        }
        if (timing) { const uint64_t t1 = __builtin_readcyclecounter(); cyc_scan += t1 - tmark; tmark = t1; }
        if (ptrace && lane == 0) {
            const unsigned long long w = wall_clock64();
            atomicMin(&sh.tr[kpair & 1u][0], w);
            atomicMax(&sh.tr[kpair & 1u][1], w);
        }
        if (last && REF) {
            MCMC_LDS_BARRIER();   // every wave's mask ORs of the group are in
            // every wave evaluates a share of the group's rows and clears their masks for the next group
            for (uint32_t e0 = wid * min(q, 64u); e0 < rows; e0 += nwaves * min(q, 64u)) {
                const uint32_t cnt = min(min(q, 64u), rows - e0);
                uint32_t acc[NW];
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    const uint32_t idx = (e0 + lane) * NW + i;
                    acc[i] = ((uint32_t)lane < cnt) ? smask[idx] : 0u;
                    if ((uint32_t)lane < cnt) smask[idx] = 0;
                }
                evaluate_ref_tile<NW>(a, C, Cs, t, r0 + e0, cnt, acc, lane, p_lds, hist_lds);
            }
            if (timing) { const uint64_t t1 = __builtin_readcyclecounter(); cyc_eval += t1 - tmark; tmark = t1; }
        } else if (last) {
            // Wave w evaluates rows w * 64 + k * 1024 (64-row tiles) and clears their masks for the
            // next group. Each tile's own colours and taboo counters are loaded two tiles ahead (the
            // first two before the next pair's quads); u_v's minstd state comes from the wave's
            // running base xg = x_t 16807^(v + 1) of its first row (no per-tile power).
            uint32_t e0 = wid * 64u, cv = cvA, tab = tabA;
            // every wave's mask ORs of the group are in, and this wave's DMA of the next pair has
            // landed (the DMA precedes the 6 first-row loads; vmcnt(6) also covers the loads above):
            // the pair's barrier after the evaluation then waits for LDS only, so the evaluation's
            // stores and the next pair's first quads stay in flight across it
            MCMC_PAIR_BARRIER();
            if (ptrace && lane == 0) atomicMax(&sh.tr[kpair & 1u][3], (unsigned long long)wall_clock64());
            uint32_t xk = xg;
            for (; e0 < rows; e0 += tstride) {
                const uint32_t cnt = min(64u, rows - e0);
                const uint32_t e2 = e0 + 2u * tstride;
                uint32_t cv1 = cvB, tab1 = tabB;
                cvB = 0;
                tabB = 0;
                if (e2 + (uint32_t)lane < rows) {
                    if (!a.eown_off) cvB = C[a.v_begin + r0 + e2 + lane];
                    if (a.taboo) tabB = a.taboo[r0 + e2 + lane];
                }
                if (a.eown_off && e0 + (uint32_t)lane < rows) cv = eown[e0 + lane];
                uint32_t acc[NW];
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    const uint32_t idx = (e0 + lane) * NW + i;
                    acc[i] = ((uint32_t)lane < cnt) ? smask[idx] : 0u;
                    if ((uint32_t)lane < cnt) smask[idx] = 0;
                }
                bool okv = (uint32_t)lane < cnt;
                if (split) {   // open rows wait in the tail queue (queue 0), with their masks
                    const bool open = okv && !is_full(acc);
                    const uint64_t om = __ballot(open);
                    if (om) {
                        uint32_t qb = 0;
                        if (lane == 0) qb = atomicAdd(&sh.qn[0], (uint32_t)__popcll(om));
                        if ((DG && a.scan_stats) && lane == 0) atomicAdd(&sh.st_qw, (uint32_t)__popcll(om));
                        qb = __shfl(qb, 0, 64);
                        if (open) {   // the entry carries what its evaluation needs: u_v's state, own colour, taboo
                            const uint32_t idx = qb + (uint32_t)__popcll(om & ((1ull << lane) - 1ull));
                            uint32_t* q = a.tq_l + ((size_t)blockIdx.x * 2u * a.tq_cap + idx) * 3u;
                            q[0] = r0 + e0 + lane;
                            q[1] = minstd_mulmod(xk, lpow);
                            q[2] = cv | (tab << 8);
#pragma unroll
                            for (int i = 0; i < NW; i++)
                                a.tq_m[((size_t)blockIdx.x * 2u * a.tq_cap + idx) * NW + i] = acc[i];
                        }
                    }
                    okv = okv && !open;
                }
                wave_viol += evaluate_lane<NW>(a, st, Cs, okv, r0 + e0 + lane, acc, lane, wave_ev, vf, cv, tab,
                                               minstd_mulmod(xk, lpow), ew);
                cv = cv1;
                tab = tab1;
                xk = minstd_mulmod(xk, xsk);
            }
            if (timing) { const uint64_t t1 = __builtin_readcyclecounter(); cyc_eval += t1 - tmark; tmark = t1; }
            if (ptrace && lane == 0) atomicMax(&sh.tr[kpair & 1u][2], (unsigned long long)wall_clock64());
        }
        // pair k+1's DMA landed everywhere (the evaluation's barrier waited for it); buffer k&1 and
        // the masks are free
        if (!REF && last) MCMC_LDS_BARRIER();
        else MCMC_PAIR_BARRIER();
        if (timing) { const uint64_t t1 = __builtin_readcyclecounter(); cyc_wait += t1 - tmark; }
        if (ptrace && threadIdx.x == 0 && kpair < kPairTraceMax) {
            unsigned long long* rec = a.pair_trace + ((size_t)blockIdx.x * kPairTraceMax + kpair) * kPairTraceRec;
            rec[0] = tr_start;
            rec[1] = sh.tr[kpair & 1u][0];
            rec[2] = sh.tr[kpair & 1u][1];
            rec[3] = sh.tr[kpair & 1u][2];
            rec[4] = wall_clock64();
            rec[6] = sh.tr[kpair & 1u][3];
            // info: block | open rows at the pair's top << 16 | drain, sparse, last, allfull << 40 | group << 44
            const uint32_t nopen = EXIT ? rows - min(nfull_run, rows) : rows;
            rec[5] = (unsigned long long)b | ((unsigned long long)nopen << 16) | ((unsigned long long)drain << 40) |
                     ((unsigned long long)sparse << 41) | ((unsigned long long)last << 42) |
                     ((unsigned long long)allfull << 43) | ((unsigned long long)g << 44);
        }
        if (REF && !RES && nbn == 0) gpar ^= 1u;   // the next pair starts a new group
        if (!REF && last) xg = minstd_mulmod(xg, xsg);
        g = ng;
        b = nbn;
        buf ^= 1u;
        kpair++;
        pstaged = nstaged;
    }
    if (TQ) tile_tail<NW, DG>(a, st, C, Cs, vf, lbase, SB, sh, fullw, x_t, lane, wave_viol, wave_ev, kpair, ew);
    if ((DG && a.scan_stats)) {   // diagnostics: quads loaded and pairs staged by this workgroup
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicAdd(&a.scan_stats[0], (unsigned long long)sh.st_quads);
            atomicAdd(&a.scan_stats[1], (unsigned long long)sh.st_pairs);
            atomicAdd(&a.scan_stats[2], (unsigned long long)sh.st_used);
            atomicAdd(&a.scan_stats[3], (unsigned long long)sh.st_slices);
            atomicAdd(&a.scan_stats[4], (unsigned long long)sh.st_qw);
            atomicAdd(&a.scan_stats[5], (unsigned long long)sh.st_qr);
        }
    }
    MCMC_PHASE(a, 3);
    if (timing && threadIdx.x == 0) {   // shader-clock cycles per phase kind, wave 0
        a.phase_ts[blockIdx.x * 8u + 5] = cyc_wait;
        a.phase_ts[blockIdx.x * 8u + 6] = cyc_scan;
        a.phase_ts[blockIdx.x * 8u + 7] = cyc_eval;
    }
    __syncthreads();   // the commit may reuse the colour-slice LDS for its sort
    if (REF) {
        // C_(t+1)'s histogram: this workgroup's counts; its same-colour arcs ride the arrival
        uint32_t* __restrict__ Hn = a.hist + ((t + 1u) & 1u) * a.hist_words;
        for (uint32_t c = threadIdx.x; c <= a.nCol; c += blockDim.x)
            if (hist_lds[c]) atomicAdd(&Hn[c], hist_lds[c]);
        uint32_t x = ecnt;
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        sweep_tail_ref(a, st, sh, (unsigned long long)x, lane);
    } else {
        sweep_tail(a, st, sh, wave_viol, wave_ev, lane, reinterpret_cast<uint32_t*>(lds_raw), a.lds_sort_cap, t, err0);
    }
    MCMC_PHASE(a, 4);
}

#include "dense_counts.h"
#include "dense_sparse.h"

// Layout construction lives in tiled_layout.hip.
__global__ void segment_kernel(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ col_idx,
                               uint32_t nloc, uint32_t nb, uint32_t block_log2, uint32_t* __restrict__ seg);

// Arc-balanced static partition of the local rows over W waves: wave w starts at the first row
// whose offset reaches w*m/W (lower bound), so every wave streams about m/W arcs.
__global__ void partition_kernel(const uint64_t* __restrict__ row_off, uint32_t nloc, uint32_t W,
                                 uint32_t* __restrict__ wave_start) {
    const uint64_t a0 = row_off[0], m = row_off[nloc] - a0;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= W; w += gridDim.x * blockDim.x) {
        if (w == W) { wave_start[w] = nloc; continue; }
        const uint64_t target = a0 + (m * w) / W;
        uint32_t lo = 0, hi = nloc;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (row_off[mid] < target) lo = mid + 1; else hi = mid;
        }
        wave_start[w] = lo;
    }
}

// ColoringMCMC_CPU ctor colouring (coloringMCMC_CPU.cpp:61): vertex v uses engine draw v + 1 when
// no earlier draw was rejected by uniform_int_distribution; rejections (P ~ nCol/2^31 each) are
// counted and handed to the exact sequential host path.
// REF initColoring (coloringMCMC_utils.cu:24-33): colour (int)(curand_uniform * nCol) -- nCol
// when u == 1.0f, as in the reference -- from each vertex's XORWOW state (advanced in place), and
// C_0's histogram.
__global__ void ref_init_kernel(uint8_t* __restrict__ C, uint32_t* __restrict__ X, uint32_t n, uint32_t nCol,
                                uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kHistWords];
    for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        xw::State s;
        for (int k = 0; k < xw::kWords; k++) s.v[k] = X[(size_t)k * n + v];
        s.d = X[(size_t)xw::kWords * n + v];
        const uint32_t c = (uint32_t)(int)(xw::uniform(xw::next(s)) * (float)nCol);
        C[v] = (uint8_t)c;
        for (int k = 0; k < xw::kWords; k++) X[(size_t)k * n + v] = s.v[k];
        X[(size_t)xw::kWords * n + v] = s.d;
        atomicAdd(&h[c], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i <= nCol; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ void init_coloring_kernel(uint8_t* C, uint32_t n, uint32_t x0, UniformIntConst k, DevState* st) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint32_t x = minstd_mulmod(x0, minstd_pow_tab((uint64_t)v + 1));
        const uint32_t r = x - 1u;
        if (r >= k.past) atomicAdd(&st->init_rejections, 1u);
        C[v] = (uint8_t)min(r / k.scaling, 255u);
    }
}

#include "sweep_wide.h"
#include "wide_tiled.h"
#include "wide_solo.h"
#include "ref_wide.h"

// ----------------------------------------------------------------------------------------------
using SweepLaunch = void (*)(const SweepArgs&, dim3, dim3, size_t, hipStream_t);
// wide sweep: grid = CUs (g.x); scan 8 x 256-thread workgroups per CU (a multiple of the 8 slabs),
// evaluation one workgroup per 2048 vertices, walk 8 per CU
void launch_wide(const SweepArgs& a, dim3 g, dim3, size_t, hipStream_t s) {
    if (a.inc) {   // incremental counts (a full sweep: zeroed here, recounted by the tile scan; an
                   // incremental one's flag pass runs in the tile scan's launch)
        wide_inc_delta_kernel<<<g.x, 1024, 0, s>>>(a);
    }
    if (a.xs_ent && a.xs_mode == 1) {
        if (!a.fp_live)
            wide_fp_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((a.n + 2047u) / 2048u, 4096u)), 256, 0, s>>>(a);
        wide_tscan_kernel<<<a.xs_nwg, kTscanThreads, kTscanLds, s>>>(a);
    }
    else if (a.xs_ent) wide_xscan_kernel<<<g.x * 8u, 256, 0, s>>>(a);
    else wide_scan_kernel<<<g.x * 8u, 256, 0, s>>>(a);
    if (a.dcap) wide_eval_kernel<true><<<a.evnblk + kWalkBlocks, 256, wide_walk_lds(a.nCol), s>>>(a);
    else wide_eval_kernel<false><<<a.evnblk + kWalkBlocks, 256, wide_walk_lds(a.nCol), s>>>(a);
}
// REF wide (ref_wide.h): grid = 8 blocks per CU (g.x = CUs) for the list kernels; masks of nCol bits
// per violator in LDS (at most 32 KiB per 256-thread block)
void launch_ref_wide(const SweepArgs& a, dim3 g, dim3, size_t, hipStream_t s) {
    const uint32_t wstride = (((a.nCol + 31u) >> 5) + 3u) & ~3u;
    refw_scan_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((a.n + 255u) / 256u, g.x * 16u)), 256, 0, s>>>(a);
    refw_rows_kernel<16><<<g.x * 8u, 256, 0, s>>>(a, kRwLong);
    refw_rows_kernel<1024><<<g.x, 1024, 0, s>>>(a, kRwHub);
    refw_walk_kernel<1><<<g.x * 8u, 64u * kRefwWalkWaves, sizeof(uint32_t) * kRefwWalkWaves * wstride, s>>>(a, kRwViol);
    refw_walk_kernel<16><<<g.x, 1024, sizeof(uint32_t) * wstride, s>>>(a, kRwViolBig);
}
template <int NW, bool LDSC>
void launch_sweep(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    sweep_kernel<NW, LDSC><<<g, b, lds, s>>>(a);
}
template <int NW>
void launch_blocked(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    sweep_blocked_kernel<NW><<<g, b, lds, s>>>(a);
}
template <int NW>
hipError_t allow_lds_blocked(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&sweep_blocked_kernel<NW>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
template <int NW, bool RES, bool REF = false, bool EX = false, bool DG = false>
void launch_tiled(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    sweep_tiled_kernel<NW, RES, REF, EX, DG><<<g, b, lds, s>>>(a);
}
template <int NW, bool RES, bool REF = false, bool EX = false, bool DG = false>
hipError_t allow_lds_tiled(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&sweep_tiled_kernel<NW, RES, REF, EX, DG>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
template <int NW, bool LDSC>
hipError_t allow_lds(size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&sweep_kernel<NW, LDSC>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
constexpr size_t kMaxLdsBytes = 160 * 1024 - 1024;   // leave room for the static shared variables

static std::once_flag g_const_once;
static hipError_t g_const_err = hipSuccess;

}  // namespace mcmc

using namespace mcmc;

struct mcmc_ctx {
    const GraphDev* g = nullptr;
    mcmc_params p{};
    uint32_t n = 0, v_begin = 0, v_end = 0;
    uint32_t nw = 1;
    uint32_t z = 0;
    uint8_t* colors[2] = {nullptr, nullptr};
    uint32_t* taboo = nullptr;
    uint32_t* events = nullptr;
    uint32_t* evdraw = nullptr;
    uint32_t ev_cap = 0;
    DevState* st = nullptr;
    unsigned long long* traj = nullptr;
    uint32_t traj_cap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipGraphExec_t batch_exec = nullptr;
    hipGraphExec_t batch_exec_ws = nullptr;   // the same batch through the persistent wide sweep
    hipGraphExec_t bench_exec = nullptr;   // mcmc_bench_prepare
    uint32_t bench_n = 0;
    bool borrowed_stream = false;
    uint32_t batch = 0;
    uint32_t batch_ws = 0;
    GlibcWindow glibc{};
    bool initialized = false;
    bool ran = false;
    uint32_t x0 = 0;            // minstd state after the initial colouring (position K0)
    uint64_t initDraws = 0;
    mcmc_run_stats last{};
    SweepLaunch sweep = nullptr;
    SweepLaunch sweep_diag = nullptr;   // tiled early exit (streaming): the diagnostics instantiation
    dim3 grid, block;
    size_t lds = 0;             // dynamic LDS of the sweep kernel (colour replica staging)
    uint32_t* wave_start = nullptr;
    uint32_t* seg = nullptr;    // blocked variant: segment offsets
    uint32_t nblocks = 0, block_log2 = 0, chunk_rows = 0;
    int variant = 0;            // 0 LDS-staged, 1 column-blocked, 2 L2-gather, 3 tiled
    const TiledLayout* tl = nullptr;   // variant 3 (owned by the graph's cache)
    uint32_t sub_log2 = 0, slice_bytes = 0;
    bool variant_res = false;          // variant 3: replica LDS-resident
    unsigned long long* phase_ts = nullptr;   // MCMC_PHASE_DUMP diagnostics
    unsigned long long* pair_trace = nullptr; // MCMC_PAIR_TRACE diagnostics (tiled sweep)
    int fused = 1;              // commit runs inside the sweep kernel (last workgroup)
    bool part = false;          // attached to a partitioned run (caller-owned buffers and stream)
    int bench_mode = 0;         // mcmc_set_bench_mode: no convergence stop (throughput timing)
    int early = 1;              // tiled: early-exit scan (MCMC_FULL_SCAN=1: every arc)
    int olist_on = 0;           // tiled early exit: R-entry open-row list in LDS (listed pairs)
    uint32_t tq_dense = 0, tq_cap = 0;       // tiled early exit: tail queue (dense blocks, entries per queue)
    uint32_t eown_off = 0;                   // tiled early exit: LDS offset of the evaluated group's own colours
    float2* ewalk = nullptr;                 // closed-form own-colour walk table (nullptr: the form is inexact)
    uint32_t ewalk_off = 0;                  // tiled: LDS offset of its copy
    uint32_t* tq_l = nullptr;                // [grid][2][tq_cap] rows
    uint32_t* tq_m = nullptr;                // [grid][2][tq_cap][nw] masks
    uint32_t drain_rows = 32;   // tiled early exit: drain threshold (MCMC_DRAIN_ROWS, 0 = off, <= 256; C3: 32 best)
    int late_stage = 0;         // tiled early exit: stage a group's next pair after the scan, if a row is open
    unsigned long long* scan_stats = nullptr;   // mcmc_set_scan_stats: [quads loaded, pairs staged]
    bool scan_stats_on = false;
    uint32_t world = 1, rank = 0;
    std::vector<uint32_t> bounds;            // partitioned: rank r sweeps rows [bounds[r], bounds[r+1])
    uint32_t* foot[2] = {nullptr, nullptr};  // partitioned: footer buffers, world x kFooterWords each
    uint32_t* dlt[2] = {nullptr, nullptr};   // native partitioned: delta slots, world x kDeltaWords each
    bool tail_done = false;                  // partitioned tail cut ran after the loop (multi.hip)
    uint64_t xs_delta = 0, xs_full = 0, xs_ovf = 0, xs_bytes = 0;   // mcmc_part_run's exchange statistics
    PartRes* pres = nullptr;                 // mcmc_part_run's stream, pinned word and events (part_resources)
    uint32_t tail_passes = 0;
    uint64_t tail_viol = 0;
    void* own_part = nullptr;                // native partitioned contexts: their own colour + footer buffers
    mcmc_comm* comm = nullptr;               // native partitioned contexts: the RCCL communicator (borrowed)
    uint32_t* spill = nullptr;               // native spill exchange: gathered lists, world x spill_stride
    uint32_t spill_stride = 0;
    uint8_t* own_colors[2] = {nullptr, nullptr};   // the context's own replicas (freed at destroy)
    std::vector<uint32_t> host_events;
    // tail cutting (mcmc_set_tailcut_repair, tailcut.hip)
    uint32_t tailcut_max = 0;   // pass cap; 0 = off
    uint8_t* vflags = nullptr;  // 2 x n violation flags kept by the sweeps
    uint32_t* tc_list = nullptr;
    uint32_t* tc_len = nullptr;
    uint32_t* tc_colorIdx = nullptr;
    unsigned long long* tc_count = nullptr;
    void* tc_tmp = nullptr;
    size_t tc_tmp_bytes = 0;
    std::vector<unsigned long long> tail_traj;   // Cviol (conflicting edges, REF) after each pass
    // reference-GPU-semantics mode (mcmc_ref_create)
    bool ref = false;
    mcmc_gpurand* rand = nullptr;   // caller-owned per-vertex XORWOW states
    uint32_t rand_base = 0;         // the states' parity when the run started
    uint32_t* hist = nullptr;       // [2][hist_words]
    uint32_t hist_words = kHistWords;
    bool refwide = false;           // REF with nCol > 255 (variant 5: uint16 replicas over the CSR, ref_wide.h)
    uint32_t* rw_cnt = nullptr;
    uint32_t* rw_lists = nullptr;
    float* ptab = nullptr;
    uint32_t own_buf_bytes = 0;
    // wide sweep (variant 4: nCol > 256, uint16 colour replicas; sweep_wide.h)
    bool wide = false;
    bool wide_tiled = false;        // variant 6: nCol > 256 over the tiled layout (wide_tiled.h)
    uint32_t* ws_buf = nullptr;     // the persistent wide sweep's lists and window (wide_solo.h)
    WsArgs wsa{};                   // (wsa.ctl != nullptr: set up)
    uint32_t* ws_dbg_host = nullptr; // MCMC_WS_DEBUG: the progress words (host memory, device-mapped)
    uint32_t ws_grid = 0;
    bool ws_on = false;             // launch_sweeps takes the persistent wide sweep
    bool bench_ws = false;          // ws_on when bench_exec was captured
    bool traj_ok = false;           // traj[t - 1] holds Cviol_{t-1} of the current chain (mcmc_run)
    long long ws_enter = 512;       // MCMC_WS_ENTER: largest Cviol a batch enters the persistent sweep
                                    // with (< 0: every batch, the colouring's first included)
    uint32_t cbytes = 1;            // bytes per colour in the replicas
    uint32_t* chunk_row = nullptr;
    uint32_t nchunks = 0;
    uint64_t arc_begin = 0, arc_count = 0;
    uint8_t* wflag = nullptr;
    uint8_t* wfp[2] = {nullptr, nullptr};   // wide LDS scan: fingerprints of colors[0/1], n (+2048) bytes
    uint32_t* wlist = nullptr;
    uint32_t* wcount = nullptr;
    uint32_t* gmask = nullptr;      // split walks: masks, then kSplitMax task counters
    uint32_t split_arcs = kSplitArcs;   // MCMC_SPLIT_ARCS (tests)
    uint32_t walk_light = kWalkLight;   // MCMC_WALK_LIGHT (0: every walk by a whole workgroup)
    uint32_t walk_tie = 1;              // MCMC_WALK_TIE: tie binades by word functions (r05 default: violator-heavy
                                        // C5 sweeps 0.265 -> 0.216 ms, converged unchanged; 0 = run by run)
    float* etab = nullptr;
    float emax = 0.0f;
    uint16_t* ftab = nullptr;       // F(u) table of the evaluation (ftab_n entries)
    uint32_t ftab_n = 0;
    uint32_t* evblk = nullptr;      // per evaluation workgroup event lists
    uint32_t* evcnt = nullptr;
    uint32_t evnblk = 0;
    uint32_t* evpow = nullptr;      // per evaluation wave: 16807^(first vertex + 1) (host-computed)
    uint32_t* gpow = nullptr;       // tiled: per (group, wave) the same (host-computed)
    uint32_t apow_grid = 0, apow_tile = 0;
    const XSlabLayout* xs = nullptr;   // wide: XCD-slab edge layout (graph-owned; nullptr: CSR arc scan)
    // wide: incremental violation counts (sweep_wide.h wide_inc_*; nullptr: the tile scan every sweep)
    uint32_t* inc = nullptr;        // kIncWords control words, then counts, lists and slots (make_args)
    unsigned long long inc_thresh = 0;
    uint32_t inc_slot = 0, inc_wslot_n = 0, inc_hub_arcs = 256;
    // dense-count sweep (dense_counts.h; MCMC_DENSE=0: the tiled scan sweep)
    bool dc = false;
    uint32_t* dc_ctl = nullptr;     // kDcWords control words, then the lists (one allocation)
    uint32_t* dc_cnt = nullptr;
    uint32_t* dc_mask = nullptr;
    unsigned long long* dc_open = nullptr;
    uint32_t dc_s0 = 0, dc_s1 = 0, dc_cap = 0, dc_max = 0, dc_apow = 1, dc_chg_cap = 0, dc_rbrows = 0;
    uint32_t dc_rbl = 0, dc_planes = 0;
    uint4* dc_tid = nullptr;        // the tile-transposed copy of S's ids (dc_build_tid) and its tile offsets
    uint64_t* dc_toff = nullptr;
    bool dc_fresh = false;          // the colouring is new: dc_prep runs the lane rebuild before its first sweep
    unsigned long long* dc_osum = nullptr;   // open summary (count + one bit per open word)
    // the persistent dense sweep (dense_sparse.h): its launch (nullptr: one dc_eval_kernel per sweep)
    // and the candidate window {L(w), w}
    void (*dcm_launch)(const SweepArgs&, uint32_t, dim3, hipStream_t) = nullptr;
    uint2* dl_tab = nullptr;
    uint32_t dl_n = 0;
    unsigned long long* solo_ts = nullptr;   // MCMC_SOLO_TRACE diagnostics (4096 x 8 stamps)
    unsigned long long* wt_tick = nullptr;   // wide tiled sweep's block rotation clock (wide_tiled.h)
    uint32_t* wt_buf = nullptr;     // its incremental counts: control words, vcnt, deg, lists (one allocation)
    uint64_t wt_arcs_max = 0;       // changed arcs up to which the next sweep stays incremental
    uint32_t wt_rc = 0;             // full sweeps as a block-major recount + the incremental kernels (its tables per round)
};

namespace {

// Incremental wide sweep: lists and statistics cleared, the next sweep a full recount (after any
// change of the colours that is not a sweep's).
hipError_t inc_reset(mcmc_ctx* c) {
    uint32_t h[kIncWords] = {};
    h[kIncMode] = 1u;
    hipError_t e = hipMemcpyAsync(c->inc, h, sizeof(h), hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;   // h lives on this frame
}

// Dense-count sweep: lists and statistics cleared, the next sweep's update a rebuild (after any
// change of the colours that is not a sweep's).
hipError_t dc_reset(mcmc_ctx* c) {
    uint32_t h[kDcWords] = {};
    h[kDcMode] = 1u;
    c->dc_fresh = true;
    hipError_t e = hipMemcpyAsync(c->dc_ctl, h, sizeof(h), hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;   // h lives on this frame
}

// The wide tiled sweep's incremental counts after the colouring changed: the next sweep scans (full).
hipError_t wt_reset(mcmc_ctx* c) {
    hipError_t e = hipMemsetAsync(c->wt_buf, 0, sizeof(uint32_t) * kWtWords, c->stream);
    return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}

// Host <-> device colour transfers (n colours in vertex order; partitioned replicas too).
int upload_colors(mcmc_ctx* c, uint8_t* dst, const uint8_t* h) {
    MCMC_HIP_TRY(hipMemcpyAsync(dst, h, (size_t)c->n * c->cbytes, hipMemcpyHostToDevice, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int download_colors(mcmc_ctx* c, const uint8_t* src, uint8_t* h) {
    MCMC_HIP_TRY(hipMemcpyAsync(h, src, (size_t)c->n * c->cbytes, hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int upload_state(mcmc_ctx* c, uint32_t t) {
    DevState h{};
    h.t = t;
    h.x_t = c->x0;
    h.lx = minstd_dlog(c->x0);
    h.glibc_head = 0;
    for (int i = 0; i < 31; i++) h.glibc_ring[i] = c->glibc.r[i];
    MCMC_HIP_TRY(hipMemcpyAsync(c->st, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int download_state(mcmc_ctx* c, DevState* h) {
    MCMC_HIP_TRY(hipMemcpyAsync(h, c->st, sizeof(*h), hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

SweepArgs make_args(const mcmc_ctx* c, int check_done) {
    SweepArgs a{};
    a.row_off = c->g->row_off ? c->g->row_off + c->v_begin : nullptr;
    a.row_off_g = c->g->row_off;
    a.col_idx = c->g->col_idx;
    a.colors0 = c->colors[0];
    a.colors1 = c->colors[1];
    a.taboo = c->taboo;
    a.events = c->events;
    a.evdraw = c->evdraw;
    a.st = c->st;
    a.traj = c->traj;
    a.traj_cap = c->traj_cap;
    a.ev_cap = c->ev_cap;
    a.n = c->n;
    a.v_begin = c->v_begin;
    a.v_end = c->v_end;
    a.nCol = c->p.nCol;
    // the tail queue's 24-bit counters (create_impl): a clamped copy, c->p keeps the caller's value
    a.tabooIteration = (c->tq_l && c->p.tabooIteration > kTabooMax24) ? c->p.maxRip + 2u : c->p.tabooIteration;
    a.maxRip = c->p.maxRip;
    a.z = c->z;
    a.aN = minstd_pow(kMinstdA, c->n);
    a.nmodN = c->n % kMinstdN;
    a.a256 = minstd_pow(kMinstdA, 256);
    a.eps = c->p.epsilon;
    a.hi = 1.0f - (float)(c->p.nCol - 1) * c->p.epsilon;   // fill_p :406, no contraction
    a.check_done = check_done;
    a.bench = c->bench_mode;
    a.early = c->early;
    a.olist_on = c->olist_on;
    a.tq_dense = c->tq_l ? c->tq_dense : 0u;
    a.tq_cap = c->tq_cap;
    a.tq_l = c->tq_l;
    a.tq_m = c->tq_m;
    a.eown_off = c->eown_off;
    a.ewalk = c->ewalk;
    a.ewalk_off = c->ewalk_off;
    a.drain_rows = c->drain_rows;
    a.late_stage = c->late_stage;
    a.scan_stats = c->scan_stats_on ? c->scan_stats : nullptr;
    a.fused = c->part ? 2 : (check_done ? c->fused : 0);
    a.seg = c->seg;
    a.nblocks = c->nblocks;
    a.block_log2 = c->block_log2;
    a.chunk_rows = c->chunk_rows;
    if (c->part) {
        a.foot0 = c->foot[0];
        a.foot1 = c->foot[1];
        a.rank = c->rank;
        if (c->dlt[0]) {
            a.dall0 = c->dlt[0];
            a.dall1 = c->dlt[1];
            a.dlt0 = c->dlt[0] + (size_t)c->rank * kDeltaWords;
            a.dlt1 = c->dlt[1] + (size_t)c->rank * kDeltaWords;
        }
    }
    a.world = c->world;
    a.lds_sort_cap = (uint32_t)(c->lds / 4);
    a.vflags = c->tailcut_max ? c->vflags : nullptr;
    if (c->ref) {
        a.vflags = nullptr;
        a.xw0 = c->rand->states[c->rand_base];
        a.xw1 = c->rand->states[c->rand_base ^ 1u];
        a.hist = c->hist;
        a.hist_words = c->hist_words;
        a.rw_cnt = c->rw_cnt;
        a.rw_lists = c->rw_lists;
        if (c->refwide) {
            a.etab = c->etab;
            a.ptab = c->ptab;
        }
        // nvcc contracts 1.0f - (nCol - 1) * eps into one fma (coloringMCMC_balance.cu:132)
        a.ref_hi = std::fma(-(float)(c->p.nCol - 1u), c->p.epsilon, 1.0f);
        a.own_buf_bytes = c->own_buf_bytes;
    }
    if (c->tl) {
        a.tcol = c->tl->tcol;
        a.gbase = c->tl->gbase;
        a.tseg = c->tl->tseg;
        a.grp_rows = c->tl->grp_rows;
        a.ngroups = c->tl->ngroups;
        a.nblocks = c->tl->nblocks;
        a.block_log2 = c->tl->block_log2;
        a.sub_log2 = c->sub_log2;
        a.slice_bytes = c->slice_bytes;
        a.seg_buf_bytes = (tseg_stride(c->tl->grp_rows) * 4u + 1023u) & ~1023u;
        a.gpow = c->gpow;
        a.apow_grid = c->apow_grid;
        a.apow_tile = c->apow_tile;
    }
    if (c->wide) {
        a.arc_begin = c->arc_begin;
        a.arc_count = c->arc_count;
        a.chunk_row = c->chunk_row;
        a.nchunks = c->nchunks;
        a.wflag = c->wflag;
        a.wfp0 = c->wfp[0];
        a.wfp1 = c->wfp[1];
        a.fp_live = (c->wfp[0] && !c->part) ? 1 : 0;   // partitioned: remote colours arrive by the exchange
        a.wlist = c->wlist;
        a.wcount = c->wcount;
        a.gmask = c->gmask;
        a.gdone = c->gmask ? c->gmask + (size_t)kSplitMax * kWideMaskWords : nullptr;
        a.split_arcs = c->split_arcs;
        a.walk_light = c->walk_light;
        a.walk_tie = c->walk_tie;
        a.etab = c->etab;
        a.emax = c->emax;
        a.ftab = c->ftab;
        a.ftab_n = c->ftab_n;
        a.evblk = c->evblk;
        a.evcnt = c->evcnt;
        a.evnblk = c->evnblk;
        a.evpow = c->evpow;
        a.fused = 0;
        if (c->xs) {
            a.xs_ent = c->xs->ent;
            a.xs_base = c->xs->base;
            a.xs_chunk0 = c->xs->chunk0;
            a.xs_pieces = c->xs->pieces;
            a.xs_wgp = c->xs->wg_piece;
            a.xs_mode = c->xs->mode;
            a.xs_nwg = c->xs->nwg;
            a.xs_S = c->xs->S;
            a.xs_cbits = c->xs->cbits;
            a.xs_sym = c->xs->sym;
        }
        if (c->inc) {   // (layout: inc_words)
            const size_t nloc = c->v_end - c->v_begin, L = c->n;
            a.inc = c->inc;
            a.inc_vcnt = c->inc + kIncWords;
            a.inc_hub = a.inc_vcnt + nloc;
            a.inc_tch = a.inc_hub + 2 * L;
            a.inc_eslot = a.inc_tch + 2 * nloc;
            a.inc_vslot = a.inc_eslot + 2 * (size_t)c->evnblk * (2 + c->inc_slot);
            a.inc_wslot = a.inc_vslot + 2 * (size_t)c->evnblk * (2 + c->inc_slot);
            a.inc_cchg = a.inc_wslot + 2 * (size_t)kIncWalkSlots * (2 + c->inc_wslot_n);
            a.inc_dense = a.inc_cchg + 2 * (2 + L);
            a.inc_hdr = a.inc_dense + 2 * L;
            a.inc_lcap = (uint32_t)L;
            a.inc_ccap = (uint32_t)L;
            a.inc_slot = c->inc_slot;
            a.inc_wslot_n = c->inc_wslot_n;
            a.inc_hub_arcs = c->inc_hub_arcs;
            a.inc_thresh = c->inc_thresh;
        }
    }
    if (c->wide_tiled) {
        a.wt_tick = c->wt_tick;
        if (c->wt_buf) {
            const size_t nloc = c->v_end - c->v_begin;
            a.wt_ctl = c->wt_buf;
            a.wt_vcnt = c->wt_buf + kWtWords;
            a.wt_deg = a.wt_vcnt + nloc;
            a.wt_list = a.wt_deg + nloc;
            a.wt_chg = reinterpret_cast<uint8_t*>(a.wt_list + 2u * nloc);
            a.wt_rc = c->wt_rc;
        }
        a.etab = c->etab;
        a.walk_tie = c->walk_tie;
        a.fused = 0;
    }
    if (c->dc) {
        a.dc_ctl = c->dc_ctl;
        a.dc_list = c->dc_ctl + kDcWords;
        a.dc_chg = a.dc_list + 4ull * c->dc_cap;
        a.dc_chg_cap = c->dc_chg_cap;
        a.dc_commit_restore = std::min<uint32_t>(kDcCommitRestore, c->dc_chg_cap / 2u);
        a.dc_open = c->dc_open;
        a.dc_cnt = c->dc_cnt;
        a.dc_mask = c->dc_mask;
        a.dc_s0 = c->dc_s0;
        a.dc_s1 = c->dc_s1;
        a.dc_cw = c->p.nCol;
        a.dc_cap = c->dc_cap;
        a.dc_max = c->dc_max;
        a.dc_apow = c->dc_apow;
        a.lds_sort_cap = kDcEvalLds / 4u;
        a.dc_osum = c->dc_osum;
        a.dc_rbrows = c->dc_rbrows;
        a.dc_rbl = c->dc_rbl;
        a.dc_poll = 1;
        if (const char* dp = getenv("MCMC_DC_POLL")) a.dc_poll = (uint32_t)std::max(1, atoi(dp));
        a.dc_planes = c->dc_planes;
        a.dc_tid = c->dc_tid;
        a.dc_toff = c->dc_toff;
        a.dl_tab = c->dl_tab;
        a.dl_n = c->dl_n;
        a.solo_ts = c->solo_ts;
    }
    a.phase_ts = c->phase_ts;
    a.pair_trace = c->pair_trace;
    a.tile = 32;  // vertices per wave-tile (evaluation batch)
    a.wave_start = c->wave_start;
    return a;
}

int ensure_constants() {
    std::call_once(g_const_once, [] {
        uint32_t pw[64], p2[64];
        pw[0] = 1;
        for (int j = 1; j < 64; j++) pw[j] = minstd_mulmod(pw[j - 1], kMinstdA);
        p2[0] = kMinstdA;
        for (int j = 1; j < 64; j++) p2[j] = minstd_mulmod(p2[j - 1], p2[j - 1]);
        g_const_err = hipMemcpyToSymbol(HIP_SYMBOL(kMinstdLanePow), pw, sizeof(pw));
        if (g_const_err == hipSuccess) g_const_err = hipMemcpyToSymbol(HIP_SYMBOL(kMinstdPow2), p2, sizeof(p2));
        // the glibc draw table: x^31 = x^28 + 1, then one multiplication by x per draw
        std::vector<uint32_t> tab((size_t)31 * kGlibcTabK);
        GlibcPoly q;
        for (int i = 0; i < 31; i++) q.c[i] = 0;
        q.c[0] = 1;
        q.c[28] = 1;
        for (uint32_t k = 0; k < kGlibcTabK; k++) {
            for (int i = 0; i < 31; i++) tab[(size_t)i * kGlibcTabK + k] = q.c[i];
            q = glibc_poly_mulx(q);
        }
        if (g_const_err == hipSuccess)
            g_const_err = hipMemcpyToSymbol(HIP_SYMBOL(kGlibcTab), tab.data(), sizeof(uint32_t) * tab.size());
    });
    if (g_const_err != hipSuccess) return fail(MCMC_E_HIP, std::string("constant upload: ") + hipGetErrorString(g_const_err));
    return MCMC_OK;
}

// The sweep launch for these arguments: the diagnostics instantiation when they ask for it.
void launch_tiled_or_diag(mcmc_ctx* c, const SweepArgs& a) {
    const bool diag = a.scan_stats || a.phase_ts || a.pair_trace;
    (diag && c->sweep_diag ? c->sweep_diag : c->sweep)(a, c->grid, c->block, c->lds, c->stream);
}

// Host launch of one (sweep, commit) pair on the context stream.
void launch_pair(mcmc_ctx* c, const SweepArgs& a) {
    launch_tiled_or_diag(c, a);
    if (a.fused) return;
    const uint32_t nloc = c->v_end - c->v_begin;
    const uint32_t lane_grid = std::max<uint32_t>(1u, std::min<uint32_t>((nloc + 255u) / 256u, 2048u));
    if (a.wt_ctl) {   // the incremental sweep's kernels (each returns at once in a full sweep)
        if (c->wt_rc) {   // (a full sweep's counts; each returns at once in an incremental one)
            const uint32_t nb = c->tl->nblocks, S = std::max<uint32_t>(1u, std::min<uint32_t>(c->tl->ngroups, (2048u + nb - 1u) / nb));
            wt_rc_zero_kernel<<<lane_grid, 256, 0, c->stream>>>(a);
            wt_recount_kernel<<<nb * S, 1024, wt_recount_lds(c->tl->block_log2, c->tl->grp_rows, c->wt_rc), c->stream>>>(a, S, c->wt_rc);
        }
        wt_eval_kernel<<<lane_grid, 256, 0, c->stream>>>(a);
        if (c->wt_tick) wt_viol_kernel<true><<<c->grid, c->block, c->lds, c->stream>>>(a);
        wt_viol_kernel<false><<<c->grid, c->block, c->lds, c->stream>>>(a);
    }
    if (c->refwide) refw_commit_kernel<<<1, 1024, 0, c->stream>>>(a);
    else if (c->wide || c->wide_tiled) commit_kernel<uint16_t, 1024><<<1, 1024, 0, c->stream>>>(a);
    else commit_kernel<uint8_t><<<1, kCommitThreads, 0, c->stream>>>(a);
    if (a.wt_ctl) {   // the counts of the next colouring
        wt_diff_kernel<<<lane_grid, 256, 0, c->stream>>>(a);
        wt_delta_kernel<<<c->grid.x, 512, 0, c->stream>>>(a, c->wt_arcs_max);
    }
}

// The host's message for DevState::err bits.
const char* dev_err_text(uint32_t err) {
    return (err & kDevErrWatchdog) ? "device watchdog: a phase of a persistent launch did not complete in 2 s "
                                     "(its workgroups were not all resident)"
                                   : "device flagged an overflow-event list overflow";
}

// The first sweep of a fresh colouring (dc_reset) rebuilds every count. Where the lane rebuild applies
// (nCol <= 32: setup_dense) it runs here as its own launches on the context stream, ahead of the
// sweep -- dc_rebuild_kernel (the copy into the other buffer + the counts) and dc_ctl_fresh_kernel
// (the update marked done) -- so the sweep's update has nothing left to do. Callers enqueue it inside
// their timed region, before the sweeps. Not while the stream is being captured (a graph replayed
// later must not carry it): the sweep's own update then rebuilds, as it does without the lane form.
int dc_prep(mcmc_ctx* c) {
    if (!c->dc || !c->dc_fresh || !c->dc_rbl) return MCMC_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    MCMC_HIP_TRY(hipStreamIsCapturing(c->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return MCMC_OK;
    c->dc_fresh = false;
    SweepArgs a = make_args(c, 1);
    const uint32_t nloc = c->v_end - c->v_begin;
    const uint32_t n1 = (nloc + kDcCopyRows - 1u) / kDcCopyRows;
    // a lane per row, 8 quads per lane in flight (measured at C3, 3 colourings each: 1024 x 8 6.53 ms,
    // 1024 x 10 6.5, 512 x 12 7.8, 512 x 16 8.7; the chunk rebuild inside the sweep 9.7;
    // gpurun_out/r06e, r06g)
    // over the tile-transposed ids (dc_build_tid): 512-thread workgroups with one 64 KiB slice each,
    // two per CU, so one counts while the other waits for its slice and quads (C3: 5.15 ms; 1024
    // threads and two slices 5.45; the layout read lane by lane 6.4; gpurun_out/r06v, r06w)
    if (c->dc_tid)
        dc_rebuild_kernel<1, 512, 8, true, 1><<<n1 + (nloc + 511u) / 512u, 512, kDcSliceBuf, c->stream>>>(a, n1);
    else
        dc_rebuild_kernel<1, 1024, 8, false, 2><<<n1 + (nloc + 1023u) / 1024u, 1024, kDcRebuildLds, c->stream>>>(a, n1);
    dc_ctl_fresh_kernel<<<1, 1, 0, c->stream>>>(c->dc_ctl);
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

// K sweeps on the context stream: one persistent dense launch (dc_multi_kernel) where the context
// has it (setup_dense_window; MCMC_DENSE_MULTI=0: never) and the arguments allow it (single context
// or a world-1 partition, committing in the sweep; no taboo, no tail-cut flags, no diagnostics); the
// persistent wide sweep (wide_solo.h) where set up and chosen (ws_choose); else K (sweep, commit) pairs.
// The persistent launch K sweeps of these arguments take, if any: 2 the wide one, 1 the dense one
int persistent_path(const mcmc_ctx* c, const SweepArgs& a) {
    const bool solo = !c->part || c->world == 1;   // nothing leaves the context
    const bool plain = solo && a.dcap == 0u && a.taboo == nullptr && a.vflags == nullptr && a.scan_stats == nullptr &&
                       a.phase_ts == nullptr && a.pair_trace == nullptr;
    if (c->wsa.ctl && c->ws_on && plain && a.inc != nullptr) return 2;
    if (c->dcm_launch && a.fused == 1 && plain) return 1;
    return 0;
}

void launch_sweeps(mcmc_ctx* c, const SweepArgs& a, uint32_t K) {
    const int pp = persistent_path(c, a);
    if (pp == 2) {
        if (K) ws_kernel<<<c->ws_grid, 1024, kWsLds, c->stream>>>(a, c->wsa, K);
        return;
    }
    if (pp == 1) {
        if (K) c->dcm_launch(a, K, c->grid, c->stream);
        return;
    }
    for (uint32_t i = 0; i < K; i++) launch_pair(c, a);
}

// The batch graph of the path c->ws_on selects (one cached graph per path: a run switches once,
// from the per-sweep path to the persistent sweep, when the violators have thinned out)
int build_batch_graph(mcmc_ctx* c, uint32_t batch) {
    hipGraphExec_t& ex = c->ws_on ? c->batch_exec_ws : c->batch_exec;
    uint32_t& key = c->ws_on ? c->batch_ws : c->batch;
    if (ex && key == batch) return MCMC_OK;
    if (ex) { (void)hipGraphExecDestroy(ex); ex = nullptr; }
    SweepArgs a = make_args(c, 1);
    hipGraph_t graph;
    MCMC_HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    launch_sweeps(c, a, batch);
    MCMC_HIP_TRY(hipStreamEndCapture(c->stream, &graph));
    hipError_t e = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    key = batch;
    return MCMC_OK;
}

void drop_graphs(mcmc_ctx* c) {
    if (c->batch_exec) (void)hipGraphExecDestroy(c->batch_exec);
    if (c->batch_exec_ws) (void)hipGraphExecDestroy(c->batch_exec_ws);
    if (c->bench_exec) (void)hipGraphExecDestroy(c->bench_exec);
    c->batch_exec = c->batch_exec_ws = c->bench_exec = nullptr;
    c->batch = c->batch_ws = c->bench_n = 0;
}

// Path choice for the next batch of a whole-graph run. The persistent wide sweep (wide_solo.h)
// rebuilds its violator lists and counts on entry and walks the violators on a few workgroups, so it
// beats the per-sweep path only near convergence (C5: 53 vs 66 us per converged sweep, but 2.1 vs
// 1.0 ms per sweep at nCol = maxDeg / 4 where every sweep has ~10^4 violators): it takes batches
// whose latest Cviol is at most ws_enter. last_viol < 0: unknown (a fresh colouring).
void ws_choose(mcmc_ctx* c, long long last_viol) {
    if (!c->wsa.ctl) { c->ws_on = false; return; }
    c->ws_on = c->ws_enter < 0 || (last_viol >= 0 && last_viol <= c->ws_enter);
}

// Cviol of the latest accepted colouring from the trajectory, -1 when it is not known
int last_cviol(mcmc_ctx* c, const DevState& h, long long* out) {
    *out = -1;
    if (!c->wsa.ctl || !c->traj_ok || h.t == 0 || h.t - 1u >= c->traj_cap) return MCMC_OK;
    unsigned long long v = 0;
    MCMC_HIP_TRY(hipMemcpy(&v, c->traj + (h.t - 1u), sizeof(v), hipMemcpyDeviceToHost));
    *out = (long long)v;
    return MCMC_OK;
}

int ensure_tail_buffers(mcmc_ctx* c) {
    if (c->vflags) return MCMC_OK;
    const size_t n = std::max<uint32_t>(c->n, 1u);
    MCMC_HIP_TRY(hipMalloc(&c->vflags, 2 * n));
    MCMC_HIP_TRY(hipMalloc(&c->tc_list, sizeof(uint32_t) * n));
    MCMC_HIP_TRY(hipMalloc(&c->tc_len, sizeof(uint32_t)));
    MCMC_HIP_TRY(hipMalloc(&c->tc_colorIdx, sizeof(uint32_t) * std::max<uint32_t>(c->p.nCol, 256u)));
    MCMC_HIP_TRY(hipMalloc(&c->tc_count, sizeof(unsigned long long)));
    MCMC_HIP_TRY(hipMemsetAsync(c->vflags, 0, 2 * n, c->stream));
    return MCMC_OK;
}

TailView tail_view(const mcmc_ctx* c) {
    TailView tv;
    tv.n = c->v_end - c->v_begin;   // a partitioned context's own rows
    tv.vb = c->v_begin;
    if (c->g->row_off) {
        tv.row_off = c->g->row_off;
        tv.col_idx = c->g->col_idx;
        tv.csr_row0 = c->v_begin;
    } else {
        tv.tcol = c->tl->tcol;
        tv.gbase = c->tl->gbase;
        tv.tseg = c->tl->tseg;
        tv.R = c->tl->grp_rows;
        tv.nb = c->tl->nblocks;
        tv.block_log2 = c->tl->block_log2;
    }
    return tv;
}

// The reference GPU colorer's tail cut (coloringMCMC_main.cu:271-290): orderedIndex by ascending
// histogram of the final colouring (std::sort with the reference's comparator), then while
// conflictCounter > 0 (at most c->tailcut_max passes; the reference loops until resolved):
// per-vertex edge counts (conflictCounter kernel), tailCutting over the first conflictCounter
// flagged vertices in order (own colour occupied -> first free colour of orderedIndex, the last
// one if none), recount. cc: the host's conflictCounter at loop exit.
int run_tailcut_ref(mcmc_ctx* c, const DevState& h, uint64_t cc, uint64_t* finalConf, uint32_t* passes) {
    const uint32_t n = c->n, nCol = c->p.nCol;
    uint8_t* C = c->colors[h.t & 1u];
    *passes = 0;
    *finalConf = h.finalViol;
    std::vector<uint8_t> hc((size_t)n * c->cbytes);
    int rc = download_colors(c, C, hc.data());
    if (rc) return rc;
    std::vector<uint32_t> stats(std::max(n, nCol) + 1u, 0u);
    for (uint32_t v = 0; v < n; v++) stats[c->cbytes == 2 ? reinterpret_cast<const uint16_t*>(hc.data())[v] : hc[v]]++;
    std::vector<uint32_t> ordered(nCol);
    for (uint32_t i = 0; i < nCol; i++) ordered[i] = i;
    std::sort(&ordered[0], &ordered[0] + nCol, [&](int i, int j) { return stats[i] < stats[j]; });
    MCMC_HIP_TRY(hipMemcpyAsync(c->tc_colorIdx, ordered.data(), sizeof(uint32_t) * nCol, hipMemcpyHostToDevice,
                                c->stream));
    const TailView tv = tail_view(c);
    rc = tail_count(tv, C, c->cbytes, c->vflags, c->tc_count, c->stream, true);
    if (rc) return rc;
    while (cc > 0 && *passes < c->tailcut_max) {
        rc = tail_select(c->vflags, n, c->tc_list, c->tc_len, &c->tc_tmp, &c->tc_tmp_bytes, c->stream);
        if (rc) return rc;
        rc = tail_repair(tv, C, c->cbytes, c->tc_list, c->tc_len, c->tc_colorIdx, nCol, c->stream, true, cc);
        if (rc) return rc;
        rc = tail_count(tv, C, c->cbytes, c->vflags, c->tc_count, c->stream, true);
        if (rc) return rc;
        unsigned long long hv = 0;
        MCMC_HIP_TRY(hipMemcpyAsync(&hv, c->tc_count, sizeof(hv), hipMemcpyDeviceToHost, c->stream));
        MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
        cc = hv;
        c->tail_traj.push_back(hv);
        (*passes)++;
        *finalConf = hv;
    }
    return MCMC_OK;
}

// Tail cutting after the loop (coloringMCMC_CPU.cpp:272-311, corrected: k++, at most
// c->tailcut_max passes; tailcut.hip). h: the device state at loop exit (done, no error).
int run_tailcut(mcmc_ctx* c, const DevState& h, uint64_t* finalViol, uint32_t* passes) {
    const uint32_t n = c->n, nCol = c->p.nCol;
    uint8_t* C = c->colors[h.t & 1u];
    *passes = 0;
    *finalViol = h.finalViol;
    // colorIdx: identity (:131-132), sorted by ascending colour histogram when z > 0 (:272-278);
    // std::sort with the reference's comparator, so ties resolve as the reference's do
    std::vector<size_t> colorIdx(nCol);
    for (uint32_t i = 0; i < nCol; i++) colorIdx[i] = i;
    if (c->z > 0) {
        std::vector<uint8_t> hc((size_t)n * c->cbytes);
        int rc = download_colors(c, C, hc.data());
        if (rc) return rc;
        std::vector<size_t> histBins(nCol, 0);
        for (uint32_t v = 0; v < n; v++)
            histBins[c->cbytes == 2 ? reinterpret_cast<const uint16_t*>(hc.data())[v] : hc[v]]++;
        std::sort(colorIdx.begin(), colorIdx.end(), [&](int i, int j) { return histBins[i] < histBins[j]; });
    }
    if (*finalViol == 0) return MCMC_OK;
    std::vector<uint32_t> ci(colorIdx.begin(), colorIdx.end());
    MCMC_HIP_TRY(hipMemcpyAsync(c->tc_colorIdx, ci.data(), sizeof(uint32_t) * nCol, hipMemcpyHostToDevice, c->stream));
    const TailView tv = tail_view(c);
    // first pass: the flags of the colouring before the last accepted sweep (run() never swaps
    // Cviols with Cstarviols, :259-260); sweep t kept those of C_t at parity t & 1
    const uint8_t* flags = c->vflags + (size_t)(h.t >= 1 ? (h.t - 1u) & 1u : 0u) * n;
    uint64_t cviol = *finalViol;
    while (cviol > 0 && *passes < c->tailcut_max) {
        int rc = tail_select(flags, n, c->tc_list, c->tc_len, &c->tc_tmp, &c->tc_tmp_bytes, c->stream);
        if (rc) return rc;
        rc = tail_repair(tv, C, c->cbytes, c->tc_list, c->tc_len, c->tc_colorIdx, nCol, c->stream, false, ~0ull);
        if (rc) return rc;
        rc = tail_count(tv, C, c->cbytes, c->vflags, c->tc_count, c->stream, false);   // :308
        if (rc) return rc;
        unsigned long long hv = 0;
        MCMC_HIP_TRY(hipMemcpyAsync(&hv, c->tc_count, sizeof(hv), hipMemcpyDeviceToHost, c->stream));
        MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
        cviol = hv;
        c->tail_traj.push_back(hv);
        flags = c->vflags;
        (*passes)++;
    }
    *finalViol = cviol;
    return MCMC_OK;
}

// Every arc of rows [vb, ve) into that range has its reverse and no row of it lists a neighbour
// twice: then, for u and w both in the range, w's row holds u exactly as often as u's row holds w
// (the dense counts' update reads u's row for the rows holding u; the wide sweep's partitioned
// incremental counts ask it of the whole graph). Generated G(n, p) graphs are so by construction.
int simple_symmetric(GraphDev& gd, uint32_t vb, uint32_t ve, hipStream_t stream, bool* ok) {
    const uint32_t nloc = ve - vb;
    const bool whole = vb == 0 && ve == gd.n;
    *ok = false;
    if (gd.simple_sym == 1 || (whole && gd.simple_sym == 0)) {
        *ok = gd.simple_sym == 1;
        return MCMC_OK;
    }
    if (!gd.row_off || !gd.sorted) return MCMC_OK;   // (tiled layouts of CSR graphs sort the rows)
    bool sym = false;
    if (int rc = csr_symmetric(gd, vb, nloc, stream, &sym)) return rc;
    if (sym && nloc) {
        uint32_t* bad = nullptr;
        uint32_t h = 0;
        MCMC_HIP_TRY(hipMalloc(&bad, sizeof(uint32_t)));
        hipError_t e = hipMemsetAsync(bad, 0, sizeof(uint32_t), stream);
        if (e == hipSuccess) {
            xs_dupcheck_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((nloc + 3u) / 4u, 65535u)), 256, 0, stream>>>(
                gd.row_off + vb, gd.col_idx, nloc, bad);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&h, bad, sizeof(uint32_t), hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        (void)hipFree(bad);
        if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("duplicate-arc check: ") + hipGetErrorString(e));
        sym = h == 0;
    }
    if (whole) gd.simple_sym = sym ? 1 : 0;
    *ok = sym;
    return MCMC_OK;
}

// The smallest minstd state x in [1, 2^31 - 1) with canonical(x) >= f (2^31 - 1 if none): the host
// twin of dense_counts.h dc_canonical_at_least (canonical is non-decreasing in x).
uint32_t host_canonical_at_least(float f) {
    uint32_t lo = 1u, hi = kMinstdM;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (minstd_canonical(mid) >= f) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}

constexpr uint32_t kDlMax = 1u << 16;   // candidate-window states of the persistent dense sweep

// The persistent dense sweep's pieces (dense_sparse.h): the open summary, and -- where the
// closed-form walk exists, no taboo, the context's ids below 2^31 - 2 and the window small -- the
// window's logarithm table. MCMC_DENSE_MULTI=0: neither (one dc_eval_kernel per sweep).
int setup_dense_window(mcmc_ctx* c) {
    const char* dm = getenv("MCMC_DENSE_MULTI");
    if (dm && atoi(dm) == 0) return MCMC_OK;
    const size_t nloc = c->v_end - c->v_begin;
    const size_t owords = (nloc + 63u) / 64u * c->nw;
    const size_t sbytes = sizeof(unsigned long long) * (1u + (owords + 63u) / 64u);
    MCMC_HIP_TRY(hipMalloc(&c->dc_osum, sbytes));
    MCMC_HIP_TRY(hipMemsetAsync(c->dc_osum, 0, sbytes, c->stream));
    if (!c->ewalk || c->p.tabooIteration != 0u || c->v_end > kMinstdN || c->part) return MCMC_OK;
    std::vector<float2> ew(c->p.nCol);
    MCMC_HIP_TRY(hipMemcpy(ew.data(), c->ewalk, sizeof(float2) * ew.size(), hipMemcpyDeviceToHost));
    uint32_t lo = 1u, hi = kMinstdM;   // the keep interval common to every colour: [lo, hi)
    for (const float2& e : ew) {
        lo = std::max(lo, host_canonical_at_least(e.x));
        hi = std::min(hi, host_canonical_at_least(e.y));
    }
    if (hi <= lo) return MCMC_OK;
    const uint64_t nwin = (uint64_t)(lo - 1u) + (uint64_t)(kMinstdM - hi);
    uint64_t dlmax = kDlMax;
    if (const char* e = getenv("MCMC_DL_MAX")) dlmax = strtoull(e, nullptr, 10);   // tests: larger windows
    if (nwin > dlmax) return MCMC_OK;   // (eps far above the reference's 1e-8: the per-sweep kernel)
    uint32_t* err = nullptr;
    MCMC_HIP_TRY(hipMalloc(&c->dl_tab, sizeof(uint2) * std::max<uint64_t>(nwin, 1)));
    MCMC_HIP_TRY(hipMalloc(&err, sizeof(uint32_t)));
    uint32_t herr = 0;
    hipError_t e = hipMemsetAsync(err, 0, sizeof(uint32_t), c->stream);
    if (e == hipSuccess && nwin) {
        dl_table_kernel<<<(uint32_t)((nwin + 255u) / 256u), 256, 0, c->stream>>>(c->dl_tab, lo, hi, (uint32_t)nwin, err);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&herr, err, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(err);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("dense window: ") + hipGetErrorString(e));
    if (herr) return fail(MCMC_E_DEVICE, "dense window: a discrete logarithm failed its check");
    c->dl_n = (uint32_t)nwin;
    if (getenv("MCMC_SOLO_TRACE")) {
        MCMC_HIP_TRY(hipMalloc(&c->solo_ts, sizeof(unsigned long long) * 8u * 4096u));
        MCMC_HIP_TRY(hipMemset(c->solo_ts, 0, sizeof(unsigned long long) * 8u * 4096u));
    }
    return MCMC_OK;
}

// The lane rebuild's coalesced input (dense_counts.h dc_tid_*): S's ids copied once per context,
// tile-transposed -- 64 consecutive rows, per S block Qt quads (the tile's longest segment) x 64
// lanes, so a wave's quad load reads 1 KiB contiguous instead of 64 scattered 16-byte pieces.
// Only where it fits with room to spare (MCMC_DC_TID=0: never; the rebuild then reads the layout).
hipError_t dc_build_tid(mcmc_ctx* c) {
    const char* env = getenv("MCMC_DC_TID");
    if (env && atoi(env) == 0) return hipSuccess;
    const uint32_t nloc = c->v_end - c->v_begin, ntiles = (nloc + 63u) / 64u;
    SweepArgs a = make_args(c, 1);
    uint64_t* tsz = nullptr;
    hipError_t e = hipMalloc(&tsz, sizeof(uint64_t) * ntiles);
    if (e != hipSuccess) { (void)hipGetLastError(); return hipSuccess; }
    const uint32_t blocks = (ntiles + 3u) / 4u;   // a wave per tile, 4 per workgroup
    dc_tid_size_kernel<<<blocks, 256, 0, c->stream>>>(a, tsz, ntiles);
    std::vector<uint64_t> h(ntiles);
    e = hipMemcpyAsync(h.data(), tsz, sizeof(uint64_t) * ntiles, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { (void)hipFree(tsz); return e; }
    uint64_t tot = 0;
    for (uint32_t t = 0; t < ntiles; t++) {
        const uint64_t q = h[t];
        h[t] = tot;
        tot += q;
    }
    size_t fr = 0, total = 0;
    const bool room = hipMemGetInfo(&fr, &total) == hipSuccess && tot * 16ull + (8ull << 30) < fr;
    (void)hipGetLastError();
    if (!room || tot == 0) { (void)hipFree(tsz); return hipSuccess; }
    e = hipMalloc(&c->dc_tid, tot * 16ull);
    if (e != hipSuccess) { (void)hipGetLastError(); c->dc_tid = nullptr; (void)hipFree(tsz); return hipSuccess; }
    e = hipMemcpyAsync(tsz, h.data(), sizeof(uint64_t) * ntiles, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    c->dc_toff = tsz;
    a = make_args(c, 1);
    dc_tid_fill_kernel<<<blocks, 256, 0, c->stream>>>(a, ntiles);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e;
}

// The dense-count sweep of a tiled context (dense_counts.h), when the graph allows it and
// MCMC_DENSE is not 0: S = the first |S| local rows, |S| such that a row's expected neighbours in
// S number nCol (ln nCol + K), K below (MCMC_DENSE_ROWS overrides |S|); counts, masks and lists allocated.
int setup_dense(mcmc_ctx* c, uint32_t nloc) {
    const char* de = getenv("MCMC_DENSE");
    if ((de && atoi(de) == 0) || nloc == 0 || c->p.nCol > 256 || !c->tl) return MCMC_OK;
    bool ok = false;
    if (int rc = simple_symmetric(const_cast<GraphDev&>(*c->g), c->v_begin, c->v_end, c->stream, &ok)) return rc;
    if (!ok) return MCMC_OK;
    const uint32_t nCol = c->p.nCol;
    const double dbar = (double)c->tl->arcs / (double)nloc;
    // K = ln(nloc) + 3: a row misses a colour in S with probability ~nloc^-1 e^-3, so the context
    // has an open row in ~5 % of its colourings. An open row costs every sweep a chain of dependent
    // loads (the scan of its other column blocks) and keeps the persistent sweep's leader from
    // running alone past kDcSoloOpenWords of them (dense_sparse.h); a unit of K costs the count
    // rebuild nloc nCol more counted arcs, once per colouring (C3: K 19.1, |S| ~ 7.2e5; r04 took
    // K = 10 there, 431 open rows in every sweep).
    double K = std::max(10.0, std::log((double)nloc) + 3.0);
    if (const char* dk = getenv("MCMC_DENSE_K")) K = atof(dk);
    const double target = (double)nCol * (std::log((double)nCol) + K);
    uint64_t S = dbar > 0.0 ? (uint64_t)std::ceil(target * (double)c->n / dbar) : nloc;
    if (const char* dr = getenv("MCMC_DENSE_ROWS")) S = (uint64_t)std::max(1, atoi(dr));
    S = std::max<uint64_t>(1, std::min<uint64_t>(S, nloc));
    const size_t cnt_bytes = (size_t)nloc * nCol * sizeof(uint32_t);
    if (cnt_bytes > (64ull << 30)) return MCMC_OK;   // counts beyond 64 GiB: the scan sweep
    // and only with room to spare on the device: the counts must not take the memory that later
    // allocations (tail queue, tail-cut buffers, the caller's tensors) need -- at most half of
    // what is free now, else the scan sweep
    {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && cnt_bytes > fr / 2) return MCMC_OK;
        (void)hipGetLastError();
    }
    c->dc_s0 = c->v_begin;
    c->dc_s1 = c->v_begin + (uint32_t)S;
    c->dc_cap = (uint32_t)S;
    c->dc_max = std::max<uint32_t>(64u, (uint32_t)(S / 8u));
    c->dc_apow = minstd_pow(kMinstdA, 64ull * c->grid.x * (c->block.x / 64u));
    c->dc_chg_cap = std::max<uint32_t>(4096u, nloc / 32u);   // past it: a full copy of the local rows
    // the streaming count rebuild (dense_counts.h dc_rebuild_chunk): chunks of rows whose uint16
    // count pairs and segment starts fill 64 KiB of LDS; its counts hold up to 65535 (every row
    // below that many arcs), else a wave per row (MCMC_DENSE_RB=0 too)
    {
        const uint32_t hw = (nCol + 1u) / 2u, R = c->tl->grp_rows;
        const uint32_t rc = std::min<uint32_t>(R, (kDcEvalLds / 4u - 1u) / (hw + 1u));
        const char* rb = getenv("MCMC_DENSE_RB");
        c->dc_rbrows = (c->g->maxDeg > 0 && c->g->maxDeg < 65536u && rc >= 1u && !(rb && atoi(rb) == 0)) ? rc : 0u;
        // the lane rebuild (dc_rebuild_lanes: a lane per row, its counts as bit planes in registers)
        // where one mask word holds every colour and the counts fit 16 planes; MCMC_DENSE_RB=1 keeps
        // the chunks, 0 a wave per row
        uint32_t planes = 4;
        while (planes < 16u && (c->g->maxDeg >> planes) != 0u) planes++;
        c->dc_planes = planes;
        c->dc_rbl = (nCol <= 32u && c->g->maxDeg < 65536u && c->dc_rbrows != 0u && !(rb && atoi(rb) == 1)) ? 1u : 0u;
        if (c->dc_rbl && (hipFuncSetAttribute(reinterpret_cast<const void*>(&dc_rebuild_kernel<1, 1024, 8, false, 2>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDcRebuildLds) != hipSuccess ||
                          hipFuncSetAttribute(reinterpret_cast<const void*>(&dc_rebuild_kernel<1, 512, 8, true, 1>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDcSliceBuf) != hipSuccess)) {
            (void)hipGetLastError();
            c->dc_rbl = 0u;
        }
    }
    if (const char* cc = getenv("MCMC_DENSE_CHG_CAP")) c->dc_chg_cap = (uint32_t)std::max(2, atoi(cc));   // tests
    const size_t open_bytes = sizeof(unsigned long long) * (((size_t)nloc + 63u) / 64u) * c->nw;
    hipError_t e = hipMalloc(&c->dc_ctl, sizeof(uint32_t) * (kDcWords + 4ull * S + 2ull * c->dc_chg_cap));
    if (e == hipSuccess) e = hipMalloc(&c->dc_cnt, std::max<size_t>(cnt_bytes, 4));
    if (e == hipSuccess) e = hipMalloc(&c->dc_mask, sizeof(uint32_t) * (size_t)nloc * c->nw);
    if (e == hipSuccess) e = hipMalloc(&c->dc_open, open_bytes);
    if (e == hipSuccess) e = hipMemsetAsync(c->dc_open, 0, open_bytes, c->stream);   // rows past nloc: never open
    if (e != hipSuccess) {
        (void)hipFree(c->dc_ctl);
        (void)hipFree(c->dc_cnt);
        (void)hipFree(c->dc_mask);
        (void)hipFree(c->dc_open);
        c->dc_ctl = c->dc_cnt = c->dc_mask = nullptr;
        c->dc_open = nullptr;
        if (e == hipErrorOutOfMemory) { (void)hipGetLastError(); return MCMC_OK; }   // the scan sweep then
        return fail(MCMC_E_HIP, std::string("dense counts: ") + hipGetErrorString(e));
    }
    c->dc = true;
    e = dc_reset(c);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("dense counts: ") + hipGetErrorString(e));
    if (c->dc_rbl) {
        e = dc_build_tid(c);
        if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("dense counts (transposed ids): ") + hipGetErrorString(e));
    }
    return setup_dense_window(c);
}

}  // namespace

extern "C" {

const char* mcmc_last_error(void) { return g_last_error.c_str(); }
int mcmc_version(void) { return 1; }

int mcmc_glibc_window(uint32_t seed, uint64_t draws, uint32_t window[31]) {
    if (!window) return fail(MCMC_E_ARG, "window is NULL");
    GlibcWindow w = glibc_srand(seed);
    if (draws) w = glibc_jump(w, draws);
    std::memcpy(window, w.r, sizeof(w.r));
    return MCMC_OK;
}

int mcmc_glibc_draw(uint32_t window[31], uint32_t count, uint32_t* out) {
    if (!window || (count && !out)) return fail(MCMC_E_ARG, "NULL argument");
    uint32_t ring[31];
    std::memcpy(ring, window, sizeof(ring));
    uint32_t head = 0;
    for (uint32_t i = 0; i < count; i++) out[i] = glibc_next(ring, head);
    for (int i = 0; i < 31; i++) window[i] = ring[(head + i) % 31];
    return MCMC_OK;
}

// ref != nullptr: a reference-GPU-semantics context (tiled REF sweep) over ref's XORWOW states.
// The persistent wide sweep (wide_solo.h) for a whole-graph context with incremental counts, eps > 0
// and no taboo: its lists, and the candidate window sorted by logarithm with a bucket index. The
// window is [1, w_lo) U [w_hi, 2^31 - 1): the states whose canonical draw is below E[nCol - 1] or
// at least hi (a case (iii) row keeps its colour exactly outside it). MCMC_WIDE_SOLO=0: off;
// MCMC_WS_MAX: window states allowed (default 2^24); MCMC_WS_LEAD_ARCS: changed arcs the leader
// moves itself; MCMC_WS_LIGHT: violator arcs walked on one wave; MCMC_WS_LEAD_HEAVY: heavy violators'
// arcs the leader walks itself (default 0: a walk phase); MCMC_WS_ENTER: largest Cviol a batch
// enters the persistent sweep with (ws_choose; < 0: always); MCMC_WS_POLL / MCMC_WS_DEBUG: the
// helpers' poll interval and the host-pinned per-wave progress words (diagnostics).
static uint32_t first_state_at_least(float thr) {
    uint32_t lo = 1, hi = kMinstdM;   // states 1 .. 2^31 - 2; hi = none
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (minstd_canonical(mid) >= thr) hi = mid; else lo = mid + 1u;
    }
    return lo;
}
// Whether `grid` workgroups of `kernel` (`block` threads, `lds` dynamic LDS bytes) can all be resident
// on the device at once -- the persistent launches' helpers spin on flags the leader posts, so a
// grid that cannot be co-resident must not take them. MCMC_PERSIST_CHECK_GRID (tests) checks that
// many workgroups instead of `grid`.
static bool coresident(const void* kernel, uint32_t grid, uint32_t block, size_t lds, int device) {
    if (const char* g = getenv("MCMC_PERSIST_CHECK_GRID")) grid = (uint32_t)strtoul(g, nullptr, 10);
    int per = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, (int)block, lds) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return (uint64_t)per * (uint64_t)cus >= grid;
}

// The persistent dense launch's workgroup size (MCMC_DCM_BS, 512 or 1024; default 512): at 512
// threads a wave may hold 256 VGPRs and dc_multi_kernel<1|2> runs without scratch (at 1024 the
// 128-VGPR cap spilled 256-544 B per lane, written once per wave and launch).
static uint32_t dcm_bs() {
    const char* e = getenv("MCMC_DCM_BS");
    return e && atoi(e) == 1024 ? 1024u : 512u;
}
extern "C++" {
template <uint32_t BS>
static hipError_t setup_dcm(mcmc_ctx* c, int wi) {
    static const decltype(c->dcm_launch) launch[4] = {launch_dcm<1, BS>, launch_dcm<2, BS>, launch_dcm<4, BS>,
                                                      launch_dcm<8, BS>};
    static hipError_t (*const allow[4])() = {allow_lds_dcm<1, BS>, allow_lds_dcm<2, BS>, allow_lds_dcm<4, BS>,
                                             allow_lds_dcm<8, BS>};
    const void* const fn[4] = {reinterpret_cast<const void*>(&dc_multi_kernel<1, BS>),
                               reinterpret_cast<const void*>(&dc_multi_kernel<2, BS>),
                               reinterpret_cast<const void*>(&dc_multi_kernel<4, BS>),
                               reinterpret_cast<const void*>(&dc_multi_kernel<8, BS>)};
    const hipError_t e = allow[wi]();
    if (e == hipSuccess && coresident(fn[wi], c->grid.x, BS, kDcMultiLds, c->g->device)) c->dcm_launch = launch[wi];
    return e;
}
}

static int setup_wide_solo(mcmc_ctx* c, uint32_t cus) {
    const char* e = getenv("MCMC_WIDE_SOLO");
    if ((e && atoi(e) == 0) || !c->inc || c->part || c->v_begin != 0 || c->v_end != c->n || c->p.tabooIteration > 0 ||
        !(c->p.epsilon > 0.0f) || !c->etab || c->p.nCol < 2)
        return MCMC_OK;
    // one minstd state per vertex and sweep (the window's runs assume it): n below the period
    if (c->n >= kMinstdN) return MCMC_OK;
    MCMC_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&ws_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)kWsLds));   // (before the occupancy query)
    if (!coresident(reinterpret_cast<const void*>(&ws_kernel), cus, 1024, kWsLds, c->g->device)) return MCMC_OK;
    const float hi = 1.0f - (float)(c->p.nCol - 1) * c->p.epsilon;
    if (!(c->emax < hi)) return MCMC_OK;
    const uint32_t wlo = first_state_at_least(c->emax), whi = first_state_at_least(hi);
    const uint64_t nw = (uint64_t)(wlo - 1u) + (uint64_t)(kMinstdM - whi);
    uint64_t wmax = 1ull << 24;
    if (const char* m = getenv("MCMC_WS_MAX")) wmax = strtoull(m, nullptr, 10);
    if (nw == 0 || nw > wmax) return MCMC_OK;
    if (const char* m = getenv("MCMC_WS_ENTER")) c->ws_enter = strtoll(m, nullptr, 10);
    const size_t nloc = c->v_end - c->v_begin;
    const size_t words = 4 + kWsWords + 2 * nloc + (nloc + 3) / 4 + 2 * nloc + 4 * nloc + (nloc + 1) + nloc + nloc + 3 * nloc +
                         2 * nw + (kWsNB + 1);
    size_t fr = 0, tot = 0;
    MCMC_HIP_TRY(hipMemGetInfo(&fr, &tot));
    if (4 * words + 16 * nw + (256ull << 20) > fr) return MCMC_OK;   // (the sort's scratch too)
    MCMC_HIP_TRY(hipMalloc(&c->ws_buf, 4 * words));
    uint32_t* b = c->ws_buf;
    WsArgs& w = c->wsa;
    w.ctl = b; b += kWsWords;
    w.vl = b; b += 2 * nloc;
    w.flag = b; b += (nloc + 3) / 4;
    w.res = b; b += 2 * nloc;
    b += (4u - ((b - c->ws_buf) & 3u)) & 3u;   // (16-byte entries)
    w.chg = b; b += 4 * nloc;
    w.pre = b; b += nloc + 1;
    w.tch = b; b += nloc;
    w.heavy = b; b += nloc;
    w.gcand = b; b += 3 * nloc;
    uint32_t* wL = b; b += nw;
    uint32_t* ww = b; b += nw;
    uint32_t* boff = b;
    w.wL = wL;
    w.ww = ww;
    w.boff = boff;
    w.nw = (uint32_t)nw;
    w.lead_arcs = 4096;
    if (const char* m = getenv("MCMC_WS_LEAD_ARCS")) w.lead_arcs = (uint32_t)strtoul(m, nullptr, 10);
    w.light_arcs = 512;   // (a wave gathers 512 arcs per round; a longer row: the workgroup, one round)
    if (const char* m = getenv("MCMC_WS_LIGHT")) w.light_arcs = std::max<uint32_t>(1u, (uint32_t)strtoul(m, nullptr, 10));
    w.lead_heavy = 0;   // (measured: a hub walk on the leader costs ~40 us, the walk phase overlaps it)
    if (const char* m = getenv("MCMC_WS_LEAD_HEAVY")) w.lead_heavy = (uint32_t)strtoul(m, nullptr, 10);
    w.sets = std::min<uint32_t>(16u, kWsLds / (4u * walk_set_words(c->p.nCol)));
    w.poll = 1;
    if (const char* m = getenv("MCMC_WS_POLL")) w.poll = (uint32_t)strtoul(m, nullptr, 10);
    w.poll_idle = 1;    // (as w.poll: a longer idle interval saves no memory traffic -- the polls are served
                        // on-die, FETCH_SIZE is the same -- and adds wake-up latency to every phase)
    if (const char* m = getenv("MCMC_WS_POLL_IDLE")) w.poll_idle = (uint32_t)strtoul(m, nullptr, 10);
    if (getenv("MCMC_WS_DEBUG")) {
        MCMC_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->ws_dbg_host), 4096 * sizeof(uint32_t),
                                   hipHostMallocMapped | hipHostMallocCoherent));
        memset(c->ws_dbg_host, 0, 4096 * sizeof(uint32_t));
        MCMC_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&w.dbg), c->ws_dbg_host, 0));
    }
    c->ws_grid = cus;
    // the window: (L, w) pairs, sorted by L, bucketed
    uint32_t *tk = nullptr, *tv = nullptr, *err = nullptr;
    void* tmp = nullptr;
    size_t tb = 0;
    hipError_t he = hipMalloc(&tk, sizeof(uint32_t) * nw);
    if (he == hipSuccess) he = hipMalloc(&tv, sizeof(uint32_t) * nw);
    if (he == hipSuccess) he = hipMalloc(&err, sizeof(uint32_t));
    if (he == hipSuccess) he = hipMemsetAsync(err, 0, sizeof(uint32_t), c->stream);
    if (he == hipSuccess) {
        ws_table_kernel<<<(uint32_t)((nw + 255) / 256), 256, 0, c->stream>>>(tk, tv, wlo, whi, (uint32_t)nw, err);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, tk, wL, tv, ww, (int)nw, 0, 31, c->stream);
    if (he == hipSuccess) he = hipMalloc(&tmp, std::max<size_t>(tb, 1));
    if (he == hipSuccess) he = hipcub::DeviceRadixSort::SortPairs(tmp, tb, tk, wL, tv, ww, (int)nw, 0, 31, c->stream);
    if (he == hipSuccess) {
        ws_bucket_kernel<<<(kWsNB + 1u + 255u) / 256u, 256, 0, c->stream>>>(wL, (uint32_t)nw, boff);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemsetAsync(w.ctl, 0, sizeof(uint32_t) * kWsWords, c->stream);
    uint32_t herr = 0;
    if (he == hipSuccess) he = hipMemcpyAsync(&herr, err, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(c->stream);
    (void)hipFree(tk);
    (void)hipFree(tv);
    (void)hipFree(err);
    (void)hipFree(tmp);
    if (he == hipSuccess) he = hipFuncSetAttribute(reinterpret_cast<const void*>(&ws_kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWsLds);
    if (he != hipSuccess) return fail(MCMC_E_HIP, std::string("persistent wide sweep setup: ") + hipGetErrorString(he));
    if (herr) return fail(MCMC_E_DEVICE, "persistent wide sweep: a window state's logarithm failed its check");
    return MCMC_OK;
}

static int create_impl(const mcmc_graph* g, const mcmc_params* p, uint32_t v_begin, uint32_t v_end,
                       mcmc_gpurand* ref, mcmc_ctx** out) {
    if (!g || !p || !out) return fail(MCMC_E_ARG, "NULL argument");
    *out = nullptr;
    const GraphDev& gd = g->g;
    if (p->nCol == 0) return fail(MCMC_E_ARG, "nCol must be >= 1");
    if (v_begin > v_end || v_end > gd.n) return fail(MCMC_E_ARG, "bad vertex range");
    // nCol > 256: the wide sweep (uint16 replicas, sweep_wide.h); MCMC_GATHER=wide forces it
    const char* gv = getenv("MCMC_GATHER");
    const std::string gsel = gv ? gv : "";
    // REF: a colour may equal nCol (initColoring at u = 1.0f), so uint8 replicas hold nCol <= 255
    const bool wide = ref ? p->nCol > 255 : (p->nCol > 256 || gsel == "wide" || gsel == "wide-tiled");
    // nCol > 256 on a generated graph (no CSR): its CSR is built from the tiled layout when it fits
    // beside it (the wide sweep's slabs and violator walks come from one); otherwise -- C3 at the
    // reference's default nCol = maxDeg, main.cu:162: 4.0e11 B of ids beside a 2.2e11 B layout --
    // the wide sweep over the tiled layout itself (wide_tiled.h). MCMC_GATHER=wide-tiled forces that
    // one, MCMC_GATHER=wide the CSR.
    bool wide_tiled = wide && !ref && gsel == "wide-tiled";
    if (wide) {
        if (p->nCol > kWideMaxCol) return fail(MCMC_E_ARG, "nCol > 65535 is not supported (uint16 colour replicas)");
        if (!gd.row_off && !wide_tiled) {
            int mr = mcmc_graph_materialize_csr(const_cast<mcmc_graph*>(g));
            if (mr == MCMC_E_NOMEM && !ref && gsel != "wide" && v_begin == 0 && v_end == gd.n) wide_tiled = true;
            else if (mr) return fail(mr, std::string("nCol > 256 on a generated graph: ") + mcmc_last_error());
        }
    }
    if (wide_tiled && (v_begin != 0 || v_end != gd.n))
        return fail(MCMC_E_ARG, "the wide tiled sweep: whole-graph contexts only (no partitions)");
    if (ref) {
        if (p->nCol < 2) return fail(MCMC_E_ARG, "reference-GPU mode: nCol >= 2");
        if (v_begin != 0 || v_end != gd.n) return fail(MCMC_E_ARG, "reference-GPU mode: whole-graph contexts");
        if (ref->n != gd.n || ref->device != gd.device)
            return fail(MCMC_E_ARG, "reference-GPU mode: the XORWOW states do not match the graph");
    }
    int rc = ensure_constants();
    if (rc) return rc;
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    mcmc_ctx* c = new mcmc_ctx();
    c->g = &gd;
    c->p = *p;
    c->n = gd.n;
    c->v_begin = v_begin;
    c->v_end = v_end;
    c->z = p->tailcut ? std::max<uint32_t>(50u, gd.n / 2000u) : 0u;   // :89-97
    // (REF: a colour equal to nCol sets no mask bit -- tile_gather_ref selects words by c >> 5)
    c->nw = p->nCol <= 32 ? 1 : p->nCol <= 64 ? 2 : p->nCol <= 128 ? 4 : 8;
    c->ref = ref != nullptr;
    c->rand = ref;
    if (const char* fs = getenv("MCMC_FULL_SCAN")) c->early = atoi(fs) ? 0 : 1;
    if (const char* dr = getenv("MCMC_DRAIN_ROWS")) c->drain_rows = std::min<uint32_t>(256u, (uint32_t)atoi(dr));
    if (ref) c->fused = 1;
    // The closed-form own-colour walk (evaluate_lane): E[c] = c-fold fp32 sum of eps, S[c] = fl(E[c] +
    // hi), exact when E never decreases and adding eps to every S[c] leaves it unchanged (standard
    // eps: S ~ 1, eps below half an ulp). Same fp32 operations as the device walk (-ffp-contract=off).
    if (!ref && !wide && p->nCol >= 1 && p->nCol <= 256 && !getenv("MCMC_NO_EWALK")) {
        const float eps = p->epsilon, hi = 1.0f - (float)(p->nCol - 1) * eps;
        std::vector<float2> tab(p->nCol);
        bool ok = eps >= 0.0f;
        float E = 0.0f;
        for (uint32_t k = 0; k < p->nCol && ok; k++) {
            const float S = E + hi;
            ok = (S + eps) == S;
            tab[k] = make_float2(E, S);
            const float En = E + eps;
            ok = ok && En >= E;
            E = En;
        }
        if (ok) {
            hipError_t ee = hipMalloc(&c->ewalk, sizeof(float2) * p->nCol);
            if (ee == hipSuccess) ee = hipMemcpy(c->ewalk, tab.data(), sizeof(float2) * p->nCol, hipMemcpyHostToDevice);
            if (ee != hipSuccess) { (void)hipFree(c->ewalk); c->ewalk = nullptr; }
        }
    }
    // Variant: the tiled layout (16-bit block-local ids, replica LDS-resident when it fits, else
    // streamed 64 KiB slices) -- fastest on every measured shape. The CSR variants stay selectable
    // for A/B runs and parity tests. Knobs: MCMC_GATHER=tiled|lds|blocked|global, MCMC_BLOCK_LOG2,
    // MCMC_SUB_LOG2, MCMC_GROUP_ROWS, MCMC_TILE_STREAM.
    const size_t lds_bytes = (((size_t)gd.n + 15) / 16) * 16;
    c->variant = (gsel == "global") ? 2 : (gsel == "blocked") ? 1 : (gsel == "lds") ? 0 : 3;
    if (c->variant == 0 && lds_bytes > kMaxLdsBytes) c->variant = 3;
    if (!gd.row_off || ref) c->variant = 3;   // generated graph / REF: tiled layout only
    if (wide_tiled) {   // the wide sweep over the tiled layout (wide_tiled.h)
        c->variant = 6;
        c->wide_tiled = true;
        c->cbytes = 2;
        c->fused = 0;
        c->sweep = launch_wide_tiled;
    } else if (wide && ref) {   // REF over the CSR with uint16 replicas (ref_wide.h)
        c->variant = 5;
        c->refwide = true;
        c->cbytes = 2;
        c->fused = 0;
        c->sweep = launch_ref_wide;
        c->hist_words = (p->nCol + 1u + 63u) & ~63u;
    } else if (wide) {
        c->variant = 4;
        c->wide = true;
        c->cbytes = 2;
        c->fused = 0;
        c->sweep = launch_wide;
    }
    const int wi = c->nw == 1 ? 0 : c->nw == 2 ? 1 : c->nw == 4 ? 2 : 3;
    hipError_t ea = hipSuccess;
    if (c->variant == 0) {
        static const SweepLaunch tab[4] = {launch_sweep<1, true>, launch_sweep<2, true>, launch_sweep<4, true>,
                                           launch_sweep<8, true>};
        c->sweep = tab[wi];
        c->lds = lds_bytes;
        ea = wi == 0 ? allow_lds<1, true>(lds_bytes) : wi == 1 ? allow_lds<2, true>(lds_bytes)
           : wi == 2 ? allow_lds<4, true>(lds_bytes) : allow_lds<8, true>(lds_bytes);
    } else if (c->variant == 1) {
        static const SweepLaunch tab[4] = {launch_blocked<1>, launch_blocked<2>, launch_blocked<4>, launch_blocked<8>};
        c->sweep = tab[wi];
        const char* bl = getenv("MCMC_BLOCK_LOG2");
        c->block_log2 = bl ? (uint32_t)std::max(6, std::min((int)kBlockLog2Max, atoi(bl))) : kBlockLog2Max;
        c->nblocks = (uint32_t)((((uint64_t)gd.n + 15) / 16 * 16 + (1ull << c->block_log2) - 1) >> c->block_log2);
        c->chunk_rows = 4096u / c->nw;
        c->lds = (size_t)(1u << c->block_log2) + (size_t)c->chunk_rows * c->nw * 4u;
        ea = wi == 0 ? allow_lds_blocked<1>(c->lds) : wi == 1 ? allow_lds_blocked<2>(c->lds)
           : wi == 2 ? allow_lds_blocked<4>(c->lds) : allow_lds_blocked<8>(c->lds);
    } else if (c->variant == 4 || c->variant == 5 || c->variant == 6) {
        // geometry and tables below
    } else if (c->variant == 3) {
        const char* bl = getenv("MCMC_BLOCK_LOG2");
        c->block_log2 = (bl && gd.row_off) ? (uint32_t)std::max(4, std::min(16, atoi(bl))) : 16u;
    } else {
        static const SweepLaunch tab[4] = {launch_sweep<1, false>, launch_sweep<2, false>, launch_sweep<4, false>,
                                           launch_sweep<8, false>};
        c->sweep = tab[wi];
    }
    if (ea != hipSuccess) {
        mcmc_destroy(c);
        return fail(MCMC_E_HIP, std::string("hipFuncSetAttribute(LDS): ") + hipGetErrorString(ea));
    }
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, gd.device);
    c->glibc = glibc_srand(1);
    const uint32_t nloc = v_end - v_begin;
    c->ev_cap = std::max<uint32_t>(nloc, 64u * 1024u);   // local events; also >= 64 ranks x footer events
    c->traj_cap = (uint32_t)std::min<uint64_t>((uint64_t)p->maxRip + 2, kTrajCapMax);
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
    chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    chk(hipEventCreate(&c->ev0));
    chk(hipEventCreate(&c->ev1));
    // colour replicas carry 256 B of slack so equal-size partition slabs can be all-gathered in place
    chk(hipMalloc(&c->colors[0], ((size_t)gd.n + 256) * c->cbytes));
    chk(hipMalloc(&c->colors[1], ((size_t)gd.n + 256) * c->cbytes));
    c->own_colors[0] = c->colors[0];
    c->own_colors[1] = c->colors[1];
    if (p->tabooIteration > 0) chk(hipMalloc(&c->taboo, sizeof(uint32_t) * std::max<uint32_t>(nloc, 1)));
    // event list sized n (+ pow2 padding room for the in-place sort fallback)
    uint32_t pcap = 1;
    while (pcap < c->ev_cap) pcap <<= 1;
    chk(hipMalloc(&c->events, sizeof(uint32_t) * pcap));
    chk(hipMalloc(&c->evdraw, sizeof(uint32_t) * pcap));
    chk(hipMalloc(&c->st, sizeof(DevState)));
    chk(hipMalloc(&c->traj, sizeof(unsigned long long) * c->traj_cap));
    if (getenv("MCMC_PAIR_TRACE")) {
        const size_t words = (size_t)kPairTraceRec * kPairTraceMax * 4096u;
        chk(hipMalloc(&c->pair_trace, sizeof(unsigned long long) * words));
        chk(hipMemsetAsync(c->pair_trace, 0, sizeof(unsigned long long) * words, c->stream));
    }
    if (getenv("MCMC_PHASE_DUMP")) {
        chk(hipMalloc(&c->phase_ts, sizeof(unsigned long long) * kPhaseWords));
        chk(hipMemsetAsync(c->phase_ts, 0, sizeof(unsigned long long) * kPhaseWords, c->stream));
    }
    if (e != hipSuccess) {
        mcmc_destroy(c);
        return fail(MCMC_E_NOMEM, std::string("allocation: ") + hipGetErrorString(e));
    }
    if (c->taboo) (void)hipMemsetAsync(c->taboo, 0, sizeof(uint32_t) * nloc, c->stream);
    // persistent grids; rows statically arc-balanced over all waves (blocked: over workgroups)
    if (c->variant == 3) {
        // Resident (replica + two segment-table buffers + masks fit one workgroup's LDS): replica
        // staged once. Otherwise (streaming) two 64 KiB colour-slice buffers. One 1024-thread
        // workgroup per CU either way. Groups of R rows: about one group per workgroup, at most
        // what the LDS holds (rmax) and kTileRowsMax.
        const size_t rep = lds_bytes;
        const char* gr = getenv("MCMC_GROUP_ROWS");
        // REF adds [p: 1 KiB][histogram][2 own-colour buffers of own_bytes(rows) (streaming)]
        auto own_bytes = [](uint32_t rows) -> size_t { return ((size_t)rows + 47u + 1023u) & ~(size_t)1023u; };
        auto lds_need = [&](bool res, uint32_t rows) -> size_t {
            const size_t segb = ((size_t)tseg_stride(rows) * 4u + 1023u) & ~(size_t)1023u;
            const size_t base = (res ? rep : 2u * (size_t)tile_slice_buf(c->block_log2)) + 2u * segb;
            if (!ref) return base + (size_t)rows * c->nw * 4u;
            return base + (((size_t)rows * c->nw * 4u + 15u) & ~(size_t)15u) + 1024u + 4u * kHistWords +
                   (res ? 0u : 2u * own_bytes(rows));
        };
        auto rmax_for = [&](bool res) -> uint32_t {
            uint32_t r = kTileRowsMax;
            while (r > 1 && lds_need(res, r) > kMaxLdsBytes) r -= 1;
            return lds_need(res, r) <= kMaxLdsBytes ? r : 0u;
        };
        // Streaming is the default: with the slices double-buffered by LDS-DMA it measured faster
        // than the resident replica even where the replica fits (C2: 44.3 vs 45.4 us).
        // MCMC_TILE_STREAM=0 selects the resident replica when it fits.
        const char* ts_env = getenv("MCMC_TILE_STREAM");
        const bool want_resident = ts_env && atoi(ts_env) == 0;
        const uint32_t rmax_res = rep <= 10u * 16u * 1024u ? rmax_for(true) : 0u;
        const bool resident = want_resident && rmax_res >= 64u;
        if (!resident) c->block_log2 = std::min<uint32_t>(c->block_log2, 16u);
        c->block = dim3(1024);
        c->grid = dim3((uint32_t)cus);
        c->slice_bytes = resident ? (uint32_t)rep : (uint32_t)std::min<size_t>(1ull << c->block_log2, rep);
        const uint32_t rmax = resident ? rmax_res : rmax_for(false);
        if (rmax == 0) {
            mcmc_destroy(c);
            return fail(MCMC_E_ARG, "tiled sweep: no group size fits the LDS for this nCol");
        }
        uint32_t R = tiled_default_rows(nloc, c->grid.x, rmax);
        if (gr) R = (uint32_t)std::max(1, std::min((int)rmax, atoi(gr)));
        c->variant_res = resident;
        int rs = get_tiled_layout(const_cast<mcmc_graph*>(g), v_begin, v_end, R, c->block_log2, c->stream, &c->tl);
        if (rs) { mcmc_destroy(c); return rs; }
        R = c->tl->grp_rows;   // a generated graph's layout brings its own group size
        if (!ref && c->block.x == 1024) {   // u_v's skip-ahead per (group, wave) and per step, once
            std::vector<uint32_t> pw((size_t)c->tl->ngroups * 16u);
            for (size_t i = 0; i < pw.size(); i++)
                pw[i] = minstd_pow(kMinstdA, (uint64_t)v_begin + (uint64_t)(i / 16) * R + 64ull * (i % 16) + 1ull);
            c->apow_grid = minstd_pow(kMinstdA, (uint64_t)c->grid.x * R);
            c->apow_tile = minstd_pow(kMinstdA, 64ull * 16ull);
            hipError_t ep = pw.empty() ? hipSuccess : hipMalloc(&c->gpow, sizeof(uint32_t) * pw.size());
            if (ep == hipSuccess && !pw.empty())
                ep = hipMemcpy(c->gpow, pw.data(), sizeof(uint32_t) * pw.size(), hipMemcpyHostToDevice);
            if (ep != hipSuccess) {
                mcmc_destroy(c);
                return fail(MCMC_E_HIP, std::string("group powers: ") + hipGetErrorString(ep));
            }
        }
        if (R > rmax) {
            mcmc_destroy(c);
            return fail(MCMC_E_ARG, "generated layout's group rows exceed this nCol's LDS budget (streaming: nCol > 64)");
        }
        c->nblocks = c->tl->nblocks;
        // lanes per row segment: the smallest power of two L >= 4 with L * kTileU quads per step
        // covering half a mean segment (measured on C2 / n = 8e5: fewer lanes make the
        // finish/reduce path run nearly every step; more leave lanes idle)
        const double arcs = (double)c->tl->ids;
        const double quads = arcs / 8.0 / std::max(1.0, (double)nloc * c->nblocks);
        uint32_t sl = 2;
        while (sl < 6 && 2.0 * (double)(1u << sl) * kTileU < quads) sl++;
        if (c->early && !ref) {
            // early exit: a row scans about min(its segment, the ids that fill its mask -- the coupon
            // collector's nCol H(nCol)) per block; the smallest L whose step covers that, so a segment
            // takes one step (the scan is instruction-issue bound: SQ_ACTIVE_INST_ANY ~ 1 issue per
            // SIMD cycle, every masked slot costs its wave instruction; measured r02: C3 L = 2 / 4 / 8
            // 1.345 / 1.257 / 1.671 ms, C2 L = 1 / 2 / 4 23.6 / 23.8 / 25.5 us)
            double hn = 0.0;
            for (uint32_t k = 1; k <= p->nCol; k++) hn += 1.0 / k;
            const double scan_ids = std::min(8.0 * quads, (double)p->nCol * hn);
            sl = 0;
            while (sl < 6 && 8.0 * (double)(1u << sl) * kTileU < scan_ids) sl++;
            // late staging where a mean segment leaves a row open with probability < 1%
            // (nCol (1 - 1/nCol)^d, d ids): C2's 500-id segments fill 16 colours inside block 0, so its
            // block-1 pair (slice, table, first quads) was staged for nothing; C3 (65 of ~130 ids) keeps
            // staging ahead. A wrong guess costs one exposed DMA round trip, never a result.
            c->late_stage = 8.0 * quads >= (double)p->nCol * std::log(100.0 * p->nCol) ? 1 : 0;
            if (const char* ls = getenv("MCMC_LATE_STAGE")) c->late_stage = atoi(ls) ? 1 : 0;
        }
        const char* sv = getenv("MCMC_SUB_LOG2");
        if (sv) sl = (uint32_t)std::max(0, std::min(6, atoi(sv)));
        c->sub_log2 = sl;
        c->lds = lds_need(resident, R);
        if (!ref && c->early && !getenv("MCMC_NO_OLIST")) {   // the open-row list of listed pairs, if it fits
            const size_t lb = ((size_t)R * 2u + 15u) & ~(size_t)15u;
            if (c->lds + lb <= kMaxLdsBytes) {
                c->lds += lb;
                c->olist_on = 1;
            }
        }
        // the closed-form own-colour walk's table (evaluate_lane), LDS copy
        if (!ref && c->ewalk && c->lds + ((8u * (size_t)p->nCol + 15u) & ~(size_t)15u) <= kMaxLdsBytes) {
            c->ewalk_off = (uint32_t)c->lds;
            c->lds += (8u * (size_t)p->nCol + 15u) & ~(size_t)15u;
        }
        // the evaluated group's own colours, LDS-DMA'd at its last pair's top (early exit, streaming)
        if (!ref && c->early && !resident) {
            const size_t ob = own_bytes(R);
            if (c->lds + ob <= kMaxLdsBytes) {
                c->eown_off = (uint32_t)c->lds;
                c->lds += ob;
            }
        }
        // the dense-count sweep (dense_counts.h) where it applies; MCMC_DENSE=0 keeps the scan
        if (!ref && c->early) {
            int rd = setup_dense(c, nloc);
            if (rd) { mcmc_destroy(c); return rd; }
        }
        // the tail queue (streaming early exit with more blocks than the dense ones): every
        // workgroup's queues hold all rows of its groups
        const char* tqe = getenv("MCMC_TQ_DENSE");
        const uint32_t tqd = tqe ? (uint32_t)std::max(0, atoi(tqe)) : 2u;
        if (!ref && c->early && !c->dc && !resident && tqd > 0 && tqd < c->nblocks && c->tl->ngroups > 0) {
            const uint32_t gpw = (c->tl->ngroups + c->grid.x - 1) / c->grid.x;
            c->tq_cap = gpw * R;
            const size_t ents = (size_t)c->grid.x * 2u * c->tq_cap;
            hipError_t qe = hipMalloc(&c->tq_l, sizeof(uint32_t) * 3u * ents);
            if (qe == hipSuccess) qe = hipMalloc(&c->tq_m, sizeof(uint32_t) * ents * c->nw);
            if (qe != hipSuccess) {
                mcmc_destroy(c);
                return fail(MCMC_E_NOMEM, std::string("tail queue: ") + hipGetErrorString(qe));
            }
            c->tq_dense = tqd;
            // The tail queue packs a row's taboo counter in 24 bits (own colour | counter << 8). A
            // counter past the loop's last sweep never expires within the loop, so the sweeps of
            // such a context see a larger tabooIteration as maxRip + 2 (make_args; c->p keeps the
            // caller's value); with a loop that long it is refused.
            if (p->tabooIteration > kTabooMax24 && (uint64_t)p->maxRip + 2u > kTabooMax24) {
                mcmc_destroy(c);
                return fail(MCMC_E_ARG, "tabooIteration >= 2^24 needs maxRip + 2 < 2^24 (24-bit taboo counters "
                                        "of the tail queue)");
            }
        }
        c->own_buf_bytes = resident ? 0u : (uint32_t)own_bytes(R);
        if (ref) {
            if (resident) {
                static const SweepLaunch tab[4] = {launch_tiled<1, true, true>, launch_tiled<2, true, true>,
                                                   launch_tiled<4, true, true>, launch_tiled<8, true, true>};
                c->sweep = tab[wi];
                ea = wi == 0 ? allow_lds_tiled<1, true, true>(c->lds) : wi == 1 ? allow_lds_tiled<2, true, true>(c->lds)
                   : wi == 2 ? allow_lds_tiled<4, true, true>(c->lds) : allow_lds_tiled<8, true, true>(c->lds);
            } else {
                static const SweepLaunch tab[4] = {launch_tiled<1, false, true>, launch_tiled<2, false, true>,
                                                   launch_tiled<4, false, true>, launch_tiled<8, false, true>};
                c->sweep = tab[wi];
                ea = wi == 0 ? allow_lds_tiled<1, false, true>(c->lds) : wi == 1 ? allow_lds_tiled<2, false, true>(c->lds)
                   : wi == 2 ? allow_lds_tiled<4, false, true>(c->lds) : allow_lds_tiled<8, false, true>(c->lds);
            }
        } else if (c->dc) {   // the dense-count sweep (update + evaluation launches)
            static const SweepLaunch tab[4] = {launch_dc<1>, launch_dc<2>, launch_dc<4>, launch_dc<8>};
            c->sweep = tab[wi];
            c->sweep_diag = nullptr;
            c->lds = kDcRebuildLds;
            ea = wi == 0 ? allow_lds_dc<1>(c->lds) : wi == 1 ? allow_lds_dc<2>(c->lds)
               : wi == 2 ? allow_lds_dc<4>(c->lds) : allow_lds_dc<8>(c->lds);
            // the persistent launch (dense_sparse.h), where sweeps can run solo and the grid can be
            // co-resident (else one dc_eval_kernel per sweep); its LDS allowance first: the
            // occupancy query needs it
            if (ea == hipSuccess && c->dc_osum && c->dl_n)
                ea = dcm_bs() == 1024u ? setup_dcm<1024>(c, wi) : setup_dcm<512>(c, wi);
        } else if (c->early) {   // the early-exit instantiations
            if (resident) {
                static const SweepLaunch tab[4] = {launch_tiled<1, true, false, true>, launch_tiled<2, true, false, true>,
                                                   launch_tiled<4, true, false, true>, launch_tiled<8, true, false, true>};
                c->sweep = tab[wi];
                ea = wi == 0 ? allow_lds_tiled<1, true, false, true>(c->lds) : wi == 1 ? allow_lds_tiled<2, true, false, true>(c->lds)
                   : wi == 2 ? allow_lds_tiled<4, true, false, true>(c->lds) : allow_lds_tiled<8, true, false, true>(c->lds);
            } else {
                static const SweepLaunch tab[4] = {launch_tiled<1, false, false, true>, launch_tiled<2, false, false, true>,
                                                   launch_tiled<4, false, false, true>, launch_tiled<8, false, false, true>};
                c->sweep = tab[wi];
                ea = wi == 0 ? allow_lds_tiled<1, false, false, true>(c->lds) : wi == 1 ? allow_lds_tiled<2, false, false, true>(c->lds)
                   : wi == 2 ? allow_lds_tiled<4, false, false, true>(c->lds) : allow_lds_tiled<8, false, false, true>(c->lds);
                static const SweepLaunch tabd[4] = {launch_tiled<1, false, false, true, true>,
                                                    launch_tiled<2, false, false, true, true>,
                                                    launch_tiled<4, false, false, true, true>,
                                                    launch_tiled<8, false, false, true, true>};
                c->sweep_diag = tabd[wi];
                if (ea == hipSuccess)
                    ea = wi == 0 ? allow_lds_tiled<1, false, false, true, true>(c->lds)
                       : wi == 1 ? allow_lds_tiled<2, false, false, true, true>(c->lds)
                       : wi == 2 ? allow_lds_tiled<4, false, false, true, true>(c->lds)
                                 : allow_lds_tiled<8, false, false, true, true>(c->lds);
            }
        } else if (resident) {
            static const SweepLaunch tab[4] = {launch_tiled<1, true>, launch_tiled<2, true>, launch_tiled<4, true>,
                                               launch_tiled<8, true>};
            c->sweep = tab[wi];
            ea = wi == 0 ? allow_lds_tiled<1, true>(c->lds) : wi == 1 ? allow_lds_tiled<2, true>(c->lds)
               : wi == 2 ? allow_lds_tiled<4, true>(c->lds) : allow_lds_tiled<8, true>(c->lds);
        } else {
            static const SweepLaunch tab[4] = {launch_tiled<1, false>, launch_tiled<2, false>, launch_tiled<4, false>,
                                               launch_tiled<8, false>};
            c->sweep = tab[wi];
            ea = wi == 0 ? allow_lds_tiled<1, false>(c->lds) : wi == 1 ? allow_lds_tiled<2, false>(c->lds)
               : wi == 2 ? allow_lds_tiled<4, false>(c->lds) : allow_lds_tiled<8, false>(c->lds);
        }
        if (ea != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("hipFuncSetAttribute(LDS): ") + hipGetErrorString(ea));
        }
    } else if (c->variant == 6) {
        // one wave per row over the tiled layout (64 KiB column blocks; a CSR graph's layout is built
        // here with 1024-row groups, a generated graph's comes with it)
        c->block_log2 = 16;
        const char* gr = getenv("MCMC_GROUP_ROWS");
        const uint32_t R = gr ? (uint32_t)std::max(1, std::min((int)kTileRowsMax, atoi(gr))) : 1024u;
        int rs = get_tiled_layout(const_cast<mcmc_graph*>(g), v_begin, v_end, R, c->block_log2, c->stream, &c->tl);
        if (rs) { mcmc_destroy(c); return rs; }
        c->nblocks = c->tl->nblocks;
        const uint32_t W = wide_tiled_waves(p->nCol), NWW = (p->nCol + 31u) >> 5;
        c->block = dim3(64u * W);
        c->grid = dim3((uint32_t)cus * wide_tiled_wgs_per_cu(p->nCol));
        c->lds = (size_t)W * (2u * NWW + 1u) * 4u;
        if (const char* e = getenv("MCMC_WALK_TIE")) c->walk_tie = (uint32_t)strtoul(e, nullptr, 10);
        std::vector<float> et((size_t)p->nCol + 1);
        eps_table(p->epsilon, p->nCol, et.data());
        hipError_t ew = hipFuncSetAttribute((const void*)wide_tiled_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)c->lds);
        if (ew == hipSuccess)
            ew = hipFuncSetAttribute((const void*)wt_viol_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds);
        if (ew == hipSuccess)
            ew = hipFuncSetAttribute((const void*)wt_viol_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds);
        if (ew == hipSuccess) ew = hipMalloc(&c->etab, sizeof(float) * et.size());
        if (ew == hipSuccess) ew = hipMemcpy(c->etab, et.data(), sizeof(float) * et.size(), hipMemcpyHostToDevice);
        const char* rot = getenv("MCMC_WT_ROTATE");   // 0: every row scans blocks 0, 1, ... (A/B runs)
        if (ew == hipSuccess && !(rot && atoi(rot) == 0)) {
            ew = hipMalloc(&c->wt_tick, sizeof(unsigned long long));
            if (ew == hipSuccess) ew = hipMemset(c->wt_tick, 0, sizeof(unsigned long long));
        }
        // incremental violation counts (wide_tiled.h; MCMC_WT_INC: 0 off -- every sweep scans --, 2 every
        // sweep after the first incremental): 16 B per row
        const char* wi = getenv("MCMC_WT_INC");
        const int wmode = wi ? atoi(wi) : 1;
        if (ew == hipSuccess && wmode != 0) {
            const size_t nloc = v_end - v_begin;
            ew = hipMalloc(&c->wt_buf, sizeof(uint32_t) * (kWtWords + 4 * (size_t)nloc + nloc / 32u + 2u));
            if (ew == hipSuccess) ew = hipMemset(c->wt_buf, 0, sizeof(uint32_t) * kWtWords);
            // full sweeps as recount + incremental kernels where a block's colours and a row group's
            // table fit the LDS (MCMC_WT_RC=0: the mask scan of wide_tiled_kernel)
            const char* rce = getenv("MCMC_WT_RC");
            const uint32_t rck = wt_rc_k(c->tl->block_log2, c->tl->grp_rows);
            c->wt_rc = (!(rce && atoi(rce) == 0) && rck > 0 &&
                        hipFuncSetAttribute(reinterpret_cast<const void*>(&wt_recount_kernel),
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)wt_recount_lds(c->tl->block_log2, c->tl->grp_rows, rck)) == hipSuccess) ? rck : 0u;
            (void)hipGetLastError();
            // A changed arc costs one colour gather (two where its other end changed too: rare); a
            // full sweep's counts cost a mask-scan gather per arc, or (recount) a streamed 2-byte id
            // per arc and a few LDS operations -- measured at C3 1/8 .. 1/32 of an arc gather in the
            // delta -- and the next sweep's violators are walked over their whole rows either way:
            // incremental while the changed rows' arcs are at most 1/2 (mask scan) or 1/32 (recount)
            // of the layout's (MCMC_WT_ARCS_DIV: the divisor, measurement)
            const char* wd = getenv("MCMC_WT_ARCS_DIV");
            const uint64_t div = wd ? std::max<uint64_t>(1, strtoull(wd, nullptr, 10)) : (c->wt_rc ? 32u : 2u);
            c->wt_arcs_max = wmode == 2 ? ~0ull : c->tl->arcs / div;
        }
        if (ew != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("wide tiled sweep setup: ") + hipGetErrorString(ew));
        }
    } else if (c->variant == 4) {
        c->grid = dim3((uint32_t)cus);   // launch_wide scales it per kernel
        c->block = dim3(256);
        uint64_t ends[2];
        hipError_t ew = hipMemcpy(&ends[0], gd.row_off + v_begin, sizeof(uint64_t), hipMemcpyDeviceToHost);
        if (ew == hipSuccess) ew = hipMemcpy(&ends[1], gd.row_off + v_end, sizeof(uint64_t), hipMemcpyDeviceToHost);
        c->arc_begin = ends[0];
        c->arc_count = ends[1] - ends[0];
        c->nchunks = (uint32_t)((c->arc_count + kWideChunk - 1) / kWideChunk);
        if (ew == hipSuccess) ew = hipMalloc(&c->chunk_row, sizeof(uint32_t) * ((size_t)c->nchunks + 1));
        if (ew == hipSuccess) ew = hipMalloc(&c->wflag, (nloc + 4u) & ~(size_t)3);   // word atomics (flag_violator)
        if (ew == hipSuccess) ew = hipMalloc(&c->wlist, 2 * sizeof(uint32_t) * std::max<size_t>(nloc, 1));
        if (ew == hipSuccess) ew = hipMalloc(&c->wcount, 4 * sizeof(uint32_t));
        const size_t gmb = sizeof(uint32_t) * ((size_t)kSplitMax * kWideMaskWords + 3 * kSplitMax);
        if (ew == hipSuccess) ew = hipMalloc(&c->gmask, gmb);
        if (ew == hipSuccess) ew = hipMemsetAsync(c->gmask, 0, gmb, c->stream);
        if (const char* e = getenv("MCMC_SPLIT_ARCS")) c->split_arcs = std::max<uint32_t>(1u, (uint32_t)strtoul(e, nullptr, 10));
        if (const char* e = getenv("MCMC_WALK_LIGHT")) c->walk_light = (uint32_t)strtoul(e, nullptr, 10);
        if (const char* e = getenv("MCMC_WALK_TIE")) c->walk_tie = (uint32_t)strtoul(e, nullptr, 10);
        std::vector<float> et((size_t)p->nCol + 1);
        eps_table(p->epsilon, p->nCol, et.data());
        c->emax = et[p->nCol - 1];
        // F(u_i) for u_i = i 2^-31 < emax (both monotone: one merge), when emax < hi and the table
        // stays below 2^22 entries (8 MiB)
        std::vector<uint16_t> ft;
        const float hi = 1.0f - (float)(p->nCol - 1) * p->epsilon;
        if (p->epsilon > 0.0f && c->emax < hi && (double)c->emax * 2147483648.0 < 4194304.0) {
            uint32_t k = 1;
            for (uint32_t i = 0;; i++) {
                const float u = (float)i * 0x1p-31f;
                if (!(u < c->emax)) break;
                while (!(et[k] > u)) k++;   // k <= nCol - 1 since E[nCol-1] > u
                ft.push_back((uint16_t)k);
            }
        }
        c->ftab_n = (uint32_t)ft.size();
        if (ew == hipSuccess && !ft.empty()) ew = hipMalloc(&c->ftab, sizeof(uint16_t) * ft.size());
        if (ew == hipSuccess && !ft.empty())
            ew = hipMemcpy(c->ftab, ft.data(), sizeof(uint16_t) * ft.size(), hipMemcpyHostToDevice);
        if (ew == hipSuccess) ew = hipMalloc(&c->etab, sizeof(float) * et.size());
        if (ew == hipSuccess) ew = hipMemcpy(c->etab, et.data(), sizeof(float) * et.size(), hipMemcpyHostToDevice);
        c->evnblk = std::max<uint32_t>(1u, (nloc + 256u * kWideEvalPer - 1u) / (256u * kWideEvalPer));
        if (ew == hipSuccess) ew = hipMalloc(&c->evblk, sizeof(uint32_t) * kEvSlot * c->evnblk);
        if (ew == hipSuccess) ew = hipMalloc(&c->evcnt, sizeof(uint32_t) * c->evnblk);
        if (ew == hipSuccess) ew = hipMemsetAsync(c->evcnt, 0, sizeof(uint32_t) * c->evnblk, c->stream);
        {   // u_v's skip-ahead to each evaluation wave's first vertex, once (a per-lane chain of ~22
            // table loads and mulmods in the kernel otherwise)
            std::vector<uint32_t> pw((size_t)c->evnblk * 4);
            for (size_t i = 0; i < pw.size(); i++)
                pw[i] = minstd_pow(kMinstdA, (uint64_t)v_begin + 256ull * kWideEvalPer * (i / 4) + 64ull * (i % 4) + 1ull);
            if (ew == hipSuccess) ew = hipMalloc(&c->evpow, sizeof(uint32_t) * pw.size());
            if (ew == hipSuccess)
                ew = hipMemcpy(c->evpow, pw.data(), sizeof(uint32_t) * pw.size(), hipMemcpyHostToDevice);
        }
        if (ew == hipSuccess) ew = hipMemsetAsync(c->wflag, 0, (nloc + 4u) & ~(size_t)3, c->stream);
        if (ew == hipSuccess) ew = hipMemsetAsync(c->wcount, 0, 4 * sizeof(uint32_t), c->stream);
        if (ew == hipSuccess) {
            const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((c->nchunks + 256) / 256, 4096u));
            wide_chunk_row_kernel<<<blocks, 256, 0, c->stream>>>(gd.row_off + v_begin, nloc, c->arc_begin,
                                                                 c->arc_count, c->nchunks, c->chunk_row);
            ew = hipStreamSynchronize(c->stream);
        }
        // the violation scan: MCMC_WIDE_SCAN = lds (default: LDS-staged colour tiles) | l2 (8 XCD
        // slabs through L2) | csr (the CSR arc scan; A/B runs, tests)
        const char* wsv = getenv("MCMC_WIDE_SCAN");
        const std::string wsel = wsv ? wsv : "lds";
        if (ew == hipSuccess && wsel != "csr") {
            int rx = get_xslab(const_cast<mcmc_graph*>(g), v_begin, v_end, wsel == "l2" ? 0u : 1u,
                                     (uint32_t)cus, c->stream, &c->xs);
            if (!rx && !c->xs && wsel != "l2")   // row deltas beyond the LDS tiles' field: the L2 slabs
                rx = get_xslab(const_cast<mcmc_graph*>(g), v_begin, v_end, 0u, (uint32_t)cus, c->stream, &c->xs);
            if (rx) {
                mcmc_destroy(c);
                return rx;
            }
            if (c->xs && c->xs->mode == 1) {
                for (int q = 0; q < 2 && ew == hipSuccess; q++) {   // slack: tile staging and row windows
                    ew = hipMalloc(&c->wfp[q], (size_t)gd.n + 2048);
                    if (ew == hipSuccess) ew = hipMemsetAsync(c->wfp[q], 0, (size_t)gd.n + 2048, c->stream);
                }
            }
        }
        // incremental violation counts: a whole-graph context over a symmetric CSR without repeated
        // arcs, with the LDS tile scan for its full sweeps. MCMC_WIDE_INC = 0 off, 2 every sweep after
        // a full one incremental (tests); MCMC_WIDE_INC_DIV: full recount above m / DIV changed arcs
        // MCMC_WIDE_INC_SLOT: changed rows per evaluation slot (walk slots: half), past which the
        // next sweep recounts (2 on, the tests: slots hold every row, no arc limit)
        const char* wie = getenv("MCMC_WIDE_INC");
        const int winc = wie ? atoi(wie) : 1;
        // A row range (a rank of a partitioned run) keeps them too when the graph holds every row's
        // arcs and is simple and symmetric as a whole: other ranks' changed vertices move this rank's
        // counts through their own rows (sweep_wide.h wide_inc_delta_kernel).
        bool inc_ok = ew == hipSuccess && winc != 0 && c->xs && c->xs->mode == 1 && c->xs->simple;
        if (inc_ok && !(v_begin == 0 && v_end == gd.n)) {
            bool whole_ss = false;
            if (!gd.partial_rows) {
                int rs = simple_symmetric(const_cast<GraphDev&>(gd), 0, gd.n, c->stream, &whole_ss);
                if (rs) { mcmc_destroy(c); return rs; }
            }
            inc_ok = whole_ss;
        }
        if (inc_ok) {
            const char* sv = getenv("MCMC_WIDE_INC_SLOT");
            c->inc_slot = winc == 2 ? 256u * kWideEvalPer : std::max<uint32_t>(1u, sv ? (uint32_t)atoi(sv) : 32u);
            c->inc_wslot_n = winc == 2 ? std::min<uint32_t>(nloc, 1u << 16) : std::max<uint32_t>(1u, c->inc_slot / 2u);
            // layout (make_args): counts [nloc], hub lists [2][n], touched [2][nloc], the evaluation's
            // and walks' slots, the commit's slots [2][2 + n], dense lists [2][n], slot headers
            const size_t L = gd.n;
            const size_t words = kIncWords + 3 * (size_t)nloc + 2 * L + 4 * (size_t)c->evnblk * (2 + c->inc_slot) +
                                 2 * (size_t)kIncWalkSlots * (2 + c->inc_wslot_n) + 2 * (2 + L) +
                                 2 * L + 4 * ((size_t)c->evnblk + kIncWalkSlots);
            ew = hipMalloc(&c->inc, sizeof(uint32_t) * words);
            if (ew == hipSuccess) ew = hipMemsetAsync(c->inc, 0, sizeof(uint32_t) * words, c->stream);
            const char* dv = getenv("MCMC_WIDE_INC_DIV");
            const uint64_t div = dv ? std::max<uint64_t>(1, strtoull(dv, nullptr, 10)) : 32;
            c->inc_thresh = winc == 2 ? ~0ull : c->arc_count / div;
            if (const char* hv = getenv("MCMC_WIDE_INC_HUB")) c->inc_hub_arcs = (uint32_t)atoi(hv);
        }
        if (ew != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("wide sweep setup: ") + hipGetErrorString(ew));
        }
        if (int rw = setup_wide_solo(c, (uint32_t)cus)) {
            mcmc_destroy(c);
            return rw;
        }
    } else if (c->variant == 5) {
        c->grid = dim3((uint32_t)cus);   // launch_ref_wide scales it per kernel
        c->block = dim3(256);
        hipError_t ew = hipMalloc(&c->rw_cnt, 4 * sizeof(uint32_t));
        if (ew == hipSuccess) ew = hipMalloc(&c->rw_lists, 4 * sizeof(uint32_t) * std::max<size_t>(nloc, 1));
        if (ew == hipSuccess) ew = hipMemsetAsync(c->rw_cnt, 0, 4 * sizeof(uint32_t), c->stream);
        std::vector<float> et((size_t)p->nCol + 1);   // E[k] = k eps in fp32 (refw_walk_own)
        eps_table(p->epsilon, p->nCol, et.data());
        if (ew == hipSuccess) ew = hipMalloc(&c->etab, sizeof(float) * et.size());
        if (ew == hipSuccess) ew = hipMemcpy(c->etab, et.data(), sizeof(float) * et.size(), hipMemcpyHostToDevice);
        if (ew == hipSuccess) ew = hipMalloc(&c->ptab, sizeof(float) * p->nCol);
        if (ew == hipSuccess) ew = hipStreamSynchronize(c->stream);
        if (ew != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("reference-GPU wide setup: ") + hipGetErrorString(ew));
        }
    } else if (c->variant != 2) {
        c->block = dim3(1024);
        c->grid = dim3((uint32_t)cus);
    } else {
        c->block = dim3(256);
        c->grid = dim3((uint32_t)cus * 8u);
    }
    if (c->variant != 3 && c->variant != 4 && c->variant != 5 && c->variant != 6) {
        const uint32_t W = c->variant == 1 ? c->grid.x : c->grid.x * (c->block.x / 64);
        hipError_t ew = hipMalloc(&c->wave_start, sizeof(uint32_t) * (W + 1));
        if (ew != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_NOMEM, std::string("allocation: ") + hipGetErrorString(ew));
        }
        partition_kernel<<<(W + 256) / 256, 256, 0, c->stream>>>(gd.row_off + v_begin, nloc, W, c->wave_start);
        ew = hipStreamSynchronize(c->stream);
        if (ew != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("partition: ") + hipGetErrorString(ew));
        }
    }
    if (c->variant == 1) {
        // segments need ascending rows (setupRnd2 graphs are; uploaded ones are sorted once, in
        // place -- neighbour order does not affect the sweep)
        if (!gd.sorted) {
            int rs = sort_rows_inplace(const_cast<GraphDev&>(gd));
            if (rs) { mcmc_destroy(c); return rs; }
        }
        const size_t segn = (size_t)(c->nblocks + 1) * std::max<uint32_t>(nloc, 1);
        hipError_t es = hipMalloc(&c->seg, sizeof(uint32_t) * segn);
        if (es == hipSuccess) {
            const uint32_t blocks = (uint32_t)std::min<size_t>((segn + 255) / 256, 65536);
            segment_kernel<<<blocks, 256, 0, c->stream>>>(gd.row_off + v_begin, gd.col_idx, nloc, c->nblocks,
                                                          c->block_log2, c->seg);
            es = hipStreamSynchronize(c->stream);
        }
        if (es != hipSuccess) {
            mcmc_destroy(c);
            return fail(MCMC_E_HIP, std::string("segments: ") + hipGetErrorString(es));
        }
    }
    if (ref && hipMalloc(&c->hist, sizeof(uint32_t) * 2u * c->hist_words) != hipSuccess) {
        mcmc_destroy(c);
        return fail(MCMC_E_NOMEM, "histogram allocation");
    }
    // the tables' null-stream uploads (hipMemcpy) do not order against the context's non-blocking
    // stream: the device is idle before the first sweep can read them
    if (hipError_t ed = hipDeviceSynchronize(); ed != hipSuccess) {
        mcmc_destroy(c);
        return fail(MCMC_E_HIP, std::string("context setup: ") + hipGetErrorString(ed));
    }
    *out = c;
    return MCMC_OK;
}

int mcmc_create(const mcmc_graph* g, const mcmc_params* p, uint32_t v_begin, uint32_t v_end, mcmc_ctx** out) {
    return create_impl(g, p, v_begin, v_end, nullptr, out);
}

int mcmc_ref_create(const mcmc_graph* g, const mcmc_params* p, mcmc_gpurand* rand, mcmc_ctx** out) {
    if (!rand) return fail(MCMC_E_ARG, "NULL XORWOW states");
    return create_impl(g, p, 0, g ? g->g.n : 0, rand, out);
}

int mcmc_set_glibc_window(mcmc_ctx* c, const uint32_t window[31]) {
    if (!c || !window) return fail(MCMC_E_ARG, "NULL argument");
    std::memcpy(c->glibc.r, window, sizeof(c->glibc.r));
    return MCMC_OK;
}

int mcmc_get_glibc_window(mcmc_ctx* c, uint32_t window[31]) {
    if (!c || !window) return fail(MCMC_E_ARG, "NULL argument");
    if (c->ran) {
        DevState h;
        int rc = download_state(c, &h);
        if (rc) return rc;
        for (int i = 0; i < 31; i++) window[i] = h.glibc_ring[(h.glibc_head + i) % 31];
    } else {
        std::memcpy(window, c->glibc.r, sizeof(c->glibc.r));
    }
    return MCMC_OK;
}

int mcmc_init_coloring(mcmc_ctx* c, const uint32_t* C0) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (c->ref) return fail(MCMC_E_STATE, "reference-GPU contexts initialise in mcmc_ref_run");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    const uint32_t n = c->n;
    const uint32_t s0 = minstd_seed_state(c->p.seed);
    if (c->wflag) MCMC_HIP_TRY(hipMemsetAsync(c->wflag, 0, std::max<uint32_t>(c->v_end - c->v_begin, 1u), c->stream));
    c->traj_ok = false;
    if (c->inc) MCMC_HIP_TRY(inc_reset(c));
    if (c->dc) MCMC_HIP_TRY(dc_reset(c));
    if (c->wt_buf) MCMC_HIP_TRY(wt_reset(c));
    if (C0) {
        for (uint32_t v = 0; v < n; v++)
            if (C0[v] >= c->p.nCol) return fail(MCMC_E_ARG, "initial colour out of range");
        std::vector<uint8_t> h((size_t)n * c->cbytes);
        for (uint32_t v = 0; v < n; v++) {
            if (c->cbytes == 2) reinterpret_cast<uint16_t*>(h.data())[v] = (uint16_t)C0[v];
            else h[v] = (uint8_t)C0[v];
        }
        int rc = upload_colors(c, c->colors[0], h.data());
        if (rc) return rc;
        c->initDraws = n;
    } else {
        DevState zero{};
        MCMC_HIP_TRY(hipMemcpyAsync(c->st, &zero, sizeof(zero), hipMemcpyHostToDevice, c->stream));
        const UniformIntConst k = uniform_int_const(c->p.nCol);
        const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 255) / 256, 4096u));
        if (c->cbytes == 2)
            init_coloring_wide_kernel<<<blocks, 256, 0, c->stream>>>(reinterpret_cast<uint16_t*>(c->colors[0]), n, s0,
                                                                     k, c->st);
        else
            init_coloring_kernel<<<blocks, 256, 0, c->stream>>>(c->colors[0], n, s0, k, c->st);
        MCMC_HIP_TRY(hipGetLastError());
        DevState h;
        int rc = download_state(c, &h);
        if (rc) return rc;
        uint64_t draws = n;
        if (h.init_rejections > 0) {
            // Exact sequential replay of uniform_int_distribution's rejection loop.
            std::vector<uint8_t> hc((size_t)n * c->cbytes);
            uint32_t x = s0;
            draws = 0;
            for (uint32_t v = 0; v < n; v++) {
                uint32_t r;
                do { x = minstd_mulmod(x, kMinstdA); r = x - 1u; draws++; } while (r >= k.past);
                if (c->cbytes == 2) reinterpret_cast<uint16_t*>(hc.data())[v] = (uint16_t)(r / k.scaling);
                else hc[v] = (uint8_t)(r / k.scaling);
            }
            rc = upload_colors(c, c->colors[0], hc.data());
            if (rc) return rc;
        }
        c->initDraws = draws;
    }
    c->x0 = minstd_mulmod(s0, minstd_pow(kMinstdA, c->initDraws));
    if (c->taboo) MCMC_HIP_TRY(hipMemsetAsync(c->taboo, 0, sizeof(uint32_t) * (c->v_end - c->v_begin), c->stream));
    int rc = upload_state(c, 0);
    if (rc) return rc;
    if (c->wfp[0]) {   // the fingerprints of C_0 (later sweeps' writers keep them when fp_live)
        SweepArgs a = make_args(c, 0);
        wide_fp_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((c->n + 2047u) / 2048u, 4096u)), 256, 0, c->stream>>>(a);
        MCMC_HIP_TRY(hipGetLastError());
        MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    }
    c->initialized = true;
    c->ran = false;
    return MCMC_OK;
}

int mcmc_run(mcmc_ctx* c, uint32_t max_sweeps, mcmc_run_stats* stats) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (c->ref) return fail(MCMC_E_STATE, "reference-GPU contexts run with mcmc_ref_run");
    if (!c->initialized) return fail(MCMC_E_STATE, "mcmc_init_coloring must precede mcmc_run");
    if (c->v_begin != 0 || c->v_end != c->n)
        return fail(MCMC_E_STATE, "mcmc_run drives whole-graph contexts; use mcmc_part_* for partitions");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    const uint32_t total = max_sweeps ? max_sweeps : c->p.maxRip + 2;   // +1 final count pass
    const uint32_t batch = std::min<uint32_t>(16u, total);
    DevState h{};
    long long lv = -1;
    int rc = MCMC_OK;
    if (c->wsa.ctl && c->ran) {
        rc = download_state(c, &h);
        if (rc == MCMC_OK) rc = last_cviol(c, h, &lv);
        if (rc) return rc;
    }
    ws_choose(c, lv);
    rc = build_batch_graph(c, batch);
    if (rc) return rc;
    c->ran = true;
    c->traj_ok = true;
    MCMC_HIP_TRY(hipEventRecord(c->ev0, c->stream));
    if ((rc = dc_prep(c))) return rc;   // a fresh colouring's count rebuild (timed with the loop)
    uint32_t launched = 0;
    while (launched < total) {
        if (total - launched >= batch) {
            MCMC_HIP_TRY(hipGraphLaunch(c->ws_on ? c->batch_exec_ws : c->batch_exec, c->stream));
            launched += batch;
        } else {
            SweepArgs a = make_args(c, 1);
            launch_sweeps(c, a, total - launched);
            launched = total;
            MCMC_HIP_TRY(hipGetLastError());
        }
        rc = download_state(c, &h);
        if (rc) return rc;
        if (h.done || h.err) break;
        if (c->wsa.ctl && !c->ws_on && launched < total) {   // near convergence: the persistent sweep
            rc = last_cviol(c, h, &lv);
            if (rc) return rc;
            ws_choose(c, lv);
            if (c->ws_on && (rc = build_batch_graph(c, batch))) return rc;
        }
    }
    MCMC_HIP_TRY(hipEventRecord(c->ev1, c->stream));
    MCMC_HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0;
    MCMC_HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (h.err) return fail(MCMC_E_DEVICE, dev_err_text(h.err));
    mcmc_run_stats s{};
    if (h.done) {
        s.iter = h.iter;
        s.maxIterReached = (int32_t)h.maxIterReached;
        s.finalViol = h.finalViol;
        s.trajLen = std::min<uint64_t>((uint64_t)h.iter + 1, c->traj_cap);   // entries kept
        s.sweepsRun = h.iter + 1;
    } else {
        // early stop (max_sweeps): h.t sweeps accepted, no final count
        s.iter = h.t;
        s.maxIterReached = 0;
        s.finalViol = ~0ull;
        s.trajLen = std::min<uint64_t>(h.t, c->traj_cap);
        s.sweepsRun = h.t;
    }
    s.glibcDraws = h.glibc_draws;
    s.initDraws = c->initDraws;
    s.loopMs = ms;
    c->tail_traj.clear();
    if (h.done && c->tailcut_max) {
        rc = run_tailcut(c, h, &s.finalViol, &s.tailcutPasses);
        if (rc) return rc;
        if (c->dc) MCMC_HIP_TRY(dc_reset(c));   // the passes changed colours outside a sweep
        if (c->wt_buf) MCMC_HIP_TRY(wt_reset(c));
        if (c->inc) MCMC_HIP_TRY(inc_reset(c));
    }
    c->last = s;
    // keep the host copy of the glibc window in step with the device stream
    for (int i = 0; i < 31; i++) c->glibc.r[i] = h.glibc_ring[(h.glibc_head + i) % 31];
    if (stats) *stats = s;
    return MCMC_OK;
}

// Conflicting vertices of the context's current colouring (violation_count, coloringMCMC_CPU.cpp:
// 329-351), counted by the tail cut's recount kernel -- a code path independent of the sweep's
// fused count (test hook for the full-size checks). Whole-graph uint8 contexts. flags: optional
// [n] host bytes, the per-vertex flags.
int mcmc_count_violations(mcmc_ctx* c, uint64_t* count, uint8_t* flags) {
    if (!c || !count) return fail(MCMC_E_ARG, "NULL argument");
    if (c->part || c->v_begin != 0 || c->v_end != c->n)
        return fail(MCMC_E_STATE, "violation recount: whole-graph contexts");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    int rc = ensure_tail_buffers(c);
    if (rc) return rc;
    uint32_t which = 0;
    if (c->ran) {
        DevState h{};
        rc = download_state(c, &h);
        if (rc) return rc;
        which = h.t & 1u;
    }
    rc = tail_count(tail_view(c), c->colors[which], c->cbytes, c->vflags, c->tc_count, c->stream, false);
    if (rc) return rc;
    unsigned long long hv = 0;
    MCMC_HIP_TRY(hipMemcpyAsync(&hv, c->tc_count, sizeof(hv), hipMemcpyDeviceToHost, c->stream));
    if (flags) MCMC_HIP_TRY(hipMemcpyAsync(flags, c->vflags, c->n, hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    *count = hv;
    return MCMC_OK;
}

int mcmc_set_scan_stats(mcmc_ctx* c, int on) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    if (on && !c->scan_stats) MCMC_HIP_TRY(hipMalloc(&c->scan_stats, 6 * sizeof(unsigned long long)));
    if (on) MCMC_HIP_TRY(hipMemsetAsync(c->scan_stats, 0, 6 * sizeof(unsigned long long), c->stream));
    c->scan_stats_on = on != 0;
    drop_graphs(c);
    return MCMC_OK;
}

int mcmc_get_scan_stats_ex(mcmc_ctx* c, uint64_t* quads, uint64_t* used, uint64_t* pairs) {
    if (!c || !quads || !pairs) return fail(MCMC_E_ARG, "NULL argument");
    unsigned long long h[3] = {0, 0, 0};
    if (c->scan_stats) {
        MCMC_HIP_TRY(hipSetDevice(c->g->device));
        MCMC_HIP_TRY(hipMemcpy(h, c->scan_stats, sizeof(h), hipMemcpyDeviceToHost));
    }
    *quads = h[0];
    if (used) *used = h[2];
    *pairs = h[1];
    return MCMC_OK;
}

int mcmc_get_scan_stats(mcmc_ctx* c, uint64_t* quads, uint64_t* pairs) {
    return mcmc_get_scan_stats_ex(c, quads, nullptr, pairs);
}

int mcmc_get_scan_stats_v2(mcmc_ctx* c, uint64_t out[6]) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    unsigned long long h[6] = {0, 0, 0, 0, 0, 0};
    if (c->scan_stats) {
        MCMC_HIP_TRY(hipSetDevice(c->g->device));
        MCMC_HIP_TRY(hipMemcpy(h, c->scan_stats, sizeof(h), hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < 6; i++) out[i] = h[i];
    return MCMC_OK;
}

int mcmc_get_wide_inc_stats(mcmc_ctx* c, uint64_t out[5]) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    for (int i = 0; i < 5; i++) out[i] = 0;
    if (c->wt_buf) {   // the wide tiled sweep's counts: [1] incremental sweeps, [2] full, [3] changed rows,
                       // [4] violators walked in incremental sweeps
        MCMC_HIP_TRY(hipSetDevice(c->g->device));
        MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
        unsigned long long h[4];
        MCMC_HIP_TRY(hipMemcpy(h, c->wt_buf + kWtStat, sizeof(h), hipMemcpyDeviceToHost));
        out[0] = 1;
        out[1] = h[1];
        out[2] = h[0];
        out[3] = h[2];
        out[4] = h[3];
        return MCMC_OK;
    }
    if (!c->inc) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned long long h[4];
    MCMC_HIP_TRY(hipMemcpy(h, c->inc + kIncStat, sizeof(h), hipMemcpyDeviceToHost));
    out[0] = 1;
    for (int i = 0; i < 4; i++) out[1 + i] = h[i];
    return MCMC_OK;
}

// The persistent wide sweep (wide_solo.h): [0] set up, [1] window states, [2] its sweeps, [3] phases
// posted, [4] violators the leader walked, [5] walk phases, [6] delta phases, [7] violator
// collections, [8] candidate rows evaluated, [9] changed rows; diagnostics: [10] the watchdog word,
// [11] / [12] the leader's last sweep of a launch and its step, [13] the phase flag word; [14..21]
// wall-clock ticks (100 MHz) of its sweeps' steps: walks, candidates, walk wait, events, changed
// rows, count moves, violator list, whole sweeps; [22..29] finer probes (diagnostics, wide_solo.h).
int mcmc_get_wide_solo_stats(mcmc_ctx* c, uint64_t out[30]) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    for (int i = 0; i < 30; i++) out[i] = 0;
    if (!c->wsa.ctl) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    uint32_t h[kWsWords];
    MCMC_HIP_TRY(hipMemcpyAsync(h, c->wsa.ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(h + kWsStat);
    out[0] = 1;
    out[1] = c->wsa.nw;
    for (int i = 0; i < 8; i++) out[2 + i] = q[i];
    out[10] = h[kWsErr];
    out[11] = h[kWsDbg];
    out[12] = h[kWsDbg + 1];
    out[13] = h[kWsGen];
    const unsigned long long* tq = reinterpret_cast<const unsigned long long*>(h + kWsTime);
    for (int i = 0; i < 16; i++) out[14 + i] = tq[i];
    return MCMC_OK;
}

// Diagnostics (MCMC_WS_DEBUG at mcmc_create): the persistent wide sweep's progress words, read from
// host memory without touching the device (callable while a launch runs).
int mcmc_ws_debug(mcmc_ctx* c, uint32_t* out, uint32_t n) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    for (uint32_t i = 0; i < n; i++) out[i] = c->ws_dbg_host && i < 4096 ? __atomic_load_n(&c->ws_dbg_host[i], __ATOMIC_RELAXED) : 0u;
    return MCMC_OK;
}

int mcmc_get_dense_stats(mcmc_ctx* c, uint64_t out[10]) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    for (int i = 0; i < 10; i++) out[i] = 0;
    if (!c->dc) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    uint32_t h[kDcWords];
    MCMC_HIP_TRY(hipMemcpyAsync(h, c->dc_ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    const unsigned long long* s = reinterpret_cast<const unsigned long long*>(h + kDcStat);
    out[0] = 1;
    out[1] = c->dc_s0;
    out[2] = c->dc_s1;
    out[3] = s[0];
    out[4] = s[1];
    out[5] = s[2];
    out[6] = s[3];
    out[7] = c->dc_max;
    out[8] = h[kDcStat2];
    out[9] = h[kDcStat2 + 1];
    return MCMC_OK;
}

int mcmc_get_dense_stats_v2(mcmc_ctx* c, uint64_t out[16]) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    for (int i = 0; i < 16; i++) out[i] = 0;
    int rc = mcmc_get_dense_stats(c, out);
    if (rc || !c->dc) return rc;
    uint32_t h[kDcWords];
    MCMC_HIP_TRY(hipMemcpyAsync(h, c->dc_ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    unsigned long long os = 0;
    if (c->dc_osum) MCMC_HIP_TRY(hipMemcpyAsync(&os, c->dc_osum, sizeof(os), hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    out[10] = reinterpret_cast<const unsigned long long*>(h + kDcSoloStat)[0];   // solo sweeps
    out[11] = c->dl_n;                                                           // window states
    out[12] = c->dcm_launch ? 1u : 0u;                                           // persistent launch
    out[13] = (uint32_t)os;                                                      // nonzero open words now
    out[14] = reinterpret_cast<const unsigned long long*>(h + kDcSoloEval)[0];   // rows solo sweeps evaluated
    out[15] = c->dc_tid ? 1u : 0u;                                               // the rebuild's transposed ids
    return MCMC_OK;
}

int mcmc_get_dense_counts(mcmc_ctx* c, uint32_t row0, uint32_t rows, uint32_t* counts, uint32_t* masks) {
    if (!c || (rows && !counts)) return fail(MCMC_E_ARG, "NULL argument");
    if (!c->dc) return fail(MCMC_E_STATE, "the context keeps no dense counts");
    const uint32_t nloc = c->v_end - c->v_begin;
    if (row0 > nloc || rows > nloc - row0) return fail(MCMC_E_ARG, "rows outside the context");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    const size_t nc = c->p.nCol;
    MCMC_HIP_TRY(hipMemcpyAsync(counts, c->dc_cnt + (size_t)row0 * nc, sizeof(uint32_t) * nc * rows,
                                hipMemcpyDeviceToHost, c->stream));
    if (masks)
        MCMC_HIP_TRY(hipMemcpyAsync(masks, c->dc_mask + (size_t)row0 * c->nw, sizeof(uint32_t) * c->nw * rows,
                                    hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int mcmc_set_bench_mode(mcmc_ctx* c, int on) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    c->bench_mode = on ? 1 : 0;
    drop_graphs(c);
    return MCMC_OK;
}

int mcmc_set_tailcut_repair(mcmc_ctx* c, uint32_t max_passes) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (!c->part && (c->v_begin != 0 || c->v_end != c->n))
        return fail(MCMC_E_STATE, "tail cutting runs on whole-graph (mcmc_run) or partitioned (mcmc_part_run) contexts");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    if (max_passes) {
        int rc = ensure_tail_buffers(c);
        if (rc) return rc;
    }
    if ((max_passes != 0) != (c->tailcut_max != 0)) {
        // captured sweeps carry the flag pointer: re-capture with the new setting
        drop_graphs(c);
    }
    c->tailcut_max = max_passes;
    return MCMC_OK;
}

int mcmc_ref_init(mcmc_ctx* c) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (!c->ref) return fail(MCMC_E_STATE, "mcmc_ref_init needs a context from mcmc_ref_create");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    const uint32_t n = c->n, nCol = c->p.nCol;
    // run() (coloringMCMC_main.cu:101-158): taboo cleared, colours from the states' next draw
    c->rand_base = c->rand->cur;
    drop_graphs(c);   // states moved
    MCMC_HIP_TRY(hipMemsetAsync(c->hist, 0, sizeof(uint32_t) * 2u * c->hist_words, c->stream));
    if (c->taboo) MCMC_HIP_TRY(hipMemsetAsync(c->taboo, 0, sizeof(uint32_t) * n, c->stream));
    int rc = upload_state(c, 0);
    if (rc) return rc;
    const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 255) / 256, 2048u));
    if (c->refwide) {
        refw_init_kernel<<<blocks, 256, 0, c->stream>>>(reinterpret_cast<uint16_t*>(c->colors[0]),
                                                        c->rand->states[c->rand_base], n, nCol, c->hist);
        const SweepArgs a = make_args(c, 1);
        refw_ptab_kernel<<<std::max<uint32_t>(1u, (nCol + 255u) / 256u), 256, 0, c->stream>>>(a, 0u);
        // sweep 0 adjusts a copy of C_0's histogram (refw_hist_move)
        MCMC_HIP_TRY(hipMemcpyAsync(c->hist + c->hist_words, c->hist, sizeof(uint32_t) * c->hist_words,
                                    hipMemcpyDeviceToDevice, c->stream));
    } else
        ref_init_kernel<<<blocks, 256, 0, c->stream>>>(c->colors[0], c->rand->states[c->rand_base], n, nCol, c->hist);
    MCMC_HIP_TRY(hipGetLastError());
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    c->initialized = true;
    c->ran = true;
    return MCMC_OK;
}

int mcmc_ref_run(mcmc_ctx* c, uint32_t tail_max_passes, mcmc_run_stats* stats) {
    int rc = mcmc_ref_init(c);
    if (rc) return rc;
    c->tailcut_max = tail_max_passes;
    if (c->p.tailcut && tail_max_passes) {
        rc = ensure_tail_buffers(c);
        if (rc) return rc;
    }
    const uint32_t cap = c->p.maxRip > 0 ? c->p.maxRip : 1u;
    const uint32_t total = cap + 1u;   // cap sweeps + the count-only pass
    const uint32_t batch = std::min<uint32_t>(16u, total);
    rc = build_batch_graph(c, batch);
    if (rc) return rc;
    MCMC_HIP_TRY(hipEventRecord(c->ev0, c->stream));
    uint32_t launched = 0;
    DevState h{};
    while (launched < total) {
        if (total - launched >= batch) {
            MCMC_HIP_TRY(hipGraphLaunch(c->batch_exec, c->stream));
            launched += batch;
        } else {
            SweepArgs a = make_args(c, 1);
            for (; launched < total; launched++) launch_pair(c, a);
            MCMC_HIP_TRY(hipGetLastError());
        }
        rc = download_state(c, &h);
        if (rc) return rc;
        if (h.done) break;
    }
    MCMC_HIP_TRY(hipEventRecord(c->ev1, c->stream));
    MCMC_HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0;
    MCMC_HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (!h.done) return fail(MCMC_E_DEVICE, "reference-GPU loop did not finish");
    c->rand->cur = (c->rand_base + h.t) & 1u;   // sweep t's own state writes were discarded
    mcmc_run_stats st{};
    st.iter = h.iter;                             // rip
    st.maxIterReached = (int32_t)h.maxIterReached;
    st.finalViol = h.finalViol;                   // conflicting edges of the returned colouring
    st.trajLen = std::min<uint64_t>((uint64_t)h.t + 1, c->traj_cap);
    st.sweepsRun = (h.t == cap) ? cap : h.t;      // selectStar launches of the reference
    st.initDraws = c->n;
    st.loopMs = ms;
    c->last = st;
    c->tail_traj.clear();
    if (c->p.tailcut && tail_max_passes) {
        // the host's conflictCounter: C_t's count, or C_(cap-1)'s when the loop ran out (:163, :229)
        unsigned long long cc = 0;
        const uint32_t idx = (h.t == cap) ? h.t - 1u : h.t;
        MCMC_HIP_TRY(hipMemcpyAsync(&cc, c->traj + idx, sizeof(cc), hipMemcpyDeviceToHost, c->stream));
        MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
        rc = run_tailcut_ref(c, h, cc, &st.finalViol, &st.tailcutPasses);
        if (rc) return rc;
        c->last = st;
    }
    if (stats) *stats = st;
    return MCMC_OK;
}

int mcmc_get_tail_trajectory(mcmc_ctx* c, uint64_t* out, uint64_t cap, uint64_t* len) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (len) *len = c->tail_traj.size();
    for (uint64_t i = 0; out && i < std::min<uint64_t>(cap, c->tail_traj.size()); i++) out[i] = c->tail_traj[i];
    return MCMC_OK;
}

int mcmc_get_coloring(mcmc_ctx* c, uint32_t* out) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    DevState h{};
    uint32_t which = 0;
    if (c->ran) {
        int rc = download_state(c, &h);
        if (rc) return rc;
        which = h.t & 1;
    }
    std::vector<uint8_t> tmp((size_t)c->n * c->cbytes);
    int rc = download_colors(c, c->colors[which], tmp.data());
    if (rc) return rc;
    if (c->cbytes == 2)
        for (uint32_t v = 0; v < c->n; v++) out[v] = reinterpret_cast<const uint16_t*>(tmp.data())[v];
    else
        for (uint32_t v = 0; v < c->n; v++) out[v] = tmp[v];
    return MCMC_OK;
}

int mcmc_get_trajectory(mcmc_ctx* c, uint64_t* out, uint64_t cap, uint64_t* len) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    const uint64_t L = std::min<uint64_t>(c->last.trajLen, c->traj_cap);
    if (len) *len = L;
    if (out && cap) {
        std::vector<unsigned long long> tmp(L);
        if (L) {
            MCMC_HIP_TRY(hipMemcpyAsync(tmp.data(), c->traj, L * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
            MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
        }
        for (uint64_t i = 0; i < std::min(L, cap); i++) out[i] = tmp[i];
    }
    return MCMC_OK;
}

int mcmc_bench_prepare(mcmc_ctx* c, uint32_t sweeps) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (sweeps == 0) return fail(MCMC_E_ARG, "sweeps must be > 0");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    long long lv = -1;
    if (c->wsa.ctl && c->ran && c->ws_enter >= 0) {
        // the path for the colouring the timed sweeps start from: its violators, recounted
        uint64_t cv = 0;
        int rc = mcmc_count_violations(c, &cv, nullptr);
        if (rc) return rc;
        lv = (long long)cv;
    }
    ws_choose(c, lv);
    if (c->bench_exec && c->bench_n == sweeps && c->bench_ws == c->ws_on) return MCMC_OK;
    if (c->bench_exec) { (void)hipGraphExecDestroy(c->bench_exec); c->bench_exec = nullptr; }
    // Throughput mode: the loop body with the stop tests disabled (no cap, no convergence stop:
    // a sweep from a proper colouring still resamples every vertex), `sweeps` launches captured
    // into one hipGraph.
    SweepArgs a = make_args(c, 1);
    a.maxRip = 0xFFFFFFF0u;
    a.traj_cap = 0;
    a.bench = 1;   // a convergent run (C5) keeps sweeping from its proper colouring
    hipGraph_t graph;
    MCMC_HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    launch_sweeps(c, a, sweeps);
    MCMC_HIP_TRY(hipStreamEndCapture(c->stream, &graph));
    hipError_t e = hipGraphInstantiate(&c->bench_exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    MCMC_HIP_TRY(hipGraphUpload(c->bench_exec, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    c->bench_n = sweeps;
    c->bench_ws = c->ws_on;
    return MCMC_OK;
}

int mcmc_bench_sweeps(mcmc_ctx* c, uint32_t sweeps, double* total_ms, double* sweep_kernel_ms) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    if (!c->initialized) return fail(MCMC_E_STATE, "mcmc_init_coloring must precede mcmc_bench_sweeps");
    if (!(c->bench_exec && c->bench_n == sweeps)) {   // (prepared for `sweeps`: as captured)
        int rc = mcmc_bench_prepare(c, sweeps);
        if (rc) return rc;
    }
    int rc = MCMC_OK;
    c->ran = true;
    c->traj_ok = false;   // throughput mode keeps no trajectory
    // one graph replay between two events on the sweep stream: total = device wall of the loop,
    // per-launch average = total / sweeps (each launch is one fused sweep, gap included)
    MCMC_HIP_TRY(hipEventRecord(c->ev0, c->stream));
    if ((rc = dc_prep(c))) return rc;   // a fresh colouring's count rebuild (timed with the sweeps)
    MCMC_HIP_TRY(hipGraphLaunch(c->bench_exec, c->stream));
    MCMC_HIP_TRY(hipEventRecord(c->ev1, c->stream));
    MCMC_HIP_TRY(hipEventSynchronize(c->ev1));
    float tot = 0;
    MCMC_HIP_TRY(hipEventElapsedTime(&tot, c->ev0, c->ev1));
    DevState h{};
    rc = download_state(c, &h);
    if (rc) return rc;
    if (h.err) return fail(MCMC_E_DEVICE, dev_err_text(h.err));
    if (total_ms) *total_ms = tot;
    if (sweep_kernel_ms) *sweep_kernel_ms = (double)tot / sweeps;
    if (c->pair_trace) {   // diagnostics: the last sweep's per-pair records, gridDim x kPairTraceMax x kPairTraceRec
        std::vector<unsigned long long> h_tr((size_t)kPairTraceRec * kPairTraceMax * c->grid.x);
        MCMC_HIP_TRY(hipMemcpy(h_tr.data(), c->pair_trace, h_tr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("MCMC_PAIR_TRACE"), "wb")) {
            fwrite(h_tr.data(), sizeof(unsigned long long), h_tr.size(), f);
            fclose(f);
        }
    }
    if (c->solo_ts) {   // diagnostics: the persistent launch's per-sweep stamps of its leader
        std::vector<unsigned long long> h_ts(8u * 4096u);
        MCMC_HIP_TRY(hipMemcpy(h_ts.data(), c->solo_ts, h_ts.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("MCMC_SOLO_TRACE"), "wb")) {
            fwrite(h_ts.data(), sizeof(unsigned long long), h_ts.size(), f);
            fclose(f);
        }
    }
    if (c->phase_ts) {   // diagnostics: the last sweep's per-workgroup phase timestamps (+ commit stamps)
        std::vector<unsigned long long> h_ts(kPhaseWords);
        MCMC_HIP_TRY(hipMemcpy(h_ts.data(), c->phase_ts, h_ts.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(getenv("MCMC_PHASE_DUMP"), "wb")) {
            fwrite(h_ts.data(), sizeof(unsigned long long), h_ts.size(), f);
            fclose(f);
        }
    }
    return MCMC_OK;
}

uint32_t mcmc_cdf_walk(const uint32_t* mask, uint32_t nCol, uint32_t cv, float eps, float p, float u) {
    if (nCol == 0) return 0;
    if (!mask) {
        std::vector<float> E((size_t)nCol + 1);
        eps_table(eps, nCol, E.data());
        const uint32_t c = cv < nCol ? cv : nCol - 1u;   // the table walk and the binade walk must agree
        const uint32_t r = walk_own_tab(E.data(), nCol, c, eps, p, u);
        return r == walk_own(nCol, c, eps, p, u) ? r : 0xFFFFFFFFu;
    }
    // the wave walk of wide_walk_kernel (host build: the 64 lanes as a loop); the per-word serial
    // walk must agree, else the hook reports 0xFFFFFFFF
    const uint32_t NWW = (nCol + 31u) >> 5;
    std::vector<uint32_t> pre((size_t)NWW + 1, 0u);
    for (uint32_t w = 0; w < NWW; w++) pre[w + 1] = pre[w] + (uint32_t)__builtin_popcount(mask[w]);
    const uint32_t r = walk_mask_pre(mask, pre.data(), nCol, eps, p, u);
    return r == walk_mask(mask, nCol, eps, p, u) ? r : 0xFFFFFFFFu;
}

int mcmc_get_info(mcmc_ctx* c, mcmc_ctx_info* out) {
    if (!c || !out) return fail(MCMC_E_ARG, "NULL argument");
    mcmc_ctx_info i{};
    const uint64_t nloc = c->v_end - c->v_begin;
    uint64_t mloc = 0;
    if (c->tl) {
        mloc = c->tl->arcs;
    } else {
        uint64_t ends[2];
        MCMC_HIP_TRY(hipMemcpy(&ends[0], c->g->row_off + c->v_begin, sizeof(uint64_t), hipMemcpyDeviceToHost));
        MCMC_HIP_TRY(hipMemcpy(&ends[1], c->g->row_off + c->v_end, sizeof(uint64_t), hipMemcpyDeviceToHost));
        mloc = ends[1] - ends[0];
    }
    const uint64_t taboo = c->p.tabooIteration > 0 ? 8 * nloc : 0;
    // REF: XORWOW states read and written (24 + 24 B per vertex), the rows' own colours (streamed
    // per group), both histograms; the reference's B_alg adds the same states plus its n*nCol
    // colorsChecker memset and row writes it does not model here
    const uint64_t ref_extra = c->ref ? 48 * nloc + nloc + 8ull * kHistWords : 0;
    i.variant = c->variant;
    i.resident = c->variant_res ? 1 : 0;
    i.block_log2 = c->block_log2;
    i.nblocks = c->nblocks;
    i.grid = c->grid.x;
    i.block = c->block.x;
    i.lds_bytes = c->lds;
    i.ref_bytes = 4 * (nloc + 1) + 4 * mloc + 4 * (uint64_t)c->n + 4 * nloc + taboo + (c->ref ? 48 * nloc : 0);
    if (c->tl) {
        const TiledLayout& t = *c->tl;
        i.grp_rows = t.grp_rows;
        i.ngroups = t.ngroups;
        i.sub_log2 = c->sub_log2;
        const uint64_t segb = 4ull * tseg_stride(t.grp_rows) * t.ngroups * t.nblocks + 8ull * (t.ngroups + 1);
        i.layout_bytes = 2 * t.ids + segb;
        i.sweep_bytes = i.layout_bytes + (uint64_t)c->cbytes * (c->n + nloc) + taboo + ref_extra;
    } else if (c->wide && c->xs) {
        // slab entries + chunk base rows; colour replica read once; per own vertex the flag, the
        // colour read and the colour write (1 + 2 + 2 B)
        i.layout_bytes = 4ull * kWideChunk * c->xs->chunks + 4ull * c->xs->chunks;
        i.sweep_bytes = i.layout_bytes + 2 * (uint64_t)c->n + 5 * nloc + taboo +
                        (c->xs->mode == 1 ? (uint64_t)c->n : 0);   // LDS mode: the fingerprint array
    } else if (c->refwide) {
        // CSR; colour replica read once, own colours read and written (2 B each), both histograms
        i.layout_bytes = 8 * (nloc + 1) + 4 * mloc;
        i.sweep_bytes = i.layout_bytes + 2 * (uint64_t)c->n + 4 * nloc + taboo + 48 * nloc + 8ull * c->hist_words;
    } else if (c->wide) {
        // CSR + per-chunk row table; colour replica read once + own colours + write (2 B each)
        i.layout_bytes = 8 * (nloc + 1) + 4 * mloc + 4ull * (c->nchunks + 1);
        i.sweep_bytes = i.layout_bytes + 2 * (uint64_t)c->n + 4 * nloc + taboo;
    } else {
        i.layout_bytes = 8 * (nloc + 1) + 4 * mloc;
        i.sweep_bytes = i.layout_bytes + c->n + nloc + taboo;
    }
    *out = i;
    return MCMC_OK;
}

void mcmc_destroy(mcmc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->g->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    drop_graphs(c);
    (void)hipFree(c->own_colors[0]);
    (void)hipFree(c->own_colors[1]);
    (void)hipFree(c->taboo);
    (void)hipFree(c->events);
    (void)hipFree(c->evdraw);
    (void)hipFree(c->st);
    (void)hipFree(c->traj);
    (void)hipFree(c->wave_start);
    (void)hipFree(c->seg);
    (void)hipFree(c->phase_ts);
    (void)hipFree(c->tq_l);
    (void)hipFree(c->ewalk);
    (void)hipFree(c->tq_m);
    (void)hipFree(c->pair_trace);
    (void)hipFree(c->vflags);
    (void)hipFree(c->tc_list);
    (void)hipFree(c->tc_len);
    (void)hipFree(c->tc_colorIdx);
    (void)hipFree(c->tc_count);
    (void)hipFree(c->tc_tmp);
    (void)hipFree(c->hist);
    (void)hipFree(c->rw_cnt);
    (void)hipFree(c->rw_lists);
    (void)hipFree(c->ptab);
    (void)hipFree(c->chunk_row);
    (void)hipFree(c->wflag);
    (void)hipFree(c->wfp[0]);
    (void)hipFree(c->wfp[1]);
    (void)hipFree(c->evblk);
    (void)hipFree(c->ftab);
    (void)hipFree(c->evcnt);
    (void)hipFree(c->evpow);
    (void)hipFree(c->gpow);
    (void)hipFree(c->wlist);
    (void)hipFree(c->wcount);
    (void)hipFree(c->inc);
    (void)hipFree(c->gmask);
    (void)hipFree(c->etab);
    (void)hipFree(c->scan_stats);
    (void)hipFree(c->dc_ctl);
    (void)hipFree(c->dc_cnt);
    (void)hipFree(c->dc_mask);
    (void)hipFree(c->dc_open);
    (void)hipFree(c->dc_tid);
    (void)hipFree(c->dc_toff);
    (void)hipFree(c->dc_osum);
    (void)hipFree(c->dl_tab);
    (void)hipFree(c->solo_ts);
    (void)hipFree(c->wt_tick);
    (void)hipFree(c->wt_buf);
    (void)hipFree(c->ws_buf);
    if (c->ws_dbg_host) (void)hipHostFree(c->ws_dbg_host);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream && !c->borrowed_stream) (void)hipStreamDestroy(c->stream);
    if (c->pres) {   // the driver's stream, pinned word and events
        (void)hipSetDevice(c->g->device);
        if (c->pres->poll) (void)hipStreamSynchronize(c->pres->poll);
        for (hipEvent_t e : c->pres->ev)
            if (e) (void)hipEventDestroy(e);
        if (c->pres->poll) (void)hipStreamDestroy(c->pres->poll);
        if (c->pres->pinned) (void)hipHostFree(c->pres->pinned);
        delete c->pres;
    }
    if (c->own_part) {   // native partitioned contexts: their buffers and their own stream
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->own_part);
        (void)hipFree(c->spill);
        if (c->stream) (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

}  // extern "C"

namespace mcmc {
int part_desc(mcmc_ctx* c, PartDesc* d) {
    if (!c || !d) return fail(MCMC_E_ARG, "NULL argument");
    if (!c->part) return fail(MCMC_E_STATE, "not a partitioned context");
    d->colors[0] = c->colors[0];
    d->colors[1] = c->colors[1];
    d->foot[0] = c->foot[0];
    d->foot[1] = c->foot[1];
    d->bounds = c->bounds.data();
    d->world = c->world;
    d->rank = c->rank;
    d->cbytes = c->cbytes;
    d->n = c->n;
    d->stream = c->stream;
    d->device = c->g->device;
    d->comm = c->comm;
    d->events = c->events;
    d->maxRip = c->p.maxRip;
    d->dlt[0] = c->dlt[0];
    d->dlt[1] = c->dlt[1];
    d->delta_ok = part_delta_ok(c);
    d->tailcut_max = c->tailcut_max;
    return MCMC_OK;
}

int part_adopt(mcmc_ctx* c, void* mem, hipStream_t own_stream, mcmc_comm* comm) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "not a partitioned context");
    c->own_part = mem;
    c->borrowed_stream = true;   // mcmc_destroy frees own_stream through the own_part path
    c->stream = own_stream;
    c->comm = comm;
    return MCMC_OK;
}

int part_stats(mcmc_ctx* c, mcmc_run_stats* s) {
    int32_t done = 0;
    uint32_t t = 0, err = 0;
    int rc = mcmc_part_state(c, &done, &t, &err);
    if (rc) return rc;
    *s = c->last;
    return MCMC_OK;
}

int part_set_delta(mcmc_ctx* c, uint32_t* d0, uint32_t* d1) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "not a partitioned context");
    c->dlt[0] = d0;
    c->dlt[1] = d1;
    return MCMC_OK;
}

bool part_delta_ok(const mcmc_ctx* c) { return c && c->part && c->dlt[0]; }

// A partition of one rank (world 1) steps exactly like a whole-graph context: the sweep commits in
// its last workgroup (no footer, no exchange, no commit launch). Not for the reference-semantics mode.
static bool part_solo(const mcmc_ctx* c) { return c->world == 1 && !c->ref && !getenv("MCMC_PART_SOLO_OFF"); }

const void* part_state_ptr(const mcmc_ctx* c) { return c->st; }
static_assert(kDeltaWords == kPartDeltaWords && kDeltaWords == MCMC_DELTA_WORDS, "delta slot size");
static_assert(offsetof(DevState, t) == 0 && offsetof(DevState, done) == 4 && offsetof(DevState, err) == 12,
              "part_state_ptr readers take {t, done, x_t, err} from the first 16 bytes");

int part_sweep(mcmc_ctx* c, bool delta) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "mcmc_part_attach first");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    if (!c->initialized) return fail(MCMC_E_STATE, "mcmc_init_coloring must precede mcmc_part_sweep_async");
    if (delta && !part_delta_ok(c)) return fail(MCMC_E_STATE, "delta exchange: tiled partitioned contexts only");
    if (int rc = dc_prep(c)) return rc;
    c->ran = true;
    SweepArgs a = make_args(c, 1);
    a.dcap = delta ? kDeltaPairs : 0u;
    if (part_solo(c)) {
        // world 1: nothing to exchange -- the one-GPU step (the last workgroup commits, or the
        // wide sweep's commit launch); the step's part_commit is then a no-op
        a.fused = c->wide ? 0 : 1;
        launch_pair(c, a);
    } else {
        launch_tiled_or_diag(c, a);
        if (c->wide) wide_footer_kernel<<<1, kCommitThreads, 0, c->stream>>>(a);
    }
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

int part_solo_batch(mcmc_ctx* c, uint32_t steps) {
    if (!c || !c->part || !part_solo(c) || !c->initialized || steps == 0) return 1;
    // the legacy null stream (mcmc_part_attach with torch's default stream) cannot be captured:
    // the caller's per-step path then
    if (c->stream == nullptr) return 1;
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    if (int rc = dc_prep(c)) return rc;
    // the persistent wide sweep near convergence (ws_choose): one sync per batch until it is taken,
    // then it stays (it handles violators too), so the driver's batches pipeline again
    if (c->wsa.ctl && !(c->ran && c->ws_on)) {
        DevState h{};
        long long lv = -1;
        if (c->ran) {
            if (int rc = download_state(c, &h)) return rc;
            if (int rc = last_cviol(c, h, &lv)) return rc;
        }
        ws_choose(c, lv);
    }
    c->ran = true;
    c->traj_ok = true;
    {   // a persistent path: one launch for the batch, no graph (nothing to capture once per size)
        SweepArgs a = make_args(c, 1);
        a.dcap = 0u;
        a.fused = c->wide ? 0 : 1;
        if (persistent_path(c, a)) {
            launch_sweeps(c, a, steps);
            MCMC_HIP_TRY(hipGetLastError());
            return MCMC_OK;
        }
    }
    // (c->batch: the one-GPU run's batches are plain counts)
    const uint32_t key = 0x80000000u | (c->ws_on ? 0x40000000u : 0u) | steps;
    if (!(c->batch_exec && c->batch == key)) {
        if (c->batch_exec) { (void)hipGraphExecDestroy(c->batch_exec); c->batch_exec = nullptr; c->batch = 0; }
        SweepArgs a = make_args(c, 1);
        a.dcap = 0u;
        a.fused = c->wide ? 0 : 1;   // as part_sweep's world-1 step
        hipGraph_t graph;
        if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            (void)hipGetLastError();
            return 1;   // capture unsupported on this stream: the per-step path
        }
        launch_sweeps(c, a, steps);   // the persistent launches of the one-GPU run where they apply
        MCMC_HIP_TRY(hipStreamEndCapture(c->stream, &graph));
        hipError_t e = hipGraphInstantiate(&c->batch_exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (e != hipSuccess) return fail(MCMC_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
        c->batch = key;
    }
    MCMC_HIP_TRY(hipGraphLaunch(c->batch_exec, c->stream));
    return MCMC_OK;
}

int part_commit(mcmc_ctx* c, int mode, const uint32_t* spill, uint32_t stride) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "mcmc_part_attach first");
    if (part_solo(c)) return MCMC_OK;   // world 1: the sweep committed (part_sweep)
    if (mode > 0 && !part_delta_ok(c)) return fail(MCMC_E_STATE, "delta exchange: tiled partitioned contexts only");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    SweepArgs a = make_args(c, 1);
    a.part_delta = mode;
    if (c->wide) part_commit_kernel<uint16_t><<<1, kCommitThreads, 0, c->stream>>>(a, spill, stride);
    else part_commit_kernel<uint8_t><<<1, kCommitThreads, 0, c->stream>>>(a, spill, stride);
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

int part_sync_remote(mcmc_ctx* c) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "mcmc_part_attach first");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    SweepArgs a = make_args(c, 1);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(1024, ((uint64_t)c->n * c->cbytes / 16 + 255) / 256 + 1);
    if (c->wide) part_sync_remote_kernel<uint16_t><<<blocks, 256, 0, c->stream>>>(a);
    else part_sync_remote_kernel<uint8_t><<<blocks, 256, 0, c->stream>>>(a);
    MCMC_HIP_TRY(hipGetLastError());
    return MCMC_OK;
}

int part_resources(mcmc_ctx* c, PartRes** out) {
    if (!c->pres) {
        MCMC_HIP_TRY(hipSetDevice(c->g->device));
        std::unique_ptr<PartRes> r(new PartRes());
        MCMC_HIP_TRY(hipStreamCreateWithFlags(&r->poll, hipStreamNonBlocking));
        MCMC_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&r->pinned), 16, hipHostMallocDefault));
        MCMC_HIP_TRY(hipEventCreateWithFlags(&r->ev[0], hipEventDisableTiming));
        MCMC_HIP_TRY(hipEventCreate(&r->ev[1]));
        MCMC_HIP_TRY(hipEventCreate(&r->ev[2]));
        MCMC_HIP_TRY(hipEventCreateWithFlags(&r->ev[3], hipEventDisableTiming));
        MCMC_HIP_TRY(hipEventCreateWithFlags(&r->ev[4], hipEventDisableTiming));
        c->pres = r.release();
    }
    *out = c->pres;
    return MCMC_OK;
}

void part_add_xstats(mcmc_ctx* c, int64_t delta_steps, int64_t full_steps, int64_t ovf, int64_t bytes) {
    c->xs_delta += delta_steps;
    c->xs_full += full_steps;
    c->xs_ovf += ovf;
    c->xs_bytes += bytes;
}

int part_run_begin(mcmc_ctx* c) {
    c->tail_done = false;
    c->xs_delta = c->xs_full = c->xs_ovf = c->xs_bytes = 0;
    if (!part_delta_ok(c)) return MCMC_OK;
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    for (int k = 0; k < 2; k++)
        MCMC_HIP_TRY(hipMemsetAsync(c->dlt[k] + (size_t)c->rank * kDeltaWords, 0, sizeof(uint32_t) * kDeltaHead,
                                    c->stream));
    return MCMC_OK;
}

// ---- partitioned tail cut (coloringMCMC_CPU.cpp:272-311, corrected), driven by multi.hip --------
// The reference's repair pass is sequential in ascending vertex order; ranks own ascending ranges,
// so a pass runs rank by rank: rank r repairs its flagged rows on its replica (seeing the colours
// earlier ranks repaired in this pass), then its range is broadcast; the recount is per rank plus a
// sum. Exactly the single-context pass (tests/test_multi.py::test_native_loopback_tailcut*).
int part_tail_init(mcmc_ctx* c, uint64_t* cviol, uint32_t* t_final, uint8_t** colors) {
    if (!c || !c->part || !c->tailcut_max) return fail(MCMC_E_STATE, "partitioned context with tail cutting");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    DevState h{};
    if (int rc = download_state(c, &h)) return rc;
    if (!h.done || (h.err & (kErrFatal | kErrSpill | kErrDelta))) return fail(MCMC_E_STATE, "the loop has not finished");
    *cviol = h.finalViol;
    *t_final = h.t;
    *colors = c->colors[h.t & 1u];
    const uint32_t nCol = c->p.nCol;
    std::vector<size_t> colorIdx(nCol);   // identity (:131-132), by ascending histogram when z > 0 (:272-278)
    for (uint32_t i = 0; i < nCol; i++) colorIdx[i] = i;
    if (c->z > 0) {
        std::vector<uint8_t> hc((size_t)c->n * c->cbytes);
        if (int rc = download_colors(c, *colors, hc.data())) return rc;
        std::vector<size_t> histBins(nCol, 0);
        for (uint32_t v = 0; v < c->n; v++)
            histBins[c->cbytes == 2 ? reinterpret_cast<const uint16_t*>(hc.data())[v] : hc[v]]++;
        std::sort(colorIdx.begin(), colorIdx.end(), [&](int i, int j) { return histBins[i] < histBins[j]; });
    }
    std::vector<uint32_t> ci(colorIdx.begin(), colorIdx.end());
    MCMC_HIP_TRY(hipMemcpyAsync(c->tc_colorIdx, ci.data(), sizeof(uint32_t) * nCol, hipMemcpyHostToDevice, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    c->tail_traj.clear();
    return MCMC_OK;
}

// One rank's share of a pass: its flagged rows (first pass: the flags of the colouring before the
// last accepted sweep, as run_tailcut) repaired in order on the replica `C`.
int part_tail_repair(mcmc_ctx* c, uint8_t* C, uint32_t t_final, bool first) {
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    const uint32_t nloc = c->v_end - c->v_begin;
    const uint8_t* flags = c->vflags + (first ? (size_t)(t_final >= 1 ? (t_final - 1u) & 1u : 0u) * nloc : 0);
    if (int rc = tail_select(flags, nloc, c->tc_list, c->tc_len, &c->tc_tmp, &c->tc_tmp_bytes, c->stream)) return rc;
    return tail_repair(tail_view(c), C, c->cbytes, c->tc_list, c->tc_len, c->tc_colorIdx, c->p.nCol, c->stream, false,
                       ~0ull);
}

// The recount of this rank's rows (:308) into its flags; *count: the device word holding the sum.
int part_tail_count(mcmc_ctx* c, const uint8_t* C, unsigned long long** count) {
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    *count = c->tc_count;
    return tail_count(tail_view(c), C, c->cbytes, c->vflags, c->tc_count, c->stream, false);
}

void part_tail_done(mcmc_ctx* c, uint64_t cviol, uint32_t passes) {
    c->tail_done = true;
    c->tail_passes = passes;
    c->tail_viol = cviol;
    // the passes changed colours outside a sweep: dense counts and incremental violation counts
    // start over, as after mcmc_run's tail cut
    if (c->dc) (void)dc_reset(c);
    if (c->wt_buf) (void)wt_reset(c);
    if (c->inc) (void)inc_reset(c);
}

int part_spill_buffer(mcmc_ctx* c, uint32_t stride, uint32_t** buf) {
    const size_t need = (size_t)c->world * stride;
    if ((size_t)c->world * c->spill_stride < need || !c->spill) {
        (void)hipFree(c->spill);
        c->spill = nullptr;
        MCMC_HIP_TRY(hipMalloc(&c->spill, sizeof(uint32_t) * std::max<size_t>(need, 1)));
    }
    c->spill_stride = stride;
    *buf = c->spill;
    return MCMC_OK;
}
}  // namespace mcmc

extern "C" {

// ---- vertex-partitioned step (device-resident; exchange by the caller or by mcmc_part_run) -----
// The replica element size mcmc_create picks for nCol (the wide sweep: uint16).
uint32_t mcmc_color_bytes(uint32_t nCol) {
    const char* gv = getenv("MCMC_GATHER");
    return (nCol > 256 || (gv && (std::string(gv) == "wide" || std::string(gv) == "wide-tiled"))) ? 2u : 1u;
}

int mcmc_part_plan_rows(uint32_t n, uint32_t world, uint32_t* bounds) {
    if (!bounds) return fail(MCMC_E_ARG, "NULL argument");
    if (world == 0 || world > kMaxWorld) return fail(MCMC_E_ARG, "bad world (1..64 ranks)");
    const uint64_t S = (((uint64_t)n + world - 1) / world + kPartAlign - 1) / kPartAlign * kPartAlign;
    for (uint32_t r = 0; r <= world; r++) bounds[r] = (uint32_t)std::min<uint64_t>(S * r, n);
    bounds[world] = n;
    return MCMC_OK;
}

int mcmc_part_plan_csr(const uint64_t* row_off, uint32_t n, uint32_t world, uint32_t* bounds) {
    if (!row_off || !bounds) return fail(MCMC_E_ARG, "NULL argument");
    if (world == 0 || world > kMaxWorld) return fail(MCMC_E_ARG, "bad world (1..64 ranks)");
    // cost of rows [0, v): their arcs plus a per-row term for the evaluation, the own colour
    // read/write and the (row, block) table entries
    auto cost = [&](uint64_t v) { return (double)row_off[v] + kPartRowWeight * (double)v; };
    const double total = cost(n);
    bounds[0] = 0;
    for (uint32_t r = 1; r < world; r++) {
        const double target = total * r / world;
        uint64_t lo = bounds[r - 1], hi = n;   // first v with cost(v) >= target
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (cost(mid) < target) lo = mid + 1; else hi = mid;
        }
        uint64_t b = (lo + kPartAlign / 2) / kPartAlign * kPartAlign;   // nearest aligned row
        b = std::max<uint64_t>(b, bounds[r - 1]);
        bounds[r] = (uint32_t)std::min<uint64_t>(b, n);
    }
    bounds[world] = n;
    return MCMC_OK;
}

int mcmc_part_plan(const mcmc_graph* g, uint32_t world, int balance, uint32_t* bounds) {
    if (!g || !bounds) return fail(MCMC_E_ARG, "NULL argument");
    const uint32_t n = g->g.n;
    if (!balance || !g->g.row_off || world == 1) return mcmc_part_plan_rows(n, world, bounds);
    MCMC_HIP_TRY(hipSetDevice(g->g.device));
    std::vector<uint64_t> ro((size_t)n + 1);
    MCMC_HIP_TRY(hipMemcpy(ro.data(), g->g.row_off, sizeof(uint64_t) * ro.size(), hipMemcpyDeviceToHost));
    return mcmc_part_plan_csr(ro.data(), n, world, bounds);
}

namespace {

int check_bounds(uint32_t n, uint32_t world, const uint32_t* bounds) {
    if (!bounds) return fail(MCMC_E_ARG, "NULL bounds");
    if (bounds[0] != 0 || bounds[world] != n) return fail(MCMC_E_ARG, "bounds must run from 0 to n");
    for (uint32_t r = 0; r < world; r++) {
        if (bounds[r] > bounds[r + 1]) return fail(MCMC_E_ARG, "bounds must be ascending");
        if (r > 0 && bounds[r] % kPartAlign && bounds[r] != n)
            return fail(MCMC_E_ARG, "inner bounds must be multiples of 64 rows (mcmc_part_plan)");
    }
    return MCMC_OK;
}

// Partitioned contexts commit events of every rank: room for n of them.
int grow_events(mcmc_ctx* c, uint32_t need) {
    if (c->ev_cap >= need) return MCMC_OK;
    uint32_t pcap = 1;
    while (pcap < need) pcap <<= 1;
    uint32_t *ev = nullptr, *dr = nullptr;
    MCMC_HIP_TRY(hipMalloc(&ev, sizeof(uint32_t) * pcap));
    MCMC_HIP_TRY(hipMalloc(&dr, sizeof(uint32_t) * pcap));
    (void)hipFree(c->events);
    (void)hipFree(c->evdraw);
    c->events = ev;
    c->evdraw = dr;
    c->ev_cap = need;
    return MCMC_OK;
}

}  // namespace

int mcmc_part_attach(mcmc_ctx* c, uint32_t world, uint32_t rank, const uint32_t* bounds, void* colors0,
                     void* colors1, uint64_t colors_bytes, void* foot0, void* foot1, void* stream) {
    if (!c || !colors0 || !colors1 || !foot0 || !foot1) return fail(MCMC_E_ARG, "NULL argument");
    if (world == 0 || world > kMaxWorld || rank >= world) return fail(MCMC_E_ARG, "bad world/rank (1..64 ranks)");
    if (c->variant != 3 && c->variant != 4)
        return fail(MCMC_E_STATE, "partitioned contexts need the tiled (MCMC_GATHER=tiled) or the wide sweep");
    if (int rc = check_bounds(c->n, world, bounds)) return rc;
    if (colors_bytes < ((uint64_t)c->n + 256) * c->cbytes)
        return fail(MCMC_E_ARG, "colour buffers must hold (n + 256) colours");
    if (c->v_begin != bounds[rank] || c->v_end != bounds[rank + 1])
        return fail(MCMC_E_ARG, "context rows must be [bounds[rank], bounds[rank+1])");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    if (int rc = grow_events(c, std::max<uint32_t>(c->n, 64u * 1024u))) return rc;
    c->colors[0] = static_cast<uint8_t*>(colors0);
    c->colors[1] = static_cast<uint8_t*>(colors1);
    c->foot[0] = static_cast<uint32_t*>(foot0);
    c->foot[1] = static_cast<uint32_t*>(foot1);
    c->bounds.assign(bounds, bounds + world + 1);
    c->world = world;
    c->rank = rank;
    c->part = true;
    if (c->dc && c->stream) MCMC_HIP_TRY(dc_reset(c));   // new replicas: the counts are rebuilt
    // the caller's stream as given: 0 is the legacy null stream (torch's default current stream)
    // the context's uploads so far ran on its own (non-blocking) stream: finish them before the
    // caller's stream takes over, or the first sweep could overtake them
    if (c->stream) MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->stream && !c->borrowed_stream) (void)hipStreamDestroy(c->stream);
    c->stream = static_cast<hipStream_t>(stream);
    c->borrowed_stream = true;
    drop_graphs(c);
    return MCMC_OK;
}

int mcmc_part_sweep_async(mcmc_ctx* c) { return part_sweep(c, false); }

int mcmc_part_commit_async(mcmc_ctx* c) { return part_commit(c, 0, nullptr, 0u); }

int mcmc_part_spill_counts(mcmc_ctx* c, uint32_t* counts) {
    if (!c || !c->part || !counts) return fail(MCMC_E_STATE, "partitioned context and counts required");
    DevState h{};
    int rc = download_state(c, &h);
    if (rc) return rc;
    if (!(h.err & kErrSpill)) return fail(MCMC_E_STATE, "no spill exchange pending");
    const uint32_t* f = c->foot[(h.t + 1) & 1];
    for (uint32_t r = 0; r < c->world; r++)
        MCMC_HIP_TRY(hipMemcpyAsync(&counts[r], f + (size_t)r * kFooterWords + 2, sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int mcmc_part_spill_local(mcmc_ctx* c, void* dst, uint32_t* count) {
    if (!c || !c->part || !count) return fail(MCMC_E_ARG, "NULL argument");
    uint32_t cnt[kMaxWorld];
    int rc = mcmc_part_spill_counts(c, cnt);
    if (rc) return rc;
    *count = cnt[c->rank];
    if (dst && *count)
        MCMC_HIP_TRY(hipMemcpyAsync(dst, c->events, sizeof(uint32_t) * *count, hipMemcpyDeviceToDevice, c->stream));
    MCMC_HIP_TRY(hipStreamSynchronize(c->stream));
    return MCMC_OK;
}

int mcmc_part_spill_commit_async(mcmc_ctx* c, const uint32_t* gathered, uint32_t stride) {
    if (!c || !c->part || !gathered) return fail(MCMC_E_ARG, "NULL argument");
    return part_commit(c, 0, gathered, stride);
}

int mcmc_part_attach_delta(mcmc_ctx* c, void* dlt0, void* dlt1) {
    if (!c || !dlt0 || !dlt1) return fail(MCMC_E_ARG, "NULL argument");
    return part_set_delta(c, static_cast<uint32_t*>(dlt0), static_cast<uint32_t*>(dlt1));
}

int mcmc_part_delta_ok(mcmc_ctx* c) { return part_delta_ok(c) ? 1 : 0; }

int mcmc_part_sweep_mode_async(mcmc_ctx* c, int delta) { return part_sweep(c, delta != 0); }

int mcmc_part_commit_mode_async(mcmc_ctx* c, int mode, const uint32_t* gathered, uint32_t stride) {
    if (mode < -1 || mode > 1) return fail(MCMC_E_ARG, "mode: 1 delta, 0 full, -1 full-mode resumption");
    return part_commit(c, mode, gathered, stride);
}

int mcmc_part_sync_remote_async(mcmc_ctx* c) { return part_sync_remote(c); }

int mcmc_part_exchange_stats(mcmc_ctx* c, uint64_t* delta_steps, uint64_t* full_steps, uint64_t* overflows,
                             uint64_t* bytes_sent) {
    if (!c || !c->part) return fail(MCMC_E_STATE, "not a partitioned context");
    if (delta_steps) *delta_steps = c->xs_delta;
    if (full_steps) *full_steps = c->xs_full;
    if (overflows) *overflows = c->xs_ovf;
    if (bytes_sent) *bytes_sent = c->xs_bytes;
    return MCMC_OK;
}

int mcmc_part_state(mcmc_ctx* c, int32_t* done, uint32_t* t, uint32_t* err) {
    if (!c) return fail(MCMC_E_ARG, "NULL context");
    MCMC_HIP_TRY(hipSetDevice(c->g->device));
    DevState h{};
    int rc = download_state(c, &h);
    if (rc) return rc;
    const bool fin = h.done && !(h.err & (kErrSpill | kErrDelta));   // paused for an exchange: not done
    if (done) *done = fin ? 1 : 0;
    if (t) *t = h.t;
    if (err) *err = h.err;
    if (fin) {
        c->last.iter = h.iter;
        c->last.maxIterReached = (int32_t)h.maxIterReached;
        c->last.finalViol = h.finalViol;
        c->last.trajLen = std::min<uint64_t>((uint64_t)h.iter + 1, c->traj_cap);
        c->last.sweepsRun = h.iter + 1;
        c->last.tailcutPasses = c->tail_done ? c->tail_passes : 0u;
        if (c->tail_done) c->last.finalViol = c->tail_viol;
    } else {
        c->last.iter = h.t;
        c->last.trajLen = std::min<uint64_t>(h.t, c->traj_cap);
        c->last.finalViol = ~0ull;
    }
    c->last.glibcDraws = h.glibc_draws;
    c->last.initDraws = c->initDraws;
    for (int i = 0; i < 31; i++) c->glibc.r[i] = h.glibc_ring[(h.glibc_head + i) % 31];
    return MCMC_OK;
}

}  // extern "C"
