/* include/mcmc_hip.h -- C ABI of libmcmc_hip.so, the MI355X-native MCMC colour-resampling sweep.
 *
 * This is the drop-in boundary for the reference's GPU colorer. The reference has no FFI layer;
 * its boundary is the C++ class surface called from src/main.cu:170-202:
 *   ColoringMCMC(Graph* inGraph_d, curandState* randStates, ColoringMCMCParams)
 *                                                      graph_coloring/coloringMCMC.h:47
 *   void ColoringMCMC::run(int iteration)              graph_coloring/coloringMCMC.h:50
 *   void ColoringMCMC::setDirectoryPath(std::string)   graph_coloring/coloringMCMC.h:51
 *   Graph(Graph* host) -- device copy of the CSR        graph/graph.h:100, graphGPU.cu:210-226
 *   GPURand(n, seed)   -- per-vertex RNG states         GPUutils/GPURandomizer.h:42-55
 * Each entry point below names the piece of that surface it replaces. The C++ wrapper
 * (include/mcmc_colorer.hpp) and the Python mirror (mcmc_colorer_amd/) rebuild the class surface
 * on top of these functions.
 *
 * Semantics: results are bit-identical to the reference's --mcmccpu path
 * (graph_coloring/coloringMCMC_CPU.cpp) under the same seed and glibc rand() stream position:
 * same final coloring, same per-sweep conflict counts ("C violations", :152), same sweep count.
 *
 * Conventions: every function returns 0 on success and a negative MCMC_E* code on failure, with a
 * thread-local message in mcmc_last_error(); nothing aborts (the reference prints and aborts,
 * GPUutils/GPUutils.h:20-26 -- the C++ wrapper restores that behaviour). Host arrays belong to the
 * caller and are copied; device buffers belong to the context. A context is not thread-safe.
 */
#ifndef MCMC_HIP_H
#define MCMC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCMC_OK 0
#define MCMC_E_ARG (-1)      /* invalid argument                       */
#define MCMC_E_HIP (-2)      /* HIP runtime error                      */
#define MCMC_E_NOMEM (-3)    /* device or host allocation failed       */
#define MCMC_E_STATE (-4)    /* call out of order / context unusable   */
#define MCMC_E_DEVICE (-5)   /* device-side failure flag (see message) */

typedef struct mcmc_ctx mcmc_ctx;
typedef struct mcmc_graph mcmc_graph;
typedef struct mcmc_gpurand mcmc_gpurand;

/* Mirrors ColoringMCMCParams (graph_coloring/coloring.h:65-74) plus the colorer seed, which the
 * reference passes separately (ColoringMCMC_CPU ctor, coloringMCMC_CPU.h:15; main.cu:171 seed+i). */
typedef struct {
    uint32_t nCol;           /* number of colours; main.cu:162 default maxDeg * numColorRatio       */
    float    epsilon;        /* 1e-8f (main.cu:163)                                                 */
    float    lambda;         /* 1.0f  (main.cu:164; unused by the sweep, kept for the surface)      */
    float    ratioFreezed;   /* 1e-2  (main.cu:165; unused)                                         */
    float    numColorRatio;  /* 1/numColRatio (main.cu:53,161)                                      */
    uint32_t maxRip;         /* 250   (main.cu:166): at most maxRip+1 sweeps (coloringMCMC_CPU.cpp:264-269) */
    uint32_t tabooIteration; /* --tabooIteration (main.cu:167), default 0                           */
    int32_t  tailcut;        /* --tailcut: loop exits when Cviol <= max(50, n/2000) (:89-97)        */
    uint32_t seed;           /* engine seed (std::default_random_engine(seed), :53)                */
} mcmc_params;

/* Per-run summary; the fields the reference writes to its .log (coloringMCMC_CPUutils.cpp:70-102). */
typedef struct {
    uint32_t iter;             /* "Iteration performed"                                          */
    int32_t  maxIterReached;   /* "Max iteration reached"                                        */
    uint64_t finalViol;        /* conflicting vertices of the returned coloring                  */
    uint64_t trajLen;          /* per-sweep Cviol entries kept = min(iter + 1, 2^20) (mcmc_get_trajectory) */
    uint64_t glibcDraws;       /* rand() draws consumed by CDF-overflow events                   */
    uint64_t initDraws;        /* engine draws of the initial coloring (n + rejections)          */
    double   loopMs;           /* device time of the sweep loop (hipEvent)                       */
    uint32_t sweepsRun;        /* sweeps executed (= iter, plus the final count-only pass)       */
    uint32_t tailcutPasses;    /* tail-cut passes run after the loop (mcmc_set_tailcut_repair)   */
} mcmc_run_stats;

const char* mcmc_last_error(void);
int mcmc_version(void);

/* ---- glibc rand() stream (the process-global stream the reference shares between setupRnd2
 *      (graphCPU.cpp:308) and the overflow fallback (coloringMCMC_CPU.cpp:518)) ---------------
 * A position is the 31-word window of glibc TYPE_3 state. srand(seed) followed by `draws` calls
 * of rand(); jumps in O(31^2 log draws). Replaces nothing in the reference (it used the libc
 * global); needed because the GPU replays the reference's exact rand() draws. */
int mcmc_glibc_window(uint32_t seed, uint64_t draws, uint32_t window[31]);
int mcmc_glibc_draw(uint32_t window[31], uint32_t count, uint32_t* out); /* advances window */

/* ---- Graph: Graph(Graph* host) device copy (graph/graph.h:100, graphGPU.cu:210-226) -------- */
/* Copies a host CSR (uint64 offsets: the reference's uint32 node_sz overflows beyond 2^32 arcs,
 * graph.h:19-20) to the device. */
int mcmc_graph_upload(const uint64_t* row_off, const uint32_t* col_idx, uint32_t n, uint64_t m,
                      int device, mcmc_graph** out);
/* Graph(n, prob, seed) -> setupRnd2 (graphCPU.cpp:291-404) generated ON the device, bit-exact:
 * the n(n+1)/2 glibc draws start at `window` (advanced on return, as the reference's global
 * stream is). Neighbour lists ascending, as the reference's. */
int mcmc_graph_simulate(uint32_t n, float prob, uint32_t window[31], int device, mcmc_graph** out);
/* Fast Erdos-Renyi G(n,p) for sizes where the reference's O(n^2) setupRnd2 is infeasible
 * (not the reference's graph): counter-based Philox4x32-10 streams with
 * geometric skips, fully defined in mcmc_colorer_amd/csrc/er_gen.h (p is used as (double)(float)).
 * The graph is written straight into the sweep's tiled layout -- no CSR is materialised (C3's
 * would be 400 GB) -- so the handle serves mcmc_create and mcmc_graph_info; mcmc_graph_download
 * reconstructs a CSR (small graphs), mcmc_graph_device_ptrs fails. _part generates only the rows
 * rank `rank` of `world` owns under mcmc_part_plan_rows, for a partitioned run; its m counts those
 * rows' arcs. */
int mcmc_graph_er_fast(uint32_t n, double prob, uint64_t seed, int device, mcmc_graph** out);
int mcmc_graph_er_fast_part(uint32_t n, double prob, uint64_t seed, uint32_t world, uint32_t rank, int device,
                            mcmc_graph** out);
/* Rows [v_begin, v_end) only (any partition plan's range). */
int mcmc_graph_er_fast_rows(uint32_t n, double prob, uint64_t seed, uint32_t v_begin, uint32_t v_end, int device,
                            mcmc_graph** out);
/* The CSR (uint64 offsets, uint32 ids; rows in layout order, not sorted) of a graph generated with
 * mcmc_graph_er_fast(_rows / _part), built on the device from its tiled layout and kept on the
 * handle (then mcmc_graph_device_ptrs works; a row-partial graph's rows outside its range are
 * empty). For the refstruct baseline at full occupancy (bench.py); mcmc_create calls it for
 * nCol > 256 (the wide sweep scans a CSR). MCMC_E_NOMEM with the byte counts when it does not fit. */
int mcmc_graph_materialize_csr(mcmc_graph* g);
/* R-MAT power-law graph (configs[4] stand-in: SNAP LiveJournal / Reddit are not available; SURVEY.md
 * §8d C5), generated on the device as a CSR with ascending neighbour lists: 2^scale vertices,
 * edge_factor * 2^scale Philox-driven quadrant draws with probabilities (a, b, c, 1-a-b-c), ids
 * scrambled by a fixed bijection, self-loops dropped, both arcs kept, duplicates merged. Fully
 * defined in mcmc_colorer_amd/csrc/er_gen.h (rmat_edge). Not a reference graph. */
int mcmc_graph_rmat(uint32_t scale, uint32_t edge_factor, double a, double b, double c, uint64_t seed, int device,
                    mcmc_graph** out);
int mcmc_graph_info(const mcmc_graph* g, uint32_t* n, uint64_t* m, uint32_t* maxDeg, uint32_t* minDeg);
/* Test hook (no reference counterpart): rows of a graph as stored on the device -- the full-range
 * tiled layout of a generated graph, or the CSR. off: [k+1]; ids: NULL for the degrees only, else
 * cap >= off[k] entries (each row's ids in layout order); pos: optional [k], the layout index
 * (uint64) of each row's first stored id. Lets tests check rows of graphs too large to download. */
int mcmc_graph_rows(const mcmc_graph* g, const uint32_t* rows, uint32_t k, uint64_t* off, uint32_t* ids,
                    uint64_t cap, uint64_t* pos);
/* Device pointers (row_off: uint64[n+1], col_idx: uint32[m]) for zero-copy callers. */
int mcmc_graph_device_ptrs(const mcmc_graph* g, const uint64_t** row_off, const uint32_t** col_idx);
int mcmc_graph_download(const mcmc_graph* g, uint64_t* row_off, uint32_t* col_idx);
void mcmc_graph_destroy(mcmc_graph* g);

/* ---- Colorer: ColoringMCMC(Graph*, curandState*, ColoringMCMCParams) (coloringMCMC.h:47) ---- */
/* Rows [v_begin, v_end) are swept by this context (the whole graph: 0, n). Colour replicas are
 * always full-length, so a vertex-partitioned multi-GPU run keeps global ids. The context
 * borrows `g` (it must outlive the context). */
int mcmc_create(const mcmc_graph* g, const mcmc_params* p, uint32_t v_begin, uint32_t v_end,
                mcmc_ctx** out);
/* Position of the glibc stream the overflow fallback draws from (default: srand(1), no draws). */
int mcmc_set_glibc_window(mcmc_ctx* c, const uint32_t window[31]);
int mcmc_get_glibc_window(mcmc_ctx* c, uint32_t window[31]);
/* ColoringMCMC_CPU ctor colouring (coloringMCMC_CPU.cpp:53-61): C[v] = uniform_int(0, nCol-1)
 * from std::default_random_engine(seed) in vertex order, or the caller's C0 if non-NULL. */
int mcmc_init_coloring(mcmc_ctx* c, const uint32_t* C0);
/* run() main loop (coloringMCMC_CPU.cpp:127-270) on the device: sweeps until Cviol <= z or the
 * maxRip cap. max_sweeps > 0 stops early after that many sweeps (bounded samples). */
int mcmc_run(mcmc_ctx* c, uint32_t max_sweeps, mcmc_run_stats* stats);
/* Tail cutting after the loop (coloringMCMC_CPU.cpp:272-311) with the inner loop's k++ fix (the
 * reference increments i at :289 and never returns): colorIdx sorted by ascending colour histogram
 * when z > 0; then, while Cviol > 0 and at most max_passes times, every flagged vertex in ascending
 * order takes the first colour of colorIdx free among its neighbours, and Cviol is recounted. The
 * first pass visits the vertices flagged in the colouring before the last accepted sweep, as the
 * reference's (unswapped) Cviols does. Call before mcmc_run; mcmc_run then reports the repaired
 * Cviol in finalViol and the passes in tailcutPasses (the trajectory is the loop's). 0 disables.
 * Whole-graph contexts only; costs n bytes of flag writes per sweep while enabled. */
int mcmc_set_tailcut_repair(mcmc_ctx* c, uint32_t max_passes);
/* Test hook: conflicting vertices of the current colouring (violation_count, coloringMCMC_CPU.cpp:
 * 329-351) recounted by the tail cut's kernel, independently of the sweep's own count; flags
 * (optional, n bytes) receives the per-vertex flags. */
int mcmc_count_violations(mcmc_ctx* c, uint64_t* count, uint8_t* flags /* nullable, n bytes */);
int mcmc_get_coloring(mcmc_ctx* c, uint32_t* out /* n */);
int mcmc_get_trajectory(mcmc_ctx* c, uint64_t* out, uint64_t cap, uint64_t* len);
/* Timed throughput mode for benchmarks: exactly `sweeps` sweeps of the loop body (no
 * convergence exit, no cap), captured into one hipGraph and timed with hipEvents on the sweep
 * stream. total_ms = device wall of the loop; sweep_kernel_ms = total / sweeps = average duration
 * of one launch of the (fused) sweep kernel, inter-launch gap included. */
int mcmc_bench_sweeps(mcmc_ctx* c, uint32_t sweeps, double* total_ms, double* sweep_kernel_ms);
/* Captures and uploads the `sweeps`-launch graph ahead of mcmc_bench_sweeps (keeps graph
 * instantiation out of a host-timed region). */
int mcmc_bench_prepare(mcmc_ctx* c, uint32_t sweeps);
/* Throughput mode for any context (partitioned ones included): sweeps never stop on convergence
 * (Cviol <= z), so a timed run of a convergent configuration still resamples every vertex each
 * sweep; lift the cap with a large maxRip. The trajectory keeps at most 2^20 entries. */
int mcmc_set_bench_mode(mcmc_ctx* c, int on);
/* The dense-count sweep of a tiled context (csrc/dense_counts.h; on unless MCMC_DENSE=0 or the graph
 * is not simple and symmetric): out = {on, dense range begin, end, incremental sweeps, count
 * rebuilds, vertices of the range moved by updates, rows that scanned beyond the range, the update
 * list's rebuild threshold, local rows that changed colour (the restore lists; a list past its
 * capacity counts as its capacity), sweeps whose restore list overflowed}; all 0 when off. */
int mcmc_get_dense_stats(mcmc_ctx* c, uint64_t out[10]);
/* The same plus the persistent dense sweep (csrc/dense_sparse.h): out[10] sweeps the leader ran
 * alone (solo), out[11] candidate-window states, out[12] 1 if the context launches it, out[13] open
 * mask words now nonzero, out[14] rows the solo sweeps evaluated. Test / bench statistics. */
int mcmc_get_dense_stats_v2(mcmc_ctx* c, uint64_t out[16]);
/* The dense-count sweep's per-row state of local rows [row0, row0 + rows): counts[rows][nCol] (the
 * neighbours in the dense column range S per colour, as of the last sweep's update) and, if masks
 * is not NULL, masks[rows][mask words] (their occupancy bits). Test / diagnostic read-back. */
int mcmc_get_dense_counts(mcmc_ctx* c, uint32_t row0, uint32_t rows, uint32_t* counts, uint32_t* masks);
/* Diagnostics of the tiled sweep's scan (no reference counterpart): with stats on, every sweep adds
 * the 16-byte id quads it loaded and the (group, column block) pairs it staged (table + colour
 * slice); mcmc_set_scan_stats(c, 1) also zeroes them. The sweep stops scanning a row once its
 * occupancy mask holds every colour (count_free_colors cannot change: results are unchanged);
 * MCMC_FULL_SCAN=1 in the environment at mcmc_create scans every arc instead. */
int mcmc_set_scan_stats(mcmc_ctx* c, int on);
int mcmc_get_scan_stats(mcmc_ctx* c, uint64_t* quads, uint64_t* pairs);
/* The same counters plus `used` (may be NULL): the quads whose ids the scan gathered. `quads` also
 * counts loads issued ahead for a row that filled up before they were needed (the scan keeps two
 * steps in flight), so `used` is the bytes the exact early exit needs, `quads` what it issued. */
int mcmc_get_scan_stats_ex(mcmc_ctx* c, uint64_t* quads, uint64_t* used, uint64_t* pairs);
/* All counters: [0] quads loaded, [1] pairs (a segment table each), [2] quads gathered, [3] colour
 * slices staged (the tail queue's resident dense slices and its blocks included), [4] / [5] tail-queue
 * entries written / read (16 B each, plus a row's 8 B segment bounds and 8 B group base per read). */
int mcmc_get_scan_stats_v2(mcmc_ctx* c, uint64_t out[6]);
/* The wide sweep's incremental violation counts (no reference counterpart; the reference recounts
 * every row each sweep, coloringMCMC_CPU.cpp:329-351): [0] 1 if the context keeps them (a whole-graph
 * context over a symmetric CSR without repeated arcs, nCol > 256), then since mcmc_init_coloring
 * [1] sweeps that moved the counts by the rows that changed, [2] full recounts, [3] rows that
 * changed colour, [4] their arcs. Results are the same either way; MCMC_WIDE_INC=0 at mcmc_create
 * turns it off. */
int mcmc_get_wide_inc_stats(mcmc_ctx* c, uint64_t out[5]);
/* The persistent wide sweep for nearly proper colourings (csrc/wide_solo.h; no reference
 * counterpart -- the same sweeps as the per-sweep path, bit for bit): [0] 1 if the context runs it
 * (whole graph, incremental counts, eps > 0, no taboo; MCMC_WIDE_SOLO=0 at mcmc_create: off),
 * [1] candidate-window states, then cumulative [2] sweeps it ran, [3] phases it handed to the
 * grid, [4] violators its leader walked, [5] walk phases, [6] count-move phases, [7] violator
 * collections, [8] candidate rows evaluated, [9] rows that changed colour; diagnostics [10] the
 * watchdog word (nonzero: a phase never completed, the run failed), [11] / [12] the leader's last
 * sweep of a launch and its step, [13] the phase flag word, [14..21] wall-clock ticks (100 MHz) of
 * its sweeps' steps: walks, candidates, walk wait, events, changed rows, count moves, violator
 * list, whole sweeps; [22..29] finer probes of those steps (diagnostics). */
int mcmc_get_wide_solo_stats(mcmc_ctx* c, uint64_t out[30]);

/* Test hook (no reference counterpart): the wide sweep's exact fp32 CDF walk (csrc/cdf_walk.h,
 * extract_new_color coloringMCMC_CPU.cpp:505-520 over runs of equal p) evaluated on the host.
 * mask == NULL: fill_p's own-colour distribution (cases (i)/(iii): p[cv] = p, eps elsewhere);
 * else case (ii): eps where a bit of mask (nCol bits, 32 per word) is set, p where clear.
 * Returns the drawn colour, or nCol for a CDF overflow. */
uint32_t mcmc_cdf_walk(const uint32_t* mask, uint32_t nCol, uint32_t cv, float eps, float p, float u);

/* Sweep kernel and adjacency layout a context chose (no reference counterpart: the reference's
 * sweep has one fixed CSR layout). sweep_bytes = B_fmt of SURVEY.md §8d, the HBM bytes one sweep
 * of this context's rows must move in its layout (adjacency + offsets/segment tables + colour
 * replica read once + local colour write [+ taboo r/w]); ref_bytes = the same rows' B_alg in the
 * reference's uint32 layout (4(n+1) + 4m + 4n + 4n [+ 8n]). */
typedef struct mcmc_ctx_info {
    int32_t variant;          /* 0 LDS-staged CSR, 1 column-blocked CSR, 2 L2-gather CSR, 3 tiled,
                                 4 wide (nCol > 256: uint16 replicas, CSR) */
    int32_t resident;         /* tiled: whole colour replica LDS-resident (else streamed slices) */
    uint32_t block_log2;      /* tiled / blocked: column block = 2^block_log2 vertices */
    uint32_t nblocks;
    uint32_t grp_rows;        /* tiled: rows per group */
    uint32_t ngroups;
    uint32_t sub_log2;        /* tiled: lanes per row segment = 2^sub_log2 */
    uint32_t grid, block;     /* sweep launch geometry */
    uint32_t reserved;
    uint64_t lds_bytes;       /* dynamic LDS per workgroup */
    uint64_t layout_bytes;    /* device bytes of the adjacency layout the sweep streams */
    uint64_t sweep_bytes;     /* B_fmt per sweep */
    uint64_t ref_bytes;       /* B_alg per sweep, reference uint32 layout */
} mcmc_ctx_info;
int mcmc_get_info(mcmc_ctx* c, mcmc_ctx_info* out);
void mcmc_destroy(mcmc_ctx* c);

/* ---- measurement baseline (not part of the colouring path) ----------------------------------
 * "refstruct" (SURVEY.md §8d): the reference CUDA path's per-sweep structure re-expressed in HIP --
 * thread-per-vertex serial row walks in 64-thread blocks, an n*nCol byte checker reset per sweep, two
 * edge-conflict passes with host-side sums, a 4n-byte D2H + host histogram + H2D per sweep
 * (coloringMCMC_main.cu:168-262, coloringMCMC_utils.cu:103-198, coloringMCMC_balance.cu:79-143).
 * Runs `sweeps` sweeps of it on `g` and returns the host wall time per sweep. Its colouring follows
 * the reference GPU semantics (XORWOW draws), so it is timed, never compared. */
int mcmc_refstruct_bench(const mcmc_graph* g, uint32_t nCol, uint32_t sweeps, uint32_t seed,
                         double* ms_per_sweep, uint64_t* conflicts);

/* ---- vertex-partitioned multi-GPU run -----------------------------------------
 * Rank r of `world` sweeps rows [bounds[r], bounds[r+1]) with global ids, full-length colour
 * replicas in vertex order (C_t in colors[t & 1], 1 byte per colour, 2 for the wide sweep: nCol >
 * 256, mcmc_color_bytes) and a replicated glibc window. Per sweep t, on the rank's stream, no host
 * sync:
 *   mcmc_part_sweep_async   sweep of the local rows into colors[(t+1)&1] and this rank's footer slot
 *                           (MCMC_FOOTER_WORDS uint32 at foot[(t+1)&1] + rank * MCMC_FOOTER_WORDS:
 *                           local Cviol, event count, flags, sorted overflow events)
 *   exchange                every rank's rows [bounds[r], bounds[r+1]) of colors[(t+1)&1] and its
 *                           footer slot of foot[(t+1)&1] to every rank (mcmc_part_run does it over
 *                           RCCL; a caller may do it itself)
 *   mcmc_part_commit_async  global Cviol, stop test, the rank-ordered glibc replay -- identical on
 *                           every replica -- RNG advance, buffer flip
 * A rank whose overflow events of a sweep outgrow its footer (> MCMC_FOOTER_WORDS - 4) pauses the
 * loop at that sweep on every rank (mcmc_part_state: err bit 1, done 0): the driver all-gathers
 * the full sorted lists (mcmc_part_spill_local / _counts) with a common stride and resumes with
 * mcmc_part_spill_commit_async. Plans: inner bounds are multiples of 64 rows. */
#define MCMC_FOOTER_WORDS 1024
#define MCMC_COMM_ID_BYTES 128
typedef struct mcmc_comm mcmc_comm;
/* Equal row ranges (ceil(n/world) rounded up to 64). */
int mcmc_part_plan_rows(uint32_t n, uint32_t world, uint32_t* bounds /* world + 1 */);
/* balance 0: equal rows; 1: arc-balanced -- each rank gets ~1/world of sum(deg(v) + 16) from the
 * CSR's degree prefix (power-law graphs whose hubs cluster in id ranges, configs[4]). Graphs without
 * a CSR (the generator's per-rank layouts; G(n,p) is uniform) get equal rows. */
int mcmc_part_plan(const mcmc_graph* g, uint32_t world, int balance, uint32_t* bounds /* world + 1 */);
/* The arc-balanced plan from a host CSR's offsets (row_off[n + 1]). */
int mcmc_part_plan_csr(const uint64_t* row_off, uint32_t n, uint32_t world, uint32_t* bounds /* world + 1 */);
uint32_t mcmc_color_bytes(uint32_t nCol);
/* Caller-exchanged contexts: a context on rows [bounds[rank], bounds[rank+1]) (mcmc_create) is
 * attached to caller-owned device buffers: colour replicas of >= (n + 256) * mcmc_color_bytes(nCol)
 * bytes and footer buffers of world * MCMC_FOOTER_WORDS uint32; `stream` is the caller's
 * hipStream_t, used as given (0 = the legacy null stream). */
int mcmc_part_attach(mcmc_ctx* c, uint32_t world, uint32_t rank, const uint32_t* bounds, void* colors0,
                     void* colors1, uint64_t colors_bytes, void* foot0, void* foot1, void* stream);
int mcmc_part_sweep_async(mcmc_ctx* c);
int mcmc_part_commit_async(mcmc_ctx* c);
/* Synchronises the stream; *done = 1 once the loop is over (colouring/trajectory then final);
 * *err: bit 0 a fatal device error, bit 1 a spill exchange is pending, bit 2 a delta slot overflowed
 * (then *t is the paused sweep). */
int mcmc_part_state(mcmc_ctx* c, int32_t* done, uint32_t* t, uint32_t* err);
/* Spill exchange of a paused sweep: every rank's list length (from the exchanged footers), this
 * rank's sorted list copied to device memory dst (NULL: the count only), and the resumption from
 * the gathered lists (rank r's list at gathered[r * stride], device memory, stride >= every count). */
int mcmc_part_spill_counts(mcmc_ctx* c, uint32_t* counts /* world */);
int mcmc_part_spill_local(mcmc_ctx* c, void* dst, uint32_t* count);
int mcmc_part_spill_commit_async(mcmc_ctx* c, const uint32_t* gathered, uint32_t stride);
/* Delta exchange (what mcmc_part_run does by default at world > 1): a step sends, instead of the
 * rank's rows, its delta slot -- MCMC_DELTA_WORDS uint32 at dlt[(t+1)&1] + rank * MCMC_DELTA_WORDS:
 * [0] pairs appended (may exceed the slot's (MCMC_DELTA_WORDS - 2) / 2), [1] 0, then (vertex, colour)
 * pairs of the rank's vertices whose colour changed (overflow events excepted: every rank replays
 * them). The commit applies every other rank's pairs to BOTH replicas, so outside its own rows a
 * rank's replicas stay equal; after full-mode steps (or at a run's start) mcmc_part_sync_remote_async
 * restores that before the next delta step. A slot that overflowed pauses the sweep on every rank
 * (mcmc_part_state err bit 2): exchange its rows as in full mode, then resume with mode -1 (and the
 * gathered lists if err bit 1 is set too). dlt0/dlt1: caller-owned device buffers of world *
 * MCMC_DELTA_WORDS uint32 each (mcmc_part_create's contexts own theirs). Tiled sweeps only (nCol <=
 * 256): mcmc_part_delta_ok. Modes of mcmc_part_commit_mode_async: 1 delta, 0 full, -1 full-mode
 * resumption of a paused sweep (gathered/stride as mcmc_part_spill_commit_async, or NULL/0). */
#define MCMC_DELTA_WORDS 4096
int mcmc_part_attach_delta(mcmc_ctx* c, void* dlt0, void* dlt1);
int mcmc_part_delta_ok(mcmc_ctx* c);
int mcmc_part_sweep_mode_async(mcmc_ctx* c, int delta);
int mcmc_part_commit_mode_async(mcmc_ctx* c, int mode, const uint32_t* gathered, uint32_t stride);
int mcmc_part_sync_remote_async(mcmc_ctx* c);
/* Exchange statistics of the context's last mcmc_part_run: steps exchanged in delta and in full
 * mode, delta-slot overflows (paused sweeps), and the bytes this rank sent to its peers. */
int mcmc_part_exchange_stats(mcmc_ctx* c, uint64_t* delta_steps, uint64_t* full_steps, uint64_t* overflows,
                             uint64_t* bytes_sent);

/* Native runs (csrc/multi.hip): RCCL communicators behind the ABI. One process per GPU:
 * rank 0 calls mcmc_comm_unique_id and hands the bytes to the others (any channel), every rank
 * mcmc_comm_init_rank; one process driving N GPUs: mcmc_comm_init_all. */
int mcmc_comm_unique_id(uint8_t id[MCMC_COMM_ID_BYTES]);
int mcmc_comm_init_rank(const uint8_t id[MCMC_COMM_ID_BYTES], uint32_t world, uint32_t rank, int device,
                        mcmc_comm** out);
int mcmc_comm_init_all(const int* devices, uint32_t ndev, mcmc_comm** out /* ndev */);
void mcmc_comm_destroy(mcmc_comm* c);
/* A partitioned context that owns its buffers and stream (rows [bounds[rank], bounds[rank+1]) of
 * `g`, which must hold them: the whole CSR, or mcmc_graph_er_fast_rows of that range). comm NULL:
 * the loopback transport -- every rank of the world in this process, exchanged by device copies
 * (tests; several ranks may share a GPU). Initialise with mcmc_set_glibc_window +
 * mcmc_init_coloring as a single context; destroy with mcmc_destroy. */
int mcmc_part_create(const mcmc_graph* g, const mcmc_params* p, uint32_t world, uint32_t rank, const uint32_t* bounds,
                     mcmc_comm* comm, mcmc_ctx** out);
/* run() (coloringMCMC_CPU.cpp:115-270) of this process's k ranks (k = 1: one process per GPU;
 * k = world: one process driving them all, or the loopback transport) inside one call: sweeps,
 * exchanges, commits, spill exchanges, until the loop stops (max_sweeps > 0: at most that many).
 * stats: k entries (identical loop fields on every rank; loopMs = device time on ctxs[0]'s stream).
 * Colourings and trajectories then come from mcmc_get_coloring / mcmc_get_trajectory of any rank. */
int mcmc_part_run(mcmc_ctx** ctxs, uint32_t k, uint32_t max_sweeps, mcmc_run_stats* stats /* k */);
/* Measurement only: `steps` steps of ONE rank of a loopback partition (comm NULL) through the same
 * driver as mcmc_part_run -- sweep, delta packing, commit launch, batches and polling -- with the
 * exchange left out (the peers' footers and delta slots stay empty). What one GPU can time of a
 * world-N step; the colouring it leaves is not the partitioned run's. */
int mcmc_part_bench_rank(mcmc_ctx* c, uint32_t steps, mcmc_run_stats* stats);

/* ---- other colorers -------------------------------------------------
 * The reference's parallel greedy first-fit colorer (ColoringGreedyFF::run,
 * graph_coloring/coloringGreedyFF.cu:50-84, `--grdffgpu`): Jacobi rounds of a tentative first fit
 * (each uncoloured node's forbidden set gains its neighbours' colours and is never cleared; the
 * first colour i >= 1, i <= maxDeg, not forbidden; node 0 always 1) and a conflict pass (the
 * larger id of a same-coloured pair is uncoloured) until every node is coloured. Deterministic.
 * colors: n host words, 1-based; num_colors = distinct colours; rounds = loop iterations. */
int mcmc_greedyff_run(const mcmc_graph* g, uint32_t* colors, uint32_t* num_colors, uint32_t* rounds);
/* The reference's greedy colorer followed by its rebalancing (ColoringVFF::run,
 * graph_coloring/coloringVFF.cu:50-228, `--vffgpu`): the GreedyFF rounds, then iterations in which
 * every unbalanced node (its colour's bin holds more than gamma = n / numColors nodes) other than
 * node 0 moves to the first colour not used by itself or a neighbour whose bin holds MORE than
 * gamma nodes (the reference's test, as written), bins are recounted, and a node stays unbalanced
 * only while a neighbour of smaller id shares its new colour; until none is unbalanced or the
 * unbalanced set repeats for nine snapshots (ensure_not_looping; then the result is the greedy
 * colouring and *valid = 0). colors: n host words, 1..numColors; iterations = rebalancing
 * iterations. Greedy colours that are not 1..numColors (the reference reads past its bins) and a
 * cycle the history misses (the reference spins) return MCMC_E_DEVICE. */
int mcmc_vff_run(const mcmc_graph* g, uint32_t* colors, uint32_t* num_colors, uint32_t* iterations, int* valid);
/* The reference's Luby colorer (ColoringLuby::run_fast, graph_coloring/coloringLubyFast.cu:21-174,
 * `--lubygpu`): one colour per outer round, built as an independent set by inner rounds in which
 * every node draws curand_uniform from its XORWOW state in `rand` (advanced in place, as the
 * reference's GPURand states are: set_initial_distr_k, coloringLuby.cu:232-243), candidates with
 * u < 0.5 are selected, a selected node with a selected neighbour of degree >= its own is dropped
 * (check_conflicts_fast_k :121-148, on the round's snapshot: the reference's in-place version is
 * timing-dependent, this is its every-read-before-any-write schedule), and the survivors and their
 * neighbours leave the candidates (update_eligible_fast_k :150-168). colors: n host words, 1..k;
 * num_colors = k; rounds = inner rounds. A node that can never survive (self loop) makes the
 * reference spin; this returns MCMC_E_DEVICE ("no progress") instead. */
int mcmc_luby_run(const mcmc_graph* g, mcmc_gpurand* rand, uint32_t* colors, uint32_t* num_colors,
                  uint32_t* rounds);

/* ---- reference-GPU-semantics mode ------------------------------------
 * The per-vertex cuRAND XORWOW states of the reference's GPURand (GPUutils/GPURandomizer.cu:8-13,
 * 85-101: curand_init(seed, v, 0) for every vertex v), shared by all repetitions (main.cu:80,193).
 * mcmc_xorwow_state: host probe of one state, {v0..v4, d}; flavor 0 = cuRAND's salts, 1 = rocRAND's
 * (the tests pin the transition and the 2^67 subsequence jump against rocRAND's engine). */
int mcmc_xorwow_state(uint64_t seed, uint64_t subsequence, int flavor, uint32_t out[6]);
int mcmc_gpurand_create(uint32_t n, uint32_t seed, int device, mcmc_gpurand** out);
int mcmc_gpurand_states(const mcmc_gpurand* r, uint32_t* out /* [n][6] */);
void mcmc_gpurand_destroy(mcmc_gpurand* r);
/* The reference's own --mcmcgpu colorer: ColoringMCMC as built by default (coloringMCMC.h:22-41:
 * COLOR_BALANCE_DYNAMIC_DISTR, STANDARD_INIT, TABOO), on the tiled sweep. Per sweep: conflicts
 * counted as edges (conflictCounter + calcConflicts, coloringMCMC_utils.cu:103-119,184-198), the
 * loop stops when they are <= z (do/while, coloringMCMC_main.cu:160-269, at most maxRip sweeps),
 * proposal selectStarColoringBalanceDynamic (coloringMCMC_balance.cu:79-143) with one XORWOW
 * draw per updated vertex. mcmc_ref_run initialises the colouring from `rand` (initColoring,
 * coloringMCMC_utils.cu:24-33), runs, then -- if params.tailcut -- the GPU tail cut
 * (coloringMCMC_main.cu:271-290) for at most tail_max_passes passes (the reference's is unbounded).
 * Stats: iter = rip, maxIterReached = (rip == maxRip), finalViol = conflicting EDGES of the
 * returned colouring, sweepsRun = sweeps, trajLen = counts of C_0 .. C_last (mcmc_get_trajectory).
 * The states advance as the reference's do; repetitions pass the same `rand`. 2 <= nCol <= 65535
 * (nCol > 255: uint16 replicas over the CSR, csrc/ref_wide.h).
 * Parity unpinned against CUDA. */
int mcmc_ref_create(const mcmc_graph* g, const mcmc_params* p, mcmc_gpurand* rand, mcmc_ctx** out);
int mcmc_ref_run(mcmc_ctx* c, uint32_t tail_max_passes, mcmc_run_stats* stats);
/* The run's initialisation alone (initial colouring from `rand`, cleared taboo and histograms):
 * then mcmc_bench_sweeps times sweeps of this semantics. */
int mcmc_ref_init(mcmc_ctx* c);
/* cudaMemGetInfo's pair for the GPU colorer's log header (coloringMCMC_prints.cu:20-22). */
int mcmc_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes);
/* HIP_VERSION the library was compiled against, and hipRuntimeGetVersion of the runtime it is bound
 * to in this process (torch's bundled runtime when torch is loaded: the majors must agree). */
int mcmc_hip_versions(int* built, int* runtime);
/* Cviol (REF: conflicting edges) after each tail-cut pass of the last run. */
int mcmc_get_tail_trajectory(mcmc_ctx* c, uint64_t* out, uint64_t cap, uint64_t* len);

#ifdef __cplusplus
}
#endif
#endif /* MCMC_HIP_H */
