// oracle/mcmc_cpu_ref.h -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
//
// CPU restatement of the reference's `--mcmccpu` path, written from the source text of
//   src/graph_coloring/coloringMCMC_CPU.{h,cpp}   (ColoringMCMC_CPU)
//   src/graph/graphCPU.cpp:291-404                 (Graph::setupRnd2, the --simulate generator)
//   src/graph/graphCPU.cpp:433-450                 (Graph::doStats -> maxDeg)
//   src/main.cu:160-171                            (ColoringMCMCParams defaults, seed+i per repetition)
// It calls the SAME third-party arithmetic the reference calls: libstdc++ <random>
// (std::default_random_engine = minstd_rand0, uniform_int_distribution<uint32_t>,
// uniform_real_distribution<float>) and glibc rand().
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
// The product (mcmc_colorer_amd/) never links or calls it.
//
// Parity status: the reference ships no tests or golden vectors and executing
// it here was refused, so this restatement is pinned by standard KATs
// (C++ [rand.predef], glibc rand()) and by a second, independent numpy restatement
// (oracle/oracle_np.py) on small graphs -- see DESIGN.md "Oracle".
#pragma once
#include <cstdint>
#include <cstddef>

extern "C" {

typedef struct {
    uint32_t nCol;            // ColoringMCMCParams::nCol          (coloring.h:65-74)
    float    epsilon;         // 1e-8f                              (main.cu:163)
    float    lambda;          // 1.0f (unused by the CPU path)      (main.cu:164)
    float    ratioFreezed;    // 1e-2 (unused)                      (main.cu:165)
    float    numColorRatio;   // 1/numColRatio                      (main.cu:53,161)
    uint32_t maxRip;          // 250                                (main.cu:166)
    uint32_t tabooIteration;  // --tabooIteration, default 0        (main.cu:167)
    int32_t  tailcut;         // --tailcut                          (main.cu:168)
    int32_t  tailcutRepair;   // 0: stop and report when Cviol > 0 at loop exit (the reference
                              //    hangs there: coloringMCMC_CPU.cpp:296 increments i, not k);
                              // 1: run the tail cut with that one bug fixed, bounded passes
} oracle_params;

typedef struct {
    uint32_t iter;              // ColoringMCMC_CPU::iter at loop exit ("Iteration performed")
    int32_t  maxIterReached;    // loop left through the maxRip cap
    uint64_t finalViol;         // Cviol at loop exit (vertices with a same-colored neighbour)
    uint64_t trajLen;           // entries written to traj (= iter + 1 when not truncated)
    uint64_t glibcDraws;        // rand() calls made by overflow events during run()
    uint64_t initDraws;         // engine draws consumed by the initial coloring (K0 = n + rejections)
    double   loopSeconds;       // steady_clock wall time of the sweep loop
    uint32_t sweepsRun;         // sweeps actually executed
    uint32_t tailcutPasses;     // tail-cut passes executed (bounded; the reference loops forever)
} oracle_result;

// ---- glibc rand() stream (the process-global one the reference uses) ----
void     oracle_srand(uint32_t seed);
int32_t  oracle_rand(void);
void     oracle_rand_skip(uint64_t k);
// Points glibc's rand() at a given TYPE_3 window (31 words, oldest first) by initstate() on a
// static buffer and writing the words where glibc's fptr/rptr expect them. Lets the oracle run
// from a stream position reached by jump-ahead instead of ~n^2/2 sequential rand() calls.
void     oracle_set_glibc_window(const uint32_t window[31]);

// ---- libstdc++ <random> probes (for RNG known-answer tests) ----
void     oracle_minstd_seq(uint32_t seed, uint64_t count, uint32_t* out);
void     oracle_canonical_seq(uint32_t seed, uint64_t skip, uint64_t count, float* out);
uint64_t oracle_uniform_int_seq(uint32_t seed, uint32_t nCol, uint64_t count, uint32_t* out);

// ---- graph: Graph(n, prob, seed) -> setupRnd2 (graphCPU.cpp:291-404) ----
// Consumes n(n+1)/2 glibc rand() draws from the current process stream.
// Allocates *row_off (n+1) and *col_idx (m) with malloc; free with oracle_free.
int      oracle_setup_rnd2(uint32_t n, float prob, uint64_t** row_off, uint32_t** col_idx, uint64_t* m);
uint32_t oracle_max_deg(uint32_t n, const uint64_t* row_off);

// ---- graph: the build's counter-based G(n, p) for C3/C4-scale runs (NOT a reference function;
// "the build's documented GPU ER generator ... parity is GPU-vs-restatement on the
// same graph"). Restated from the definition in mcmc_colorer_amd/csrc/er_gen.h: Philox4x32-10
// streams per (row i, 65536-column block Y >= i's block), geometric skips
// 1 + floor(ln(u) / log1p(-p)), u = (x + 1) / 2^32, ln by the same +-*/ series.
// Rows ascending. Allocates like oracle_setup_rnd2.
int      oracle_er_fast(uint32_t n, double prob, uint64_t seed, uint64_t** row_off, uint32_t** col_idx, uint64_t* m);
// Neighbour lists (ascending) of selected rows of that graph, without enumerating the whole of it:
// the C3 graph (1e11 arcs) checked row by row. *row_off: [k + 1], rows in the given order.
int      oracle_er_rows(uint32_t n, double prob, uint64_t seed, const uint32_t* rows, uint32_t k, int nthreads,
                        uint64_t** row_off, uint32_t** col_idx);
void     oracle_free(void* p);

// ---- per-vertex pieces for sampled checks at sizes where the whole run cannot be restated ----
// u of engine draw pos[i] (1-based) of default_random_engine(seed) (coloringMCMC_CPU.cpp:139).
void     oracle_canonical_at(uint32_t seed, const uint64_t* pos, uint64_t k, float* out);
void     oracle_canonical_from(uint32_t seed, uint64_t start, uint64_t k, float* out);
// One vertex of the sweep from its neighbours' colours (violation_count, count_free_colors, fill_p,
// extract_new_color with taboo 0). Returns 1 on a CDF overflow (colour from rand()), else 0.
int      oracle_vertex_update(uint32_t nCol, float epsilon, uint32_t cv, const uint32_t* nbr_colors, uint64_t deg,
                              float u, uint32_t* color, int* viol);

// ---- MCMC: ColoringMCMC_CPU(g, params, seed) + run() ----
// out_init   : optional [n]  initial coloring (after the ctor)
// out_colors : [n]           final coloring C
// traj       : optional [traj_cap] Cviol at the top of every sweep, then the final Cviol
// sweep_limit: 0 = reference semantics; k > 0 stops after k sweeps (bounded baseline samples)
// nthreads   : 1 = faithful single-thread restatement; >1 = OpenMP variant (bit-identical)
int      oracle_mcmc_run(uint32_t n, const uint64_t* row_off, const uint32_t* col_idx,
                         const oracle_params* prm, uint32_t seed,
                         uint32_t* out_init, uint32_t* out_colors,
                         uint64_t* traj, uint64_t traj_cap,
                         uint32_t sweep_limit, int nthreads, oracle_result* res);

// ---- reference-GPU-semantics mode (oracle/mcmc_gpu_ref.cpp) ----
typedef struct {
    uint32_t rip;               // ColoringMCMC::rip after the loop (coloringMCMC_main.cu:160-269)
    int32_t  maxIterReached;    // rip == maxRip (:294-295)
    uint32_t sweeps;            // sweeps executed
    uint32_t tailcutPasses;     // passes of the GPU tail cut (:279-289), bounded by tail_max_passes
    uint64_t conflictCounter;   // the host's conflictCounter at loop exit (tail-cut entry value)
    uint64_t finalConflicts;    // conflicting edges of the returned colouring
    uint64_t trajLen;           // conflicting-edge counts written: C_0 .. C_last
} oracle_gpu_result;

// cuRAND XORWOW (flavor 0; 1 = rocRAND's salts): state after curand_init(seed, subsequence, 0),
// out = {v0..v4, d}; _next advances a state and returns `count` outputs.
void     oracle_xorwow_init(uint64_t seed, uint64_t subsequence, int flavor, uint32_t out[6]);
void     oracle_xorwow_next(uint32_t st[6], uint32_t count, uint32_t* out);
// GPURand(n, seed) (GPURandomizer.cu:85-101): states [n][6].
void     oracle_gpurand_init(uint32_t n, uint32_t seed, uint32_t* states);
// ColoringMCMC::run() with the default build's kernels. states: in/out [n][6] (the per-vertex
// curandStates shared by all repetitions, main.cu:80,193). traj: conflicting-edge count of every
// colouring the loop counted, plus the last sweep's when the loop ran out. The tail cut runs when
// prm->tailcut (as the reference's), at most tail_max_passes passes; tail_traj: optional
// [tail_max_passes] counts after each pass.
int      oracle_mcmc_gpu_run(uint32_t n, const uint64_t* row_off, const uint32_t* col_idx, const oracle_params* prm,
                             uint32_t* states, uint32_t* out_colors, uint64_t* traj, uint64_t traj_cap,
                             uint32_t tail_max_passes, uint64_t* tail_traj, oracle_gpu_result* res);

// Writes the reference's saveStats / saveColor text outputs (coloringMCMC_CPUutils.cpp:70-109).
int      oracle_save_outputs(const char* log_path, const char* colors_path, uint32_t n, uint64_t nEdges,
                             uint32_t maxDeg, uint32_t minDeg, float meanDeg, float prob, uint32_t seed,
                             uint32_t repetition, float duration, const oracle_params* prm,
                             const oracle_result* res, const uint32_t* colors);
}
