// include/mcmc_colorer.hpp -- header-only C++ class surface of the reference's MCMC colorer,
// rebuilt over the C ABI in mcmc_hip.h (link with -lmcmc_hip).
//
// Reference surface (paths relative to /root/reference/src), as called from src/main.cu:60-202:
//   struct ColoringMCMCParams                      graph_coloring/coloring.h:65-74
//   template<nodeW,edgeW> struct GraphStruct       graph/graph.h:37-79  (uint64 cumulDegs here)
//   template<nodeW,edgeW> class Graph              graph/graph.h:84-133
//       Graph(node nn, float prob, uint32_t seed)  -> setupRnd2 (graphCPU.cpp:291-404), on the GPU
//       Graph(fileImporter*, bool)                 -> setupImporterNew (graphCPU.cpp:112-170)
//       Graph(Graph* host)                         -> device copy (graphGPU.cu:210-226)
//   class GPURand(n, seed), member randStates      GPUutils/GPURandomizer.h:42-55
//   template<nodeW,edgeW> class ColoringMCMC       graph_coloring/coloringMCMC.h:44-140
//       ColoringMCMC(Graph* g_d, randStates, ColoringMCMCParams); run(int); setDirectoryPath(string)
//
// Behaviour: run(i) computes exactly what ColoringMCMC_CPU(g, params, seed + i).run() computes
// (main.cu:171), on the GPU. The reference's process-global glibc rand() stream (setupRnd2 draws and
// CDF-overflow draws) is a process-global glibc window here (mcmc::glibc_global()). Like the
// reference (GPUutils/GPUutils.h:20-26), errors print and abort.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "mcmc_hip.h"

typedef uint32_t node;
typedef uint32_t node_sz;
typedef uint32_t col;
typedef uint32_t col_sz;

namespace mcmc {

inline void check(int rc, const char* file, int line) {
    if (rc != MCMC_OK) {
        std::fprintf(stderr, "libmcmc_hip error %d: %s (%s:%d)\n", rc, mcmc_last_error(), file, line);
        std::abort();
    }
}
#define MCMC_CHECK(x) ::mcmc::check((x), __FILE__, __LINE__)

// The process-wide glibc rand() position (unseeded == srand(1), ArgHandle.cpp:272-276).
struct GlibcWindow {
    uint32_t w[31];
};
inline GlibcWindow& glibc_global() {
    static GlibcWindow g = [] {
        GlibcWindow x;
        MCMC_CHECK(mcmc_glibc_window(1, 0, x.w));
        return x;
    }();
    return g;
}
// srand(seed) (ArgHandle.cpp:275, used when --seed is 0).
inline void glibc_srand(uint32_t seed) { MCMC_CHECK(mcmc_glibc_window(seed, 0, glibc_global().w)); }

}  // namespace mcmc

// ColoringMCMCParams (coloring.h:65-74)
struct ColoringMCMCParams {
    uint32_t maxRip;
    col_sz nCol;
    float numColorRatio;
    float lambda;
    float epsilon;
    float ratioFreezed;
    uint32_t tabooIteration;
    bool tailcut;
    uint32_t tailcutRepair = 0;   // extension: corrected tail-cut pass cap (mcmc_set_tailcut_repair), 0 = off
};

// GraphStruct (graph.h:37-79) -- host view; cumulDegs widened to uint64.
template <typename nodeW, typename edgeW>
struct GraphStruct {
    node nNodes{0};
    uint64_t nEdges{0};
    std::vector<uint64_t> cumulDegsV;
    std::vector<node> neighsV;
    uint64_t* cumulDegs{nullptr};
    node* neighs{nullptr};
    uint64_t deg(node i) const { return cumulDegs[i + 1] - cumulDegs[i]; }
};

template <typename nodeW, typename edgeW>
class Graph {
public:
    // Graph(n, prob, seed) -> setupRnd2; `seed` is unused by the reference too (graphCPU.cpp:291).
    Graph(node nn, float prob_, uint32_t /*seed*/, int device = 0) : prob(prob_), device_(device) {
        MCMC_CHECK(mcmc_graph_simulate(nn, prob_, mcmc::glibc_global().w, device, &h_));
        info();
    }
    // The build's counter-based G(n, p) (csrc/er_gen.h) for sizes where setupRnd2 is infeasible
    // (C3: n = 1e7): generated straight into the sweep's tiled layout; no CSR is materialised.
    struct ErFast {};
    Graph(ErFast, node nn, float prob_, uint64_t seed, int device = 0) : prob(prob_), device_(device) {
        MCMC_CHECK(mcmc_graph_er_fast(nn, prob_, seed, device, &h_));
        info();
    }
    // Only rows [v_begin, v_end) of that graph (one rank of a partitioned run).
    Graph(ErFast, node nn, float prob_, uint64_t seed, int device, node v_begin, node v_end)
        : prob(prob_), device_(device) {
        MCMC_CHECK(mcmc_graph_er_fast_rows(nn, prob_, seed, v_begin, v_end, device, &h_));
        info();
    }
    // Host CSR (e.g. from the edge-list importer) -> device copy.
    Graph(const std::vector<uint64_t>& cumulDegs, const std::vector<node>& neighs, float prob_, int device = 0)
        : prob(prob_), device_(device) {
        MCMC_CHECK(mcmc_graph_upload(cumulDegs.data(), neighs.data(), (uint32_t)(cumulDegs.size() - 1),
                                     neighs.size(), device, &h_));
        info();
    }
    // A host-only graph (no device copy): the CSR as the reference's host Graph holds it, for
    // ColoringMCMC_CPU's per-vertex hooks and violation_count without a GPU; run() needs a device graph.
    struct HostOnly {};
    Graph(HostOnly, const std::vector<uint64_t>& cumulDegs, const std::vector<node>& neighs, float prob_ = 0.0f)
        : prob(prob_) {
        n_ = (node)(cumulDegs.size() - 1);
        m_ = neighs.size();
        str_.nNodes = n_;
        str_.nEdges = m_;
        str_.cumulDegsV = cumulDegs;
        str_.neighsV = neighs.empty() ? std::vector<node>(1) : neighs;
        str_.cumulDegs = str_.cumulDegsV.data();
        str_.neighs = str_.neighsV.data();
        maxDeg_ = 0;
        minDeg_ = n_ ? ~node(0) : 0;
        for (node i = 0; i < n_; i++) {   // doStats (graphCPU.cpp:432-450)
            maxDeg_ = std::max<node>(maxDeg_, (node)str_.deg(i));
            minDeg_ = std::min<node>(minDeg_, (node)str_.deg(i));
        }
    }
    ~Graph() {
        if (h_) mcmc_graph_destroy(h_);
    }
    Graph(const Graph&) = delete;
    Graph& operator=(const Graph&) = delete;

    GraphStruct<nodeW, edgeW>* getStruct() {
        if (!str_.cumulDegs && h_) {
            str_.nNodes = n_;
            str_.nEdges = m_;
            str_.cumulDegsV.resize((size_t)n_ + 1);
            str_.neighsV.resize(m_ ? m_ : 1);
            MCMC_CHECK(mcmc_graph_download(h_, str_.cumulDegsV.data(), str_.neighsV.data()));
            str_.cumulDegs = str_.cumulDegsV.data();
            str_.neighs = str_.neighsV.data();
        }
        return &str_;
    }
    node getNNodes() const { return n_; }
    uint64_t getNEdges() const { return m_; }
    node getMaxNodeDeg() const { return maxDeg_; }
    node getMinNodeDeg() const { return minDeg_; }
    float getMeanNodeDeg() const { return n_ ? (float)m_ / (float)n_ : 0.0f; }
    const mcmc_graph* handle() const { return h_; }
    bool onDevice() const { return h_ != nullptr; }
    int device() const { return device_; }
    float prob{0.0f};
    // Row-partial graphs (ErFast with a row range: one rank's rows) describe only their rows; the
    // whole graph's statistics (sum of arcs, max / min degree over every rank's rows) make the
    // default nCol (main.cu:162) and the reports equal the one-GPU run's.
    static void mergePartitionStats(const std::vector<Graph*>& parts) {
        uint64_t m = 0;
        node mx = 0, mn = ~node(0);
        for (const Graph* p : parts) {
            m += p->m_;
            mx = std::max(mx, p->maxDeg_);
            mn = std::min(mn, p->minDeg_);
        }
        for (Graph* p : parts) {
            p->m_ = m;
            p->maxDeg_ = mx;
            p->minDeg_ = parts.empty() ? 0 : mn;
        }
    }

private:
    void info() { MCMC_CHECK(mcmc_graph_info(h_, &n_, &m_, &maxDeg_, &minDeg_)); }
    mcmc_graph* h_{nullptr};
    int device_{0};
    node n_{0};
    uint64_t m_{0};
    node maxDeg_{0}, minDeg_{0};
    GraphStruct<nodeW, edgeW> str_;
};

// GPURand (GPURandomizer.h:42-55): the reference keeps one cuRAND state per vertex; the sweep
// derives every draw by minstd skip-ahead, so only the seed is kept.
struct GPURandHandle {
    uint32_t seed;
};
class GPURand {
public:
    GPURand(uint32_t n, long seed) : num(n) { state.seed = (uint32_t)seed; randStates = &state; }
    uint32_t num;
    GPURandHandle* randStates;

private:
    GPURandHandle state{};
};

template <typename nodeW, typename edgeW>
class ColoringMCMC {
public:
    ColoringMCMC(Graph<nodeW, edgeW>* inGraph_d, GPURandHandle* randStates, ColoringMCMCParams params)
        : graph(inGraph_d), seed(randStates->seed), param(params) {}
    // Extension: the same colorer vertex-partitioned over several GPUs of this node,
    // one graph per device (each holding at least the rows [bounds[i], bounds[i+1]) of its rank, in
    // rank order), driven from this thread with RCCL inside the library (mcmc_comm_init_all,
    // mcmc_part_create, mcmc_part_run). run() / save() / the results are those of the one-GPU run.
    ColoringMCMC(std::vector<Graph<nodeW, edgeW>*> perDevice, std::vector<uint32_t> bounds_, GPURandHandle* randStates,
                 ColoringMCMCParams params)
        : graph(perDevice.at(0)), parts(perDevice), bounds(bounds_), seed(randStates->seed), param(params) {
        if (bounds.size() != parts.size() + 1) {
            std::fprintf(stderr, "ColoringMCMC: %zu graphs need %zu bounds\n", parts.size(), parts.size() + 1);
            std::abort();
        }
        std::vector<int> devs;
        for (auto* g : parts) devs.push_back(g->device());
        comms.assign(parts.size(), nullptr);
        // ranks sharing one device run over the library's loopback transport (device copies; RCCL
        // refuses two ranks on one GPU) -- a rehearsal of the partitioned run on a single GPU
        const bool one_device = std::all_of(devs.begin(), devs.end(), [&](int x) { return x == devs[0]; });
        if (!one_device || devs.size() == 1)
            MCMC_CHECK(mcmc_comm_init_all(devs.data(), (uint32_t)devs.size(), comms.data()));
    }
    ~ColoringMCMC() {
        if (ctx) mcmc_destroy(ctx);
        for (auto* c : pctx) mcmc_destroy(c);
        for (auto* c : comms) mcmc_comm_destroy(c);
    }

    void setDirectoryPath(std::string directory) { this->directory = directory; }

    // One repetition: engine seed = seed + iteration (main.cu:171), glibc stream = process global.
    void run(int iteration) {
        if (ctx) mcmc_destroy(ctx);
        ctx = nullptr;
        mcmc_params p{};
        p.nCol = param.nCol;
        p.epsilon = param.epsilon;
        p.lambda = param.lambda;
        p.ratioFreezed = param.ratioFreezed;
        p.numColorRatio = param.numColorRatio;
        p.maxRip = param.maxRip;
        p.tabooIteration = param.tabooIteration;
        p.tailcut = param.tailcut;
        p.seed = seed + (uint32_t)iteration;
        mcmc_ctx* res = nullptr;
        if (parts.empty()) {
            MCMC_CHECK(mcmc_create(graph->handle(), &p, 0, graph->getNNodes(), &ctx));
            MCMC_CHECK(mcmc_set_glibc_window(ctx, mcmc::glibc_global().w));
            if (param.tailcutRepair) MCMC_CHECK(mcmc_set_tailcut_repair(ctx, param.tailcutRepair));
            MCMC_CHECK(mcmc_init_coloring(ctx, nullptr));
            MCMC_CHECK(mcmc_run(ctx, 0, &stats));
            res = ctx;
        } else {
            for (auto* c : pctx) mcmc_destroy(c);
            pctx.assign(parts.size(), nullptr);
            const uint32_t world = (uint32_t)parts.size();
            for (uint32_t r = 0; r < world; r++) {
                MCMC_CHECK(mcmc_part_create(parts[r]->handle(), &p, world, r, bounds.data(), comms[r], &pctx[r]));
                MCMC_CHECK(mcmc_set_glibc_window(pctx[r], mcmc::glibc_global().w));
                if (param.tailcutRepair) MCMC_CHECK(mcmc_set_tailcut_repair(pctx[r], param.tailcutRepair));
                MCMC_CHECK(mcmc_init_coloring(pctx[r], nullptr));
            }
            std::vector<mcmc_run_stats> st(world);
            MCMC_CHECK(mcmc_part_run(pctx.data(), world, 0, st.data()));
            stats = st[0];
            res = pctx[0];
        }
        MCMC_CHECK(mcmc_get_glibc_window(res, mcmc::glibc_global().w));
        coloring.resize(graph->getNNodes());
        MCMC_CHECK(mcmc_get_coloring(res, coloring.data()));
        trajectory.resize(stats.trajLen);
        uint64_t len = 0;
        MCMC_CHECK(mcmc_get_trajectory(res, trajectory.data(), trajectory.size(), &len));
        lastSeed = p.seed;
        lastRepetition = iteration;
        if (!directory.empty()) save();
    }

    // Report in the layout of saveStats (coloringMCMC_CPUutils.cpp:70-102), parseable by the
    // reference's pyScripts/logParser.py, plus the per-sweep trajectory; colours as "<v> <c>".
    void save() const {
        std::ofstream out(directory + ".log");
        const uint32_t nCol = param.nCol;
        out << "MCMC Colorer - GPU (MI355X) version - Report" << std::endl;
        out << "-------------------------------------------" << std::endl;
        out << "GRAPH INFO" << std::endl;
        out << "Nodes: " << graph->getNNodes() << " - Edges: " << graph->getNEdges() << std::endl;
        out << "Max deg: " << graph->getMaxNodeDeg() << " - Min deg: " << graph->getMinNodeDeg()
            << " - Avg deg: " << graph->getMeanNodeDeg() << std::endl;
        out << "Edge probability (for randomly generated graphs): " << graph->prob << std::endl;
        out << "Seed: " << lastSeed << std::endl;
        out << "-------------------------------------------" << std::endl;
        out << "EXECUTION INFO" << std::endl;
        out << "Repetition: " << lastRepetition << std::endl;
        out << "Execution time: " << stats.loopMs / 1000.0 << std::endl;
        out << "Iteration performed: " << stats.iter << std::endl;
        out << "Max iteration reached: " << (stats.maxIterReached ? "yes" : "no") << std::endl;
        out << "-------------------------------------------" << std::endl;
        out << "Color histogram:" << std::endl;
        std::vector<size_t> hist(nCol, 0);
        for (uint32_t c : coloring) hist[c]++;
        size_t used = 0;
        for (size_t i = 0; i < nCol; i++) { out << i << ": " << hist[i] << std::endl; if (hist[i]) used++; }
        out << "Number of colors: " << nCol << " - Used colors: " << used << std::endl;
        out << "Color ratio: " << param.numColorRatio << std::endl;
        float mean = 0;
        for (size_t h : hist) mean += (float)h;
        mean /= (float)nCol;
        float var = 0;
        for (size_t h : hist) var += ((h - mean) * (h - mean));
        var /= (float)nCol;
        out << "Average number of nodes for each color: " << mean << std::endl;
        out << "Variance: " << var << std::endl;
        out << "StD: " << std::sqrt(var) << std::endl;
        out << "Conflicts per sweep (C violations):";
        for (uint64_t x : trajectory) out << " " << x;
        out << std::endl;
        std::ofstream cf(directory + "-colors.txt");
        for (size_t i = 0; i < coloring.size(); i++) cf << i << " " << coloring[i] << "\n";
    }

    const std::vector<uint32_t>& getColoring() const { return coloring; }
    const std::vector<uint64_t>& getTrajectory() const { return trajectory; }
    const mcmc_run_stats& getStats() const { return stats; }

private:
    Graph<nodeW, edgeW>* graph;
    std::vector<Graph<nodeW, edgeW>*> parts;   // partitioned: one graph per device, rank order
    std::vector<uint32_t> bounds;
    std::vector<mcmc_comm*> comms;
    std::vector<mcmc_ctx*> pctx;
    uint32_t seed;
    ColoringMCMCParams param;
    std::string directory;
    mcmc_ctx* ctx{nullptr};
    mcmc_run_stats stats{};
    std::vector<uint32_t> coloring;
    std::vector<uint64_t> trajectory;
    uint32_t lastSeed{0};
    int lastRepetition{0};
};

// ---- ColoringMCMC_CPU's class surface (graph_coloring/coloringMCMC_CPU.h:15-31) ----------------
// The reference's --mcmccpu colorer, run by the same HIP sweep as ColoringMCMC (its semantics ARE
// the CPU colorer's: bit-identical colouring, iteration count and glibc stream). Kept: the ctor
// (graph, params, seed -- main.cu:171 passes seed + repetition; it draws the initial colouring C
// with default_random_engine(seed) and uniform_int_distribution, coloringMCMC_CPU.cpp:53-61), run(),
// show_histogram(), violation_count() (on the GPU for a device graph, else on the host), saveStats()
// and saveColor() in the reference's layout (coloringMCMC_CPUutils.cpp:70-109), and the per-vertex
// hooks the reference made public for its GoogleTest (coloringMCMC_CPU.h:20-28): count_free_colors,
// fill_p, extract_new_color, fill_qstar -- host restatements of coloringMCMC_CPU.cpp:362-551 over
// the class's own buffers (p, q, qstar, freeColors, Cviols, taboo, colorIdx = identity), CDF
// overflows drawing rand() from the process-global glibc window like the sweep. With the dbg
// accessors (getC, getCstar, getp, ...) a test drives loop 1 of run() vertex by vertex.
template <typename nodeW, typename edgeW>
class ColoringMCMC_CPU {
public:
    ColoringMCMC_CPU(Graph<nodeW, edgeW>* g, ColoringMCMCParams params, uint32_t seed)
        : graph(g), param(params), seed(seed), nCol(params.nCol), epsilon(params.epsilon) {
        const size_t n = g->getNNodes();
        gen.seed(seed);
        std::uniform_int_distribution<uint32_t> unifInitColors(0, nCol - 1);
        C.resize(n);
        for (size_t i = 0; i < n; i++) C[i] = unifInitColors(gen);   // coloringMCMC_CPU.cpp:61
        Cstar.assign(n, 0);
        p.assign(nCol, 0.0f);
        q.assign(n, 0.0f);
        qstar.assign(n, 0.0f);
        freeColors.assign(nCol, false);
        Cviols.assign(n, false);
        Cstarviols.assign(n, false);
        taboo.assign(n, 0);
        colorIdx.resize(nCol);
        std::iota(colorIdx.begin(), colorIdx.end(), (size_t)0);
    }
    ~ColoringMCMC_CPU() {
        if (ctx) mcmc_destroy(ctx);
    }

    void run() {
        if (ctx) mcmc_destroy(ctx);
        ctx = nullptr;
        mcmc_params p_ = to_params();
        MCMC_CHECK(mcmc_create(graph->handle(), &p_, 0, graph->getNNodes(), &ctx));
        MCMC_CHECK(mcmc_set_glibc_window(ctx, mcmc::glibc_global().w));   // rand(): the process stream
        if (param.tailcutRepair) MCMC_CHECK(mcmc_set_tailcut_repair(ctx, param.tailcutRepair));
        MCMC_CHECK(mcmc_init_coloring(ctx, nullptr));
        MCMC_CHECK(mcmc_run(ctx, 0, &stats));
        MCMC_CHECK(mcmc_get_glibc_window(ctx, mcmc::glibc_global().w));
        C.resize(graph->getNNodes());
        MCMC_CHECK(mcmc_get_coloring(ctx, C.data()));
        iter = stats.iter;
        maxIterReached = stats.maxIterReached != 0;
    }

    void show_histogram() const {
        std::vector<size_t> hist(param.nCol, 0);
        for (uint32_t c : C) hist[c]++;
        for (size_t i = 0; i < hist.size(); i++) std::cout << i << ": " << hist[i] << std::endl;
    }

    // Vertices with a neighbour of their own colour in `currentColoring` (coloringMCMC_CPU.cpp:329-351),
    // their flags in `violations`; counted on the GPU for a device graph, else on the host.
    size_t violation_count(const std::vector<uint32_t>& currentColoring, std::vector<bool>& violations) {
        if (!graph->onDevice()) {
            const GraphStruct<nodeW, edgeW>* str = graph->getStruct();
            violations.assign(currentColoring.size(), false);
            size_t count = 0;
            for (size_t i = 0; i < currentColoring.size(); i++) {
                for (uint64_t k = str->cumulDegs[i]; k < str->cumulDegs[i + 1]; k++)
                    if (currentColoring[str->neighs[k]] == currentColoring[i]) {
                        violations[i] = true;
                        count++;
                        break;
                    }
            }
            return count;
        }
        mcmc_params p_ = to_params();
        mcmc_ctx* vc = nullptr;
        MCMC_CHECK(mcmc_create(graph->handle(), &p_, 0, graph->getNNodes(), &vc));
        MCMC_CHECK(mcmc_init_coloring(vc, currentColoring.data()));
        uint64_t count = 0;
        std::vector<uint8_t> flags(graph->getNNodes());
        MCMC_CHECK(mcmc_count_violations(vc, &count, flags.data()));
        mcmc_destroy(vc);
        violations.assign(flags.begin(), flags.end());
        return (size_t)count;
    }

    // count_free_colors (coloringMCMC_CPU.cpp:362-383): freeColors[c] = no neighbour of `node_` has
    // colour c in currentColoring; returns how many are free (Zvcomp).
    size_t count_free_colors(const size_t node_, const std::vector<uint32_t>& currentColoring,
                             std::vector<bool>& freeCols) {
        const GraphStruct<nodeW, edgeW>* str = graph->getStruct();
        std::fill(std::begin(freeCols), std::end(freeCols), true);
        for (uint64_t k = str->cumulDegs[node_]; k < str->cumulDegs[node_ + 1]; k++) freeCols[currentColoring[str->neighs[k]]] = false;
        return (size_t)std::count(std::begin(freeCols), std::end(freeCols), true);
    }

    // fill_p (coloringMCMC_CPU.cpp:393-481, the baseline branch): p from C[currentNode], Cviols and
    // the member freeColors (count_free_colors(node, C, freeColors) fills it), Zv = occupied colours.
    void fill_p(const size_t currentNode, const size_t Zv) {
        const size_t Zvcomp = nCol - Zv;
        const uint32_t currentColor = C[currentNode];
        if (Cviols[currentNode]) {
            const int nFreeColors = std::accumulate(std::begin(freeColors), std::end(freeColors), 0);
            if (nFreeColors == 0) {
                for (size_t idx = 0; idx < p.size(); idx++) p[idx] = idx == currentColor ? 1.0f - (nCol - 1) * epsilon : epsilon;
                return;
            }
            for (size_t idx = 0; idx < p.size(); idx++)
                p[idx] = freeColors[idx] ? (1.0f - epsilon * Zv) / (float)Zvcomp : epsilon;
        } else {
            for (size_t idx = 0; idx < p.size(); idx++) p[idx] = colorIdx[idx] == currentColor ? 1.0f - (nCol - 1) * epsilon : epsilon;
        }
    }

    // extract_new_color (coloringMCMC_CPU.cpp:493-528): taboo; else the first colour whose fp32 CDF
    // passes the vertex's draw (strict >), on overflow rand() % (nCol - 1) from the process-global
    // glibc window; qVect[currentNode] = p of the colour chosen; taboo set when the colour stays.
    void extract_new_color(const size_t currentNode, const std::vector<float>& pVect,
                           const std::vector<float>& experimentVect, std::vector<float>& qVect,
                           std::vector<uint32_t>& newColoring) {
        if (taboo[currentNode] > 0) {
            taboo[currentNode]--;
            newColoring[currentNode] = C[currentNode];
            qVect[currentNode] = (1.0f - (nCol - 1) * epsilon);
            return;
        }
        const float experimentThrsh = experimentVect[currentNode];
        float cdf = 0;
        size_t idx;
        for (idx = 0; idx < pVect.size(); idx++) {
            cdf += pVect[idx];
            if (cdf > experimentThrsh) break;
        }
        if (idx >= nCol) {
            uint32_t r = 0;
            MCMC_CHECK(mcmc_glibc_draw(mcmc::glibc_global().w, 1, &r));
            idx = r % (nCol - 1);
        }
        qVect[currentNode] = pVect[idx];
        newColoring[currentNode] = (uint32_t)idx;
        taboo[currentNode] = (newColoring[currentNode] == C[currentNode]) * param.tabooIteration;
    }

    // fill_qstar (coloringMCMC_CPU.cpp:532-551): the Hastings term of the new colour, into the member
    // qstar (as the reference: its qVect argument is not written).
    void fill_qstar(const size_t currentNode, const size_t Zv, const std::vector<uint32_t>& newColoring,
                    const std::vector<uint32_t>& oldColoring, const std::vector<bool>& freeCols,
                    const std::vector<bool>& newColoringViols, std::vector<float>& /*qVect*/) {
        const size_t Zvcomp = nCol - Zv;
        const uint32_t currentColor = newColoring[currentNode];
        if (newColoringViols[currentNode]) {
            qstar[currentNode] = freeCols[currentColor] ? (1.0f - epsilon * Zv) / (float)Zvcomp : epsilon;
        } else {
            qstar[currentNode] = newColoring[currentNode] == oldColoring[currentNode] ? 1.0f - (nCol - 1) * epsilon : epsilon;
        }
    }

    void saveStats(size_t it, float duration, std::ofstream& outFile) const {
        const uint32_t nCol_ = param.nCol;
        outFile << "MCMC Colorer - CPU version - Report" << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "GRAPH INFO" << std::endl;
        outFile << "Nodes: " << graph->getNNodes() << " - Edges: " << graph->getNEdges() << std::endl;
        outFile << "Max deg: " << graph->getMaxNodeDeg() << " - Min deg: " << graph->getMinNodeDeg()
                << " - Avg deg: " << graph->getMeanNodeDeg() << std::endl;
        outFile << "Edge probability (for randomly generated graphs): " << graph->prob << std::endl;
        outFile << "Seed: " << seed << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "EXECUTION INFO" << std::endl;
        outFile << "Repetition: " << it << std::endl;
        outFile << "Execution time: " << duration << std::endl;
        outFile << "Iteration performed: " << iter << std::endl;
        outFile << "Max iteration reached: " << (maxIterReached ? "yes" : "no") << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "Color histogram:" << std::endl;
        std::vector<size_t> hist(nCol_, 0);
        for (uint32_t c : C) hist[c]++;
        size_t used = 0;
        for (size_t i = 0; i < nCol_; i++) {
            outFile << i << ": " << hist[i] << std::endl;
            if (hist[i]) used++;
        }
        outFile << "Number of colors: " << nCol_ << " - Used colors: " << used << std::endl;
        outFile << "Color ratio: " << param.numColorRatio << std::endl;
        size_t total = 0;
        for (size_t h : hist) total += h;
        const float mean = (float)(int)total / (float)nCol_;   // std::accumulate(..., 0): an int sum
        float var = 0;
        for (size_t h : hist) var += ((h - mean) * (h - mean));
        var /= (float)nCol_;
        outFile << "Average number of nodes for each color: " << mean << std::endl;
        outFile << "Variance: " << var << std::endl;
        outFile << "StD: " << std::sqrt(var) << std::endl;
    }

    void saveColor(std::ofstream& outfile) const {
        for (size_t i = 0; i < C.size(); i++) outfile << i << " " << C[i] << std::endl;
    }

    // the dbg accessors (coloringMCMC_CPU.h:34-51)
    std::vector<uint32_t>* getC() { return &C; }
    std::vector<uint32_t>* getCstar() { return &Cstar; }
    std::vector<float>* getp() { return &p; }
    std::vector<float>* getq() { return &q; }
    std::vector<float>* getqstar() { return &qstar; }
    std::vector<bool>* getfreeColors() { return &freeColors; }
    std::vector<bool>* getCviols() { return &Cviols; }
    std::vector<bool>* getCstarviols() { return &Cstarviols; }
    std::vector<uint32_t>* getTaboo() { return &taboo; }
    uint32_t* getnCol() { return &nCol; }
    float* getepsilon() { return &epsilon; }
    const mcmc_run_stats& getStats() const { return stats; }

private:
    mcmc_params to_params() const {
        mcmc_params p_{};
        p_.nCol = param.nCol;
        p_.epsilon = param.epsilon;
        p_.lambda = param.lambda;
        p_.ratioFreezed = param.ratioFreezed;
        p_.numColorRatio = param.numColorRatio;
        p_.maxRip = param.maxRip;
        p_.tabooIteration = param.tabooIteration;
        p_.tailcut = param.tailcut;
        p_.seed = seed;
        return p_;
    }

    Graph<nodeW, edgeW>* graph;
    ColoringMCMCParams param;
    uint32_t seed;
    uint32_t nCol;
    float epsilon;
    std::default_random_engine gen;
    mcmc_ctx* ctx{nullptr};
    mcmc_run_stats stats{};
    std::vector<uint32_t> C, Cstar, taboo;
    std::vector<float> p, q, qstar;
    std::vector<bool> freeColors, Cviols, Cstarviols;
    std::vector<size_t> colorIdx;
    uint32_t iter{0};
    bool maxIterReached{false};
};

// ---- reference-GPU-semantics mode -------------------------------------
// GPURand's per-vertex curandStates (GPURandomizer.cu:85-101), shared by every repetition.
class CurandStates {
public:
    CurandStates(uint32_t n, long seed, int device = 0) : num(n) {
        MCMC_CHECK(mcmc_gpurand_create(n, (uint32_t)seed, device, &h_));
    }
    ~CurandStates() { mcmc_gpurand_destroy(h_); }
    CurandStates(const CurandStates&) = delete;
    CurandStates& operator=(const CurandStates&) = delete;
    mcmc_gpurand* handle() const { return h_; }
    uint32_t num;

private:
    mcmc_gpurand* h_{nullptr};
};

// The reference's own ColoringMCMC (coloringMCMC.h:44-140 as built by default: balance-dynamic
// proposal, XORWOW per vertex, conflicts counted as edges, the GPU tail cut) on the MI355X sweep.
// run() writes <dir>.log in the layout of coloringMCMC_prints.cu and <dir>-colors.txt.
template <typename nodeW, typename edgeW>
class ColoringMCMCGpuRef {
public:
    ColoringMCMCGpuRef(Graph<nodeW, edgeW>* inGraph_d, CurandStates* randStates, ColoringMCMCParams params,
                       uint32_t tailMaxPasses = 1000)
        : graph(inGraph_d), states(randStates), param(params), tailMax(tailMaxPasses) {}
    ~ColoringMCMCGpuRef() { if (ctx) mcmc_destroy(ctx); }
    void setDirectoryPath(std::string directory) { this->directory = directory; }

    void run(int /*iteration*/) {
        if (ctx) mcmc_destroy(ctx);
        mcmc_params p{};
        p.nCol = param.nCol;
        p.epsilon = param.epsilon;
        p.lambda = param.lambda;
        p.ratioFreezed = param.ratioFreezed;
        p.numColorRatio = param.numColorRatio;
        p.maxRip = param.maxRip;
        p.tabooIteration = param.tabooIteration;
        p.tailcut = param.tailcut;
        MCMC_CHECK(mcmc_ref_create(graph->handle(), &p, states->handle(), &ctx));
        MCMC_CHECK(mcmc_ref_run(ctx, tailMax, &stats));
        coloring.resize(graph->getNNodes());
        MCMC_CHECK(mcmc_get_coloring(ctx, coloring.data()));
        uint64_t len = 0;
        trajectory.resize(stats.trajLen);
        MCMC_CHECK(mcmc_get_trajectory(ctx, trajectory.data(), trajectory.size(), &len));
        MCMC_CHECK(mcmc_get_tail_trajectory(ctx, nullptr, 0, &len));
        tail.resize(len);
        MCMC_CHECK(mcmc_get_tail_trajectory(ctx, tail.data(), tail.size(), &len));
        if (!directory.empty()) save();
    }

    // coloringMCMC_prints.cu: __customPrintRun0_start (:20-36), per iteration Run2/Run3 (:55-75),
    // the tail cut's (Run2 with "---> TailCutting"; its "nuovi conflitti" is the last sweep's
    // count, conflictCounterStar is not updated there), Run7_end (:95-110) + getStatsNumColors.
    void save() const {
        std::ofstream log(directory + ".log");
        uint64_t fr = 0, tot = 0;
        (void)mcmc_device_mem_info(0, &fr, &tot);
        log << "total memory: " << tot << " free memory:" << fr << std::endl;
        log << "numCol: " << param.nCol << std::endl;
        log << "epsilon: " << param.epsilon << std::endl;
        log << "lambda: " << param.lambda << std::endl;
        log << "ratioFreezed: " << param.ratioFreezed << std::endl;
        log << "maxRip: " << param.maxRip << std::endl << std::endl;
        log << "numColorRatio: " << param.numColorRatio << std::endl;
        const uint32_t sweeps = stats.sweepsRun;
        for (uint32_t k = 1; k <= sweeps; k++) {
            log << "***** Tentativo numero: " << k << std::endl;
            log << "conflitti rilevati: " << trajectory[k - 1] << std::endl;
            log << "nuovi conflitti rilevati: " << trajectory[k] << std::endl;
        }
        uint64_t cc = sweeps == param.maxRip && sweeps > 0 ? trajectory[sweeps - 1] : trajectory[stats.trajLen - 1];
        const uint64_t star = sweeps ? trajectory[sweeps] : 0;
        for (uint64_t x : tail) {
            log << "***** Tentativo numero: " << stats.iter << std::endl << "---> TailCutting" << std::endl;
            log << "conflitti rilevati: " << cc << std::endl;
            log << "nuovi conflitti rilevati: " << star << std::endl;
            cc = x;
        }
        log << "COLORAZIONE FINALE" << std::endl;
        log << "Time " << stats.loopMs / 1000.0 << std::endl;
        log << "Max iteration reached " << (stats.maxIterReached ? "yes" : "no") << std::endl;
        // getStatsNumColors("end_") (:123-218)
        const uint32_t n = graph->getNNodes(), nCol = param.nCol;
        std::vector<uint32_t> h(std::max(n, nCol) + 1, 0);
        for (uint32_t c : coloring) h[c]++;
        int counter = 0, max_i = 0, min_i = (int)n, max_c = 0, min_c = (int)n;
        const float average = (float)n / (float)nCol;
        float variance = 0, balancingIndex = 0;
        for (uint32_t i = 0; i < nCol; i++) {
            if (h[i] > 0) {
                counter++;
                if ((int)h[i] > max_c) { max_i = (int)i; max_c = (int)h[i]; }
                if ((int)h[i] < min_c) { min_i = (int)i; min_c = (int)h[i]; }
                const float d = (float)h[i] - average;
                balancingIndex += d * d;
            }
        }
        balancingIndex /= ((float)n * graph->prob);
        balancingIndex = std::sqrt(balancingIndex);
        for (uint32_t i = 0; i < nCol; i++) {
            const float d = (float)h[i] - average;
            variance += d * d;
        }
        variance /= (float)nCol;
        log << "Number of used colors is " << counter << " on " << nCol << " available" << std::endl;
        log << "Most used colors is " << max_i << " used " << max_c << " times" << std::endl;
        log << "Least used colors is " << min_i << " used " << min_c << " times" << std::endl << std::endl;
        log << "Average " << average << std::endl;
        log << "Variance " << variance << std::endl;
        log << "StandardDeviation " << std::sqrt(variance) << std::endl;
        log << "BalancingIndex " << balancingIndex << std::endl << std::endl;
        log << std::endl << "end colorazione finale -------------------------------------------------------------------"
            << std::endl << std::endl;
        std::ofstream cf(directory + "-colors.txt");
        for (size_t i = 0; i < coloring.size(); i++) cf << i << " " << coloring[i] << "\n";
    }

    const std::vector<uint32_t>& getColoring() const { return coloring; }
    const std::vector<uint64_t>& getTrajectory() const { return trajectory; }
    const std::vector<uint64_t>& getTailTrajectory() const { return tail; }
    const mcmc_run_stats& getStats() const { return stats; }

private:
    Graph<nodeW, edgeW>* graph;
    CurandStates* states;
    ColoringMCMCParams param;
    uint32_t tailMax;
    std::string directory;
    mcmc_ctx* ctx{nullptr};
    mcmc_run_stats stats{};
    std::vector<uint32_t> coloring;
    std::vector<uint64_t> trajectory, tail;
};

// ---- other colorers ------------------------------------------------------
// ColoringGreedyFF (graph_coloring/coloringGreedyFF.h / .cu): run(), getColoring()->nCol / colClass
// (1-based colours), saveStats / saveColor in the reference's report layout (:225-303).
struct Coloring {
    uint32_t nCol{0};
    const uint32_t* colClass{nullptr};
};

template <typename nodeW, typename edgeW>
class ColoringGreedyFF {
public:
    explicit ColoringGreedyFF(Graph<nodeW, edgeW>* graph_d) : graph(graph_d) {}
    void run() {
        colors.resize(graph->getNNodes());
        MCMC_CHECK(mcmc_greedyff_run(graph->handle(), colors.data(), &numColors, &rounds));
        coloring.nCol = numColors;
        coloring.colClass = colors.data();
    }
    Coloring* getColoring() { return &coloring; }
    uint32_t getRounds() const { return rounds; }
    void saveStats(size_t iteration, float duration, std::ofstream& file) const {
        file << "Greedy First Fit Colorer - GPU implementation - Report\n";
        file << "-------------------------------------------\n";
        file << "GRAPH INFO\n";
        file << "Nodes: " << graph->getNNodes() << " - Edges: " << graph->getNEdges() << "\n";
        file << "Max deg: " << graph->getMaxNodeDeg() << " - Min deg: " << graph->getMinNodeDeg()
             << " - Avg deg: " << graph->getMeanNodeDeg() << "\n";
        file << "Edge Probability (for randomly generated graphs): " << graph->prob << "\n";
        file << "-------------------------------------------\n";
        file << "EXECUTION INFO\n";
        file << "Repetition: " << iteration << "\n";
        file << "Execution time: " << duration << "\n";
        file << "-------------------------------------------\n";
        file << "Number of colors: " << numColors << "\n";
        file << "Color histogram: \n";
        // convert_to_standard_notation (:200-209): class sizes of colours 1..numColors
        std::vector<uint32_t> histogram(numColors, 0);
        for (uint32_t c : colors)
            if (c >= 1 && c <= numColors) histogram[c - 1]++;
        for (uint32_t i = 1; i < numColors + 1; ++i) file << i << "\t: " << histogram[i - 1] << "\n";
        int sum = 0;   // std::accumulate(.., 0): an int sum
        for (uint32_t h : histogram) sum += (int)h;
        const float mean = sum / static_cast<float>(numColors);
        float variance = 0;
        for (uint32_t h : histogram) variance += (h - mean) * (h - mean);
        variance /= static_cast<float>(numColors);
        file << "Average number of nodes for each color: " << mean << "\n";
        file << "Variance: " << variance << "\n";
        file << "StD: " << sqrtf(variance) << "\n";
    }
    void saveColor(std::ofstream& file) const {
        for (uint32_t i = 0; i < graph->getNNodes(); ++i) file << i << " " << colors[i] << "\n";
    }

private:
    Graph<nodeW, edgeW>* graph;
    std::vector<uint32_t> colors;
    uint32_t numColors{0}, rounds{0};
    Coloring coloring;
};

// ColoringLuby (graph_coloring/coloringLuby.h:17-68): ColoringLuby(Graph*, randStates), run_fast()
// (coloringLubyFast.cu:21-49), getColoringGPU()->nCol, saveStats / saveColor in the layout of
// coloringLuby.cu:151-215. randStates: the per-vertex XORWOW states (CurandStates), advanced.
template <typename nodeW, typename edgeW>
class ColoringLuby {
public:
    ColoringLuby(Graph<nodeW, edgeW>* graph_d, CurandStates* randStates) : graph(graph_d), states(randStates) {}
    void run_fast() {
        colors.resize(graph->getNNodes());
        MCMC_CHECK(mcmc_luby_run(graph->handle(), states->handle(), colors.data(), &numOfColors, &rounds));
        coloring.nCol = numOfColors;
        coloring.colClass = colors.data();
    }
    void run() { run_fast(); }
    Coloring* getColoringGPU() { return &coloring; }
    uint32_t getRounds() const { return rounds; }
    void saveStats(size_t it, float duration, std::ofstream& outFile) const {
        outFile << "Luby Colorer - GPU version - Report" << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "GRAPH INFO" << std::endl;
        outFile << "Nodes: " << graph->getNNodes() << " - Edges: " << graph->getNEdges() << std::endl;
        outFile << "Max deg: " << graph->getMaxNodeDeg() << " - Min deg: " << graph->getMinNodeDeg()
                << " - Avg deg: " << graph->getMeanNodeDeg() << std::endl;
        outFile << "Edge probability (for randomly generated graphs): " << graph->prob << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "EXECUTION INFO" << std::endl;
        outFile << "Repetition: " << it << std::endl;
        outFile << "Execution time: " << duration << std::endl;
        outFile << "-------------------------------------------" << std::endl;
        outFile << "Number of colors: " << numOfColors << std::endl;
        outFile << "Color histogram:" << std::endl;
        std::vector<size_t> histBins(numOfColors, 0);   // bins of colours 1..k, printed from index 0
        for (uint32_t c : colors) histBins[c - 1]++;
        for (size_t i = 0; i < histBins.size(); i++) outFile << i << ": " << histBins[i] << std::endl;
        int sum = 0;   // std::accumulate(.., 0): an int sum
        for (size_t h : histBins) sum += (int)h;
        const float mean = sum / (float)numOfColors;
        float variance = 0;
        for (size_t h : histBins) variance += ((h - mean) * (h - mean));
        variance /= (float)numOfColors;
        outFile << "Average number of nodes for each color: " << mean << std::endl;
        outFile << "Variance: " << variance << std::endl;
        outFile << "StD: " << sqrtf(variance) << std::endl;
    }
    void saveColor(std::ofstream& outfile) const {
        for (size_t i = 0; i < colors.size(); i++) outfile << i << " " << colors[i] << std::endl;
    }

private:
    Graph<nodeW, edgeW>* graph;
    CurandStates* states;
    std::vector<uint32_t> colors;
    uint32_t numOfColors{0}, rounds{0};
    Coloring coloring;
};

// ColoringVFF (graph_coloring/coloringVFF.h:8-48): ColoringVFF(Graph*), run() (greedy first fit,
// then the rebalancing), getColoring()->nCol / colClass, saveStats / saveColor in the layout of
// coloringVFF.cu:437-490 (saveStats prints "Valid result? (boolean)" = not_looping).
template <typename nodeW, typename edgeW>
class ColoringVFF {
public:
    explicit ColoringVFF(Graph<nodeW, edgeW>* graph_d) : graph(graph_d) {}
    void run() {
        colors.resize(graph->getNNodes());
        int v = 1;
        MCMC_CHECK(mcmc_vff_run(graph->handle(), colors.data(), &numColors, &iterations, &v));
        notLooping = v != 0;
        if (!notLooping) std::cout << "Rebalancing failed. Coloring resetted to Greedy First Fit.\n\n";
        coloring.nCol = numColors;
        coloring.colClass = colors.data();
    }
    Coloring* getColoring() { return &coloring; }
    uint32_t getIterations() const { return iterations; }
    bool isValid() const { return notLooping; }
    void saveStats(size_t iteration, float duration, std::ofstream& file) const {
        file << "Greedy FF Colorer followed by Vertex First Fit Rebalancing - GPU implementation - Report\n";
        file << "-------------------------------------------\n";
        file << "GRAPH INFO\n";
        file << "Nodes: " << graph->getNNodes() << " - Edges: " << graph->getNEdges() << "\n";
        file << "Max deg: " << graph->getMaxNodeDeg() << " - Min deg: " << graph->getMinNodeDeg()
             << " - Avg deg: " << graph->getMeanNodeDeg() << "\n";
        file << "Edge Probability (for randomly generated graphs): " << graph->prob << "\n";
        file << "-------------------------------------------\n";
        file << "EXECUTION INFO\n";
        file << "Repetition: " << iteration << "\n";
        file << "Execution time: " << duration << "\n";
        file << "Valid result? (boolean) " << notLooping << "\n";
        file << "-------------------------------------------\n";
        file << "Number of colors: " << numColors << "\n";
        file << "Color histogram: \n";
        std::vector<uint32_t> histogram(numColors, 0);   // convert_to_standard_notation's class sizes
        for (uint32_t c : colors)
            if (c >= 1 && c <= numColors) histogram[c - 1]++;
        for (uint32_t i = 1; i < numColors + 1; ++i) file << i << "\t: " << histogram[i - 1] << "\n";
        int sum = 0;   // std::accumulate(.., 0): an int sum
        for (uint32_t h : histogram) sum += (int)h;
        const float mean = sum / static_cast<float>(numColors);
        float variance = 0;
        for (uint32_t h : histogram) variance += (h - mean) * (h - mean);
        variance /= static_cast<float>(numColors);
        file << "Average number of nodes for each color: " << mean << "\n";
        file << "Variance: " << variance << "\n";
        file << "StD: " << sqrtf(variance) << "\n";
    }
    void saveColor(std::ofstream& file) const {
        for (uint32_t i = 0; i < graph->getNNodes(); ++i) file << i << " " << colors[i] << "\n";
    }

private:
    Graph<nodeW, edgeW>* graph;
    std::vector<uint32_t> colors;
    uint32_t numColors{0}, iterations{0};
    bool notLooping{true};
    Coloring coloring;
};
