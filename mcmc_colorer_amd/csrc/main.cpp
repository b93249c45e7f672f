// mcmc_colorer_amd/csrc/main.cpp -- `mcmc_colorer`, the --mcmcgpu command line of the reference
// (src/main.cu:28-215, src/utils/ArgHandle.cpp:25-308) on the MI355X colorer.
//
// Same options, defaults and output naming as the reference:
//   --graph FILE | --simulate P -n N, --mcmcgpu, --nCol N, --numColRatio R, --tabooIteration N,
//   --tailcut, --repet N, --seed N, --outDir D
//   --mcmcgpu-ref: the reference's own GPU colorer semantics (ColoringMCMC as built by default:
//   balance-dynamic proposal, cuRAND XORWOW per vertex, conflicts as edges, the GPU tail cut) on the
//   same sweep; outputs <graph>-MCMC_GPU-<i>.log in coloringMCMC_prints.cu's layout
//   --tailcutRepair: after the loop, run the reference's tail cut (coloringMCMC_CPU.cpp:272-311)
//   with its inner loop fixed (k++; the reference's never returns), at most 1000 passes
// Outputs <outDir>/<graphName>-MCMC_GPU-<i>.log and -colors.txt per repetition.
// --mcmccpu: ColoringMCMC_CPU's surface (-MCMC_CPU-<i> files, seed + i), run by the same HIP sweep --
// the CPU colorer's results, bit for bit (the oracle, oracle/build/mcmc_cpu_ref, is test infrastructure);
// --lubygpu (ColoringLuby), --grdffgpu (ColoringGreedyFF) and --vffgpu (ColoringVFF) write
// <graphName>-LUBY-<i> / -GFF-<i> / -VFF-<i> .log and -colors.txt.
#include <getopt.h>
#include <sys/stat.h>

#include <chrono>
#include <ctime>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_set>
#include <vector>

#include "mcmc_colorer.hpp"

namespace {

std::vector<std::string> split_str(const std::string& s, const std::string& delims) {
    std::vector<std::string> out;
    std::string cur;
    for (char ch : s) {
        if (delims.find(ch) != std::string::npos) { if (!cur.empty()) out.push_back(cur); cur.clear(); }
        else cur += ch;
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

// fileImporter (utils/fileImporter.cpp:5-66, 118-143) + Graph::setupImporterNew (graphCPU.cpp:112-170).
// Vertex ids follow std::unordered_set<std::string> iteration order (same libstdc++ => same ids);
// the first line is a header; self loops are dropped; both arc directions are added in file order.
bool import_edge_list(const std::string& path, std::vector<uint64_t>& cumulDegs, std::vector<node>& neighs) {
    std::ifstream f(path);
    if (!f) { std::cout << "Error opening graph file" << std::endl; return false; }
    std::string inStr, src, dst;
    float ww;
    std::stringstream ss;
    std::unordered_set<std::string> names;
    std::getline(f, inStr);
    while (f) {
        std::getline(f, inStr);
        if (inStr == "") continue;
        ss << inStr;
        ss >> src;
        ss >> dst;
        ss >> ww;
        names.insert(src);
        names.insert(dst);
        ss.str("");
        ss.clear();
    }
    std::map<std::string, int> geneMap;
    int i = 0;
    for (auto it = names.begin(); it != names.end(); ++it) geneMap.insert(std::pair<std::string, int>(*it, i++));
    const uint32_t nn = (uint32_t)names.size();
    // two passes over the edges, as setupImporterNew
    std::vector<std::pair<uint32_t, uint32_t>> edges;
    f.clear();
    f.seekg(0);
    std::getline(f, inStr);
    ss.str("");
    ss.clear();
    double ww_d;
    while (true) {
        do { std::getline(f, inStr); } while ((inStr == "") && f);
        if (!f) break;
        ss << inStr;
        ss >> src;
        ss >> dst;
        ss >> ww_d;
        edges.emplace_back((uint32_t)geneMap.at(src), (uint32_t)geneMap.at(dst));
        ss.str("");
        ss.clear();
    }
    cumulDegs.assign((size_t)nn + 1, 0);
    for (auto& e : edges)
        if (e.first != e.second) { cumulDegs[e.first + 1]++; cumulDegs[e.second + 1]++; }
    for (uint32_t v = 1; v < nn + 1; v++) cumulDegs[v] += cumulDegs[v - 1];
    neighs.assign(cumulDegs[nn], 0);
    std::vector<uint64_t> tmp(nn, 0);
    for (auto& e : edges) {
        if (e.first == e.second) continue;
        neighs[cumulDegs[e.first] + tmp[e.first]++] = e.second;
        neighs[cumulDegs[e.second] + tmp[e.second]++] = e.first;
    }
    return true;
}

void help(const char* argv0) {
    std::cout << "Usage: " << argv0 << " [options]\n"
              << "  --graph file.txt     edge list (header line, then 'src dst [weight]' per line)\n"
              << "  --simulate P -n N    Erdos-Renyi graph, the reference's generator replayed on the GPU\n"
              << "  --simulate-fast P -n N [--er-seed S]\n"
              << "                       G(n,p) from the build's counter-based generator (csrc/er_gen.h):\n"
              << "                       for n where the reference's O(n^2) generator is infeasible (1e7)\n"
              << "  --mcmcgpu            MCMC colorer on the MI355X (default)\n"
              << "  --mcmcgpu-ref        the reference's GPU colorer semantics (XORWOW, balance-dynamic)\n"
              << "  --mcmccpu            ColoringMCMC_CPU's outputs (-MCMC_CPU- files), computed by the same GPU sweep\n"
              << "  --grdffgpu           parallel greedy first-fit colorer (ColoringGreedyFF)\n"
              << "  --lubygpu            Luby independent-set colorer (ColoringLuby::run_fast)\n"
              << "  --vffgpu             greedy first fit + vertex-first-fit rebalancing (ColoringVFF)\n"
              << "  --nCol N             number of colours (default maxDeg / numColRatio)\n"
              << "  --numColRatio R      1.0 <= R <= 16.0 (default 1.0)\n"
              << "  --tabooIteration N   taboo iterations (default 0)\n"
              << "  --tailcut            stop at Cviol <= max(50, n/2000)\n"
              << "  --tailcutRepair      then repair the remaining conflicts (corrected tail cut, <= 1000 passes)\n"
              << "  --repet N            repetitions, seeds seed+i (default 1)\n"
              << "  --seed N             seed (default: time, which also srand()s glibc)\n"
              << "  --outDir D           output directory\n"
              << "  --device D           HIP device (default 0)\n"
              << "  --gpus N             --mcmcgpu vertex-partitioned over devices D .. D+N-1 of this node\n"
              << "  --loopback           with --gpus N: all N ranks on device D, exchanged by device copies (rehearsal)\n"
              << "                       (RCCL inside the library; arc-balanced plan for CSR graphs)\n";
}

}  // namespace

int main(int argc, char** argv) {
    std::string graphFilename, outDir;
    double prob = 0.0, numColRatio = 0.0;
    uint32_t n = 0, nCol = 0, seed = 0, repetitions = 1, tabooIteration = 0;
    bool simulate = false, mcmccpu = false, mcmcgpu = false, tailcut = false, fast = false,
         tailcutRepair = false, mcmcgpuref = false, greedyff = false, lubygpu = false, vffgpu = false;
    uint64_t erSeed = 1;
    int device = 0, gpus = 1;
    bool loopback = false;
    const struct option longopts[] = {
        {"graph", required_argument, 0, 'g'},    {"outDir", required_argument, 0, 'o'},
        {"simulate", required_argument, 0, 's'}, {"nodes", required_argument, 0, 'n'},
        {"mcmccpu", no_argument, 0, '1'},        {"mcmcgpu", no_argument, 0, '2'},
        {"lubygpu", no_argument, 0, '3'},        {"grdffgpu", no_argument, 0, '4'},
        {"vffgpu", no_argument, 0, '5'},         {"nCol", required_argument, 0, 'k'},
        {"numColRatio", required_argument, 0, 'r'}, {"tabooIteration", required_argument, 0, 't'},
        {"tailcut", no_argument, 0, 'l'},        {"repet", required_argument, 0, 'R'},
        {"seed", required_argument, 0, 'S'},     {"help", no_argument, 0, 'h'},
        {"device", required_argument, 0, 'D'},   {"simulate-fast", required_argument, 0, 'F'},
        {"er-seed", required_argument, 0, 'E'},  {"tailcutRepair", no_argument, 0, 'X'},
        {"mcmcgpu-ref", no_argument, 0, 'G'},    {"gpus", required_argument, 0, 'P'}, {"loopback", no_argument, 0, 'L'},
        {0, 0, 0, 0}};
    int c;
    while ((c = getopt_long(argc, argv, "g:o:s:n:12345k:r:t:lR:S:hD:", longopts, nullptr)) != -1) {
        try {
            switch (c) {
                case 'g': graphFilename = optarg; break;
                case 'o': outDir = optarg; break;
                case 's': simulate = true; prob = std::stod(optarg);
                          if (prob < 0 || prob > 1) { std::cout << "Simulation: probabilty of positive class must be 0 < prob < 1." << std::endl; return 255; }
                          break;
                case 'n': if (std::stoi(optarg) < 1) throw 1; n = std::stoi(optarg); break;
                case '1': mcmccpu = true; break;
                case '2': mcmcgpu = true; break;
                case '4': greedyff = true; break;
                case '3': lubygpu = true; break;
                case '5': vffgpu = true; break;
                case 'k': if (std::stoi(optarg) < 1) throw 1; nCol = std::stoi(optarg); break;
                case 'r': numColRatio = std::stod(optarg); if (numColRatio < 1.0 || numColRatio > 16.0) throw 1; break;
                case 't': if (std::stoi(optarg) < 1) throw 1; tabooIteration = std::stoi(optarg); break;
                case 'l': tailcut = true; break;
                case 'R': if (std::stoi(optarg) < 1) throw 1; repetitions = std::stoi(optarg); break;
                case 'S': seed = (uint32_t)std::stoi(optarg); break;
                case 'D': device = std::stoi(optarg); break;
                case 'F': simulate = fast = true; prob = std::stod(optarg);
                          if (prob < 0 || prob > 1) { std::cout << "Simulation: probabilty of positive class must be 0 < prob < 1." << std::endl; return 255; }
                          break;
                case 'E': erSeed = std::stoull(optarg); break;
                case 'X': tailcutRepair = true; break;
                case 'G': mcmcgpuref = true; break;
                case 'P': if (std::stoi(optarg) < 1) throw 1; gpus = std::stoi(optarg); break;
                case 'L': loopback = true; break;
                case 'h': help(argv[0]); return 0;
                default: break;
            }
        } catch (...) {
            std::cout << "invalid argument for option -" << (char)c << std::endl;
            return 255;
        }
    }
    if (!simulate && graphFilename.empty()) {
        std::cout << "Graph file undefined (--graph). Specify a graph file or enable simulation mode." << std::endl;
        return 255;
    }
    if (mcmcgpu && mcmcgpuref) {
        std::cout << "--mcmcgpu and --mcmcgpu-ref write the same files: choose one" << std::endl;
        return 255;
    }
    if (!mcmcgpu && !mcmcgpuref && !mcmccpu && !greedyff && !lubygpu && !vffgpu) {
        std::cout << "No coloring algorithm specified: enabling MCMC GPU (--mcmcgpu)" << std::endl;
        mcmcgpu = true;
    }
    if (simulate && n == 0) { std::cout << "Simualtion enabled: specify the number of nodes (-n)." << std::endl; return 255; }
    if (numColRatio == 0.0) numColRatio = 1.0;
    if (seed == 0) {                                              // ArgHandle.cpp:272-276
        seed = (uint32_t)time(NULL);
        std::cout << "No seed specified. Generating a random seed: " << seed << " (--seed)." << std::endl;
        mcmc::glibc_srand(seed);
    }
    std::string graphName;
    if (!simulate) {
        auto justFilename = split_str(graphFilename, "/\\");
        auto parts = split_str(justFilename.back(), ".");
        if (parts.size() > 1) {
            graphName = parts[0];
            for (size_t i = 1; i + 1 < parts.size(); i++) graphName += "." + parts[i];
        } else {
            graphName = parts[0];
        }
    } else {
        graphName = std::to_string(n) + "_" + std::to_string(prob) + "_" + std::to_string(numColRatio);
        if (fast) graphName += "_er" + std::to_string(erSeed);
    }
    if (outDir.empty()) outDir = graphName + "_out";
    mkdir(outDir.c_str(), 0775);

    const float numColorRatio = 1.0f / (float)numColRatio;        // main.cu:53
    if (gpus > 1 && (mcmcgpuref || mcmccpu || greedyff || lubygpu || vffgpu)) {
        std::cout << "--gpus > 1 partitions --mcmcgpu only (no --mcmcgpu-ref, --mcmccpu or other colorers)" << std::endl;
        return 255;
    }
    Graph<float, float>* g;
    std::vector<Graph<float, float>*> parts;   // --gpus N: one graph per device, rank order
    std::vector<uint32_t> bounds;
    auto t0 = std::chrono::steady_clock::now();
    if (fast) {
        if (gpus > 1) {   // every rank generates only its rows (G(n,p) is uniform: equal rows)
            bounds.resize((size_t)gpus + 1);
            MCMC_CHECK(mcmc_part_plan_rows(n, (uint32_t)gpus, bounds.data()));
            for (int r = 0; r < gpus; r++)
                parts.push_back(new Graph<float, float>(Graph<float, float>::ErFast{}, n, (float)prob, erSeed,
                                                        device + (loopback ? 0 : r), bounds[r], bounds[r + 1]));
            Graph<float, float>::mergePartitionStats(parts);   // default nCol and reports: whole-graph stats
            g = parts[0];
        } else {
            g = new Graph<float, float>(Graph<float, float>::ErFast{}, n, (float)prob, erSeed, device);
        }
    } else if (simulate) {
        const mcmc::GlibcWindow w0 = mcmc::glibc_global();
        for (int r = 0; r < gpus; r++) {   // the exact graph on every device, from the same stream position
            mcmc::glibc_global() = w0;
            parts.push_back(new Graph<float, float>(n, (float)prob, seed, device + (loopback ? 0 : r)));
        }
        g = parts[0];
    } else {
        std::vector<uint64_t> off;
        std::vector<node> idx;
        if (!import_edge_list(graphFilename, off, idx)) return 255;
        const uint32_t nn = (uint32_t)(off.size() - 1);
        const float p = (float)idx.size() / (float)(nn * nn);      // main.cu:68 (uint32 product, as the reference)
        for (int r = 0; r < gpus; r++) parts.push_back(new Graph<float, float>(off, idx, p, device + (loopback ? 0 : r)));
        g = parts[0];
    }
    if (gpus > 1 && bounds.empty()) {   // CSR graphs: arc-balanced plan from the degree prefix
        bounds.resize((size_t)gpus + 1);
        MCMC_CHECK(mcmc_part_plan(g->handle(), (uint32_t)gpus, 1, bounds.data()));
    }
    if (gpus == 1) parts.clear();
    const double tgen = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "Nodes: " << g->getNNodes() << " - Edges: " << g->getNEdges() << std::endl;
    std::cout << "Min Degree: " << g->getMinNodeDeg() << " - Max Degree: " << g->getMaxNodeDeg()
              << " - Mean Degree: " << g->getMeanNodeDeg() << "  (graph ready in " << tgen << " s)" << std::endl;

    GPURand GPURandGen(g->getNNodes(), (long)seed);
    CurandStates* curand = (mcmcgpuref || lubygpu) ? new CurandStates(g->getNNodes(), (long)seed, device) : nullptr;   // main.cu:80
    for (uint32_t i = 0; i < repetitions; i++) {
        std::cout << "Repetition: " << i << std::endl;
        if (lubygpu) {   // main.cu:89-109 (first: it advances the shared states)
            ColoringLuby<float, float> colLuby(g, curand);
            const auto s0 = std::chrono::steady_clock::now();
            colLuby.run_fast();
            const double duration = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
            std::cout << "LubyGPU - number of colors: " << colLuby.getColoringGPU()->nCol << std::endl;
            std::cout << "LubyGPU elapsed time: " << duration << std::endl;
            std::ofstream lubyFileLog(outDir + "/" + graphName + "-LUBY-" + std::to_string(i) + ".log");
            colLuby.saveStats(i, (float)duration, lubyFileLog);
            std::ofstream lubyFileColors(outDir + "/" + graphName + "-LUBY-" + std::to_string(i) + "-colors.txt");
            colLuby.saveColor(lubyFileColors);
        }
        if (greedyff) {   // main.cu:111-132
            ColoringGreedyFF<float, float> greedy(g);
            const auto s0 = std::chrono::steady_clock::now();
            greedy.run();
            const double duration = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
            std::cout << "Parallel Greedy First Fit - number of colors: " << greedy.getColoring()->nCol << std::endl;
            std::cout << "Parallel Greedy First Fit - elapsed time: " << duration << std::endl;
            std::ofstream gffFileLog(outDir + "/" + graphName + "-GFF-" + std::to_string(i) + ".log");
            greedy.saveStats(i, (float)duration, gffFileLog);
            std::ofstream gffFileColors(outDir + "/" + graphName + "-GFF-" + std::to_string(i) + "-colors.txt");
            greedy.saveColor(gffFileColors);
        }
        if (vffgpu) {   // main.cu:134-158
            ColoringVFF<float, float> balanced(g);
            const auto s0 = std::chrono::steady_clock::now();
            balanced.run();
            const double duration = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
            std::cout << "Vertex-centric First Fit rebalancing after Greedy FF coloring - number of colors: " << balanced.getColoring()->nCol << std::endl;
            std::cout << "Vertex-centric First Fit rebalancing after Greedy FF coloring - elapsed time: " << duration << std::endl;
            std::ofstream vffFileLog(outDir + "/" + graphName + "-VFF-" + std::to_string(i) + ".log");
            balanced.saveStats(i, (float)duration, vffFileLog);
            std::ofstream vffFileColors(outDir + "/" + graphName + "-VFF-" + std::to_string(i) + "-colors.txt");
            balanced.saveColor(vffFileColors);
        }
        if (!mcmcgpu && !mcmcgpuref && !mcmccpu) continue;
        ColoringMCMCParams params;                                   // main.cu:160-168
        params.numColorRatio = numColorRatio;
        params.nCol = (nCol != 0) ? nCol : (col_sz)(g->getMaxNodeDeg() * numColorRatio);
        params.epsilon = 1e-8f;
        params.lambda = 1.0f;
        params.ratioFreezed = 1e-2f;
        params.maxRip = 250;
        params.tabooIteration = tabooIteration;
        params.tailcut = tailcut;
        params.tailcutRepair = tailcutRepair ? 1000u : 0u;
        if (mcmccpu) {   // main.cu:170-190: before the GPU colorer, on the same glibc stream
            ColoringMCMC_CPU<float, float> mcmcCpu(g, params, seed + i);
            const auto s0 = std::chrono::steady_clock::now();
            mcmcCpu.run();
            const float duration = (float)std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
            std::cout << "MCMC_CPU elapsed time: " << duration << std::endl;
            std::ofstream cpuFileLog(outDir + "/" + graphName + "-MCMC_CPU-" + std::to_string(i) + ".log");
            mcmcCpu.saveStats(i, duration, cpuFileLog);
            std::ofstream cpuFileColors(outDir + "/" + graphName + "-MCMC_CPU-" + std::to_string(i) + "-colors.txt");
            mcmcCpu.saveColor(cpuFileColors);
        }
        if (!mcmcgpu && !mcmcgpuref) continue;
        if (mcmcgpuref) {
            ColoringMCMCGpuRef<float, float> colRef(g, curand, params);
            colRef.setDirectoryPath(outDir + "/" + graphName + "-MCMC_GPU-" + std::to_string(i));
            colRef.run((int)i);
            const auto& st = colRef.getStats();
            std::cout << "MCMC GPU elapsed time: " << st.loopMs / 1000.0 << " (" << st.sweepsRun
                      << " sweeps, final conflicting edges " << st.finalViol
                      << (st.maxIterReached ? ", max iteration reached" : "") << ")" << std::endl << std::endl;
            continue;
        }
        std::unique_ptr<ColoringMCMC<float, float>> colPtr(
            gpus > 1 ? new ColoringMCMC<float, float>(parts, bounds, GPURandGen.randStates, params)
                     : new ColoringMCMC<float, float>(g, GPURandGen.randStates, params));
        ColoringMCMC<float, float>& colMCMC = *colPtr;
        colMCMC.setDirectoryPath(outDir + "/" + graphName + "-MCMC_GPU-" + std::to_string(i));
        colMCMC.run((int)i);
        const auto& st = colMCMC.getStats();
        std::cout << "MCMC GPU elapsed time: " << st.loopMs / 1000.0 << " (" << st.iter << " sweeps, final conflicts "
                  << st.finalViol << (st.maxIterReached ? ", max iteration reached" : "");
        if (tailcutRepair) std::cout << ", " << st.tailcutPasses << " tail-cut passes";
        std::cout << ")" << std::endl
                  << std::endl;
    }
    delete curand;
    if (parts.empty()) delete g;
    for (auto* pg : parts) delete pg;
    return EXIT_SUCCESS;
}
