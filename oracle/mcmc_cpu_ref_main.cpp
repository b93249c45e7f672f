// oracle/mcmc_cpu_ref_main.cpp -- TEST INFRASTRUCTURE ONLY.
// `--mcmccpu` command line of the reference (src/main.cu:28-215, src/utils/ArgHandle.cpp:25-308)
// driving the oracle restatement. Used to produce golden fixtures and CPU baselines.
//
// Deviations, all documented in DESIGN.md: no easylogging / no debugger hook; the tail cut stops
// and reports instead of hanging (coloringMCMC_CPU.cpp:296) unless --tailcutRepair is given;
// --threads N selects the bit-identical OpenMP variant; --trajectory FILE dumps per-sweep Cviol.
#include <getopt.h>
#include <sys/stat.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_set>
#include <cstdlib>
#include <ctime>
#include <string>
#include <vector>

#include "mcmc_cpu_ref.h"

// fileImporter (utils/fileImporter.cpp:5-66, 118-143) + setupImporterNew (graph/graphCPU.cpp:112-170):
// ids in std::unordered_set<std::string> iteration order, header line skipped, self loops dropped,
// both arc directions in file order.
static bool import_graph(const std::string& path, std::vector<uint64_t>& cumulDegs, std::vector<uint32_t>& neighs) {
    std::ifstream graphFile(path);
    if (!graphFile) return false;
    std::string inStr, src, dst;
    float ww;
    double ww_d;
    std::stringstream ss;
    std::unordered_set<std::string> tempGeneNamesSet;
    std::getline(graphFile, inStr);
    while (graphFile) {
        std::getline(graphFile, inStr);
        if (inStr == "") continue;
        ss << inStr;
        ss >> src;
        ss >> dst;
        ss >> ww;
        tempGeneNamesSet.insert(src);
        tempGeneNamesSet.insert(dst);
        ss.str("");
        ss.clear();
    }
    std::map<std::string, int> geneMap;
    int i = 0;
    for (auto it = tempGeneNamesSet.begin(); it != tempGeneNamesSet.end(); ++it)
        geneMap.insert(std::pair<std::string, int>(*it, i++));
    const uint32_t nn = (uint32_t)tempGeneNamesSet.size();
    cumulDegs.assign((size_t)nn + 1, 0);
    for (int pass = 0; pass < 2; pass++) {
        std::vector<uint64_t> tempDegs(nn, 0);
        graphFile.clear();
        graphFile.seekg(0);
        std::getline(graphFile, inStr);
        ss.str("");
        ss.clear();
        while (true) {
            do { std::getline(graphFile, inStr); } while ((inStr == "") && graphFile);
            if (!graphFile) break;
            ss << inStr;
            ss >> src;
            ss >> dst;
            ss >> ww_d;
            const uint32_t s_ = geneMap.at(src), d_ = geneMap.at(dst);
            ss.str("");
            ss.clear();
            if (s_ == d_) continue;
            if (pass == 0) {
                cumulDegs[s_ + 1]++;
                cumulDegs[d_ + 1]++;
            } else {
                neighs[cumulDegs[s_] + tempDegs[s_]++] = d_;
                neighs[cumulDegs[d_] + tempDegs[d_]++] = s_;
            }
        }
        if (pass == 0) {
            for (uint32_t v = 1; v < nn + 1; v++) cumulDegs[v] += cumulDegs[v - 1];
            neighs.assign(cumulDegs[nn], 0);
        }
    }
    return true;
}

int main(int argc, char** argv) {
    std::string outDir, trajFile, graphFile;
    double prob = 0.0, numColRatio = 0.0;
    uint32_t n = 0, nCol = 0, seed = 0, repet = 1, taboo = 0;
    bool simulate = false, tailcut = false, tailcutRepair = false;
    int threads = 1, sweepLimit = 0;
    const struct option longopts[] = {
        {"outDir", required_argument, 0, 'o'},   {"simulate", required_argument, 0, 's'},
        {"nodes", required_argument, 0, 'n'},    {"mcmccpu", no_argument, 0, '1'},
        {"nCol", required_argument, 0, 'k'},     {"numColRatio", required_argument, 0, 'r'},
        {"tabooIteration", required_argument, 0, 't'}, {"tailcut", no_argument, 0, 'l'},
        {"repet", required_argument, 0, 'R'},    {"seed", required_argument, 0, 'S'},
        {"threads", required_argument, 0, 'T'},  {"trajectory", required_argument, 0, 'J'},
        {"tailcutRepair", no_argument, 0, 'X'},  {"sweepLimit", required_argument, 0, 'L'},
        {"graph", required_argument, 0, 'g'},
        {0, 0, 0, 0}};
    int c;
    while ((c = getopt_long(argc, argv, "o:s:n:1k:r:t:lR:S:T:J:XL:g:", longopts, nullptr)) != -1) {
        switch (c) {
            case 'o': outDir = optarg; break;
            case 's': simulate = true; prob = std::stod(optarg); break;
            case 'n': n = std::stoi(optarg); break;
            case '1': break;
            case 'k': nCol = std::stoi(optarg); break;
            case 'r': numColRatio = std::stod(optarg); break;
            case 't': taboo = std::stoi(optarg); break;
            case 'l': tailcut = true; break;
            case 'R': repet = std::stoi(optarg); break;
            case 'S': seed = std::stoi(optarg); break;
            case 'T': threads = std::stoi(optarg); break;
            case 'J': trajFile = optarg; break;
            case 'X': tailcutRepair = true; break;
            case 'L': sweepLimit = std::stoi(optarg); break;
            case 'g': graphFile = optarg; break;
            default: return 2;
        }
    }
    if ((!simulate || n == 0) && graphFile.empty()) { fprintf(stderr, "need --simulate P -n N or --graph FILE\n"); return 2; }
    if (numColRatio == 0.0) numColRatio = 1.0;
    if (seed == 0) { seed = (uint32_t)time(NULL); srand(seed); }          // ArgHandle.cpp:272-276
    std::string graphName = std::to_string(n) + "_" + std::to_string(prob) + "_" + std::to_string(numColRatio);
    if (!simulate) {   // ArgHandle.cpp:289-298: file name without its last extension
        std::string base = graphFile.substr(graphFile.find_last_of("/\\") == std::string::npos ? 0 : graphFile.find_last_of("/\\") + 1);
        const size_t dot = base.find_last_of('.');
        graphName = (dot == std::string::npos || dot == 0) ? base : base.substr(0, dot);
    }
    if (outDir.empty()) outDir = graphName + "_out";
    mkdir(outDir.c_str(), 0775);

    uint64_t *off = nullptr, m = 0;
    uint32_t* idx = nullptr;
    std::vector<uint64_t> offv;
    std::vector<uint32_t> idxv;
    if (simulate) {
        if (oracle_setup_rnd2(n, (float)prob, &off, &idx, &m) != 0) return 1;
    } else {
        if (!import_graph(graphFile, offv, idxv)) { fprintf(stderr, "Error opening graph file\n"); return 1; }
        n = (uint32_t)(offv.size() - 1);
        m = idxv.size();
        off = offv.data();
        idx = idxv.data();
        prob = (float)m / (float)(n * n);                                 // main.cu:68
    }
    uint32_t maxDeg = oracle_max_deg(n, off), minDeg = n;
    for (uint32_t v = 0; v < n; v++) minDeg = std::min<uint32_t>(minDeg, (uint32_t)(off[v + 1] - off[v]));
    printf("Nodes: %u - Edges: %llu\n", n, (unsigned long long)m);

    const float numColorRatio = 1.0f / (float)numColRatio;                // main.cu:53
    oracle_params prm{};
    prm.numColorRatio = numColorRatio;
    prm.nCol = nCol != 0 ? nCol : (uint32_t)(maxDeg * numColorRatio);    // main.cu:162
    prm.epsilon = 1e-8f;
    prm.lambda = 1.0f;
    prm.ratioFreezed = 1e-2f;
    prm.maxRip = 250;
    prm.tabooIteration = taboo;
    prm.tailcut = tailcut;
    prm.tailcutRepair = tailcutRepair;

    std::vector<uint32_t> colors(n);
    std::vector<uint64_t> traj(prm.maxRip + 2);
    for (uint32_t i = 0; i < repet; i++) {
        oracle_result res{};
        auto t0 = std::clock();
        oracle_mcmc_run(n, off, idx, &prm, seed + i, nullptr, colors.data(), traj.data(), traj.size(),
                        sweepLimit, threads, &res);
        double duration = (std::clock() - t0) / (double)CLOCKS_PER_SEC;
        printf("MCMC_CPU elapsed time: %g (loop %.6f s, %u sweeps, final Cviol %llu)\n", duration, res.loopSeconds,
               res.sweepsRun, (unsigned long long)res.finalViol);
        std::string base = outDir + "/" + graphName + "-MCMC_CPU-" + std::to_string(i);
        oracle_save_outputs((base + ".log").c_str(), (base + "-colors.txt").c_str(), n, m, maxDeg, minDeg,
                            (float)m / (float)n, (float)prob, seed + i, i, (float)duration, &prm, &res, colors.data());
        if (!trajFile.empty()) {
            FILE* f = fopen((trajFile + "." + std::to_string(i)).c_str(), "w");
            for (uint64_t k = 0; k < res.trajLen; k++) fprintf(f, "%llu\n", (unsigned long long)traj[k]);
            fclose(f);
        }
    }
    if (simulate) {
        oracle_free(off);
        oracle_free(idx);
    }
    return 0;
}
