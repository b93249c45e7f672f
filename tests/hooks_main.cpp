// tests/hooks_main.cpp -- drives ColoringMCMC_CPU's per-vertex hooks (include/mcmc_colorer.hpp, the
// reference's coloringMCMC_CPU.h:20-28) on a host-only graph, no GPU: loop 1 of run() vertex by
// vertex (coloringMCMC_CPU.cpp:183-204) with the draws given on stdin. tests/test_cpu_hooks.py
// compares the output with the oracle's one-vertex update.
// stdin:  n m nCol eps seed tabooIteration / n+1 offsets / m neighbours / n draws u
// stdout: "C0" n colours / per vertex "v viol Zvcomp newColour q bits(p[0..nCol))" / "violations k"
#include <cstring>

#include "mcmc_colorer.hpp"

int main() {
    size_t n, m;
    uint32_t nCol, seed, taboo;
    float eps;
    if (!(std::cin >> n >> m >> nCol >> eps >> seed >> taboo)) return 2;
    std::vector<uint64_t> off(n + 1);
    std::vector<node> nb(m);
    std::vector<float> u(n);
    for (auto& x : off) std::cin >> x;
    for (auto& x : nb) std::cin >> x;
    for (auto& x : u) std::cin >> x;
    Graph<float, float> g(Graph<float, float>::HostOnly{}, off, nb);
    ColoringMCMCParams params{250, nCol, 1.0f, 1.0f, eps, 0.01f, taboo, false};
    ColoringMCMC_CPU<float, float> cc(&g, params, seed);
    std::vector<uint32_t>& C = *cc.getC();
    std::cout << "C0";
    for (uint32_t c : C) std::cout << " " << c;
    std::cout << "\n";
    std::vector<bool>& viols = *cc.getCviols();
    const size_t k = cc.violation_count(C, viols);
    std::vector<uint32_t>& Cstar = *cc.getCstar();
    std::vector<float>& q = *cc.getq();
    for (size_t v = 0; v < n; v++) {   // loop 1 of run(): count_free_colors, fill_p, extract_new_color
        const size_t Zvcomp = cc.count_free_colors(v, C, *cc.getfreeColors());
        cc.fill_p(v, nCol - Zvcomp);
        cc.extract_new_color(v, *cc.getp(), u, q, Cstar);
        uint32_t qb;
        std::memcpy(&qb, &q[v], 4);
        std::cout << v << " " << (viols[v] ? 1 : 0) << " " << Zvcomp << " " << Cstar[v] << " " << qb;
        for (float x : *cc.getp()) {
            uint32_t b;
            std::memcpy(&b, &x, 4);
            std::cout << " " << b;
        }
        std::cout << "\n";
    }
    std::cout << "violations " << k << "\n";
    return 0;
}
