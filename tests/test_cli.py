"""The product CLI (`mcmc_colorer --mcmcgpu`, C++ over the C ABI) against the oracle CLI
(`oracle/build/mcmc_cpu_ref`, the --mcmccpu restatement) on the reference's command lines:
same graph, same colours file, same "Iteration performed" per repetition."""
import random
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CLI = ROOT / "mcmc_colorer_amd" / "mcmc_colorer"
ORACLE = ROOT / "oracle" / "build" / "mcmc_cpu_ref"


def test_cli_help_without_gpu():
    assert CLI.exists(), "build the CLI: python -m mcmc_colorer_amd.build"
    r = subprocess.run([str(CLI), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--simulate" in r.stdout


def run_pair(tmp_path, args, name, repet=1):
    po, oo = tmp_path / "gpu", tmp_path / "cpu"
    r1 = subprocess.run([str(CLI), "--mcmcgpu", *args, "--outDir", str(po)], capture_output=True, text=True,
                        timeout=600)
    assert r1.returncode == 0, r1.stdout + r1.stderr
    r2 = subprocess.run([str(ORACLE), "--mcmccpu", *args, "--outDir", str(oo)], capture_output=True, text=True,
                        timeout=600)
    assert r2.returncode == 0, r2.stdout + r2.stderr
    for i in range(repet):
        g = (po / f"{name}-MCMC_GPU-{i}-colors.txt").read_text()
        c = (oo / f"{name}-MCMC_CPU-{i}-colors.txt").read_text()
        assert g == c, f"repetition {i}: colours differ"
        it = [re.search(r"Iteration performed: (\d+)", (d / f"{name}-MCMC_{k}-{i}.log").read_text()).group(1)
              for d, k in ((po, "GPU"), (oo, "CPU"))]
        assert it[0] == it[1]


@pytest.mark.gpu
def test_cli_simulate_c1(tmp_path):
    """BASELINE.json configs[0] command line, --seed 1."""
    run_pair(tmp_path, ["--simulate", "0.1", "-n", "1000", "--seed", "1"], "1000_0.100000_1.000000")


@pytest.mark.gpu
def test_cli_tailcut_repair(tmp_path):
    """--tailcut --tailcutRepair: the loop stops within z, the corrected tail cut repairs the rest."""
    run_pair(tmp_path, ["--simulate", "0.02", "-n", "2500", "--nCol", "24", "--tailcut", "--tailcutRepair",
                        "--seed", "1"], "2500_0.020000_1.000000")


@pytest.mark.gpu
def test_cli_simulate_repetitions_taboo_ratio(tmp_path):
    run_pair(tmp_path, ["--simulate", "0.05", "-n", "1500", "--numColRatio", "2.5", "--tabooIteration", "2",
                        "--repet", "3", "--seed", "7"], "1500_0.050000_2.500000", repet=3)


@pytest.mark.gpu
def test_cli_graph_file(tmp_path):
    """--graph: string vertex names (ids in unordered_set order), duplicates, self loops, blank lines."""
    rnd = random.Random(5)
    names = [f"g{rnd.randrange(10**6):06d}" for _ in range(700)]
    lines = ["src\tdst\tweight"]
    for _ in range(9000):
        a, b = rnd.choice(names), rnd.choice(names)
        lines.append(f"{a}\t{b}\t{rnd.random():.3f}")
        if rnd.random() < 0.01:
            lines.append("")
    f = tmp_path / "mygraph.edges.txt"
    f.write_text("\n".join(lines) + "\n")
    run_pair(tmp_path, ["--graph", str(f), "--nCol", "24", "--seed", "11", "--repet", "2"], "mygraph.edges", repet=2)


@pytest.mark.gpu
def test_cli_simulate_fast(tmp_path):
    """--simulate-fast (the build's G(n,p) generator, two column blocks): the colours file equals the
    oracle's run on the restated graph (seed 5, 16 colours, maxRip 250 -> 251 sweeps)."""
    import oracle_ref as O

    n, p, seed = 70000, 0.002, 5
    r1 = subprocess.run([str(CLI), "--mcmcgpu", "--simulate-fast", str(p), "-n", str(n), "--er-seed", "3",
                         "--nCol", "16", "--seed", str(seed), "--outDir", str(tmp_path)],
                        capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stdout + r1.stderr
    name = f"{n}_{p:.6f}_1.000000_er3"
    got = (tmp_path / f"{name}-MCMC_GPU-0-colors.txt").read_text().split("\n")
    off, idx = O.er_fast(n, p, 3)
    O.srand(1)      # --seed S leaves glibc unseeded (ArgHandle.cpp:272-276); the generator draws none
    r = O.mcmc_run(off, idx, 16, seed, nthreads=8)
    want = [f"{v} {c}" for v, c in enumerate(r.colors.tolist())]
    assert [l for l in got if l] == want


@pytest.mark.gpu
def test_cli_mcmcgpu_ref(tmp_path):
    """--mcmcgpu-ref: the reference's GPU colorer semantics, two repetitions sharing the XORWOW
    states (main.cu:80,193), with the GPU tail cut; colours against the oracle's restatement, the
    log in coloringMCMC_prints.cu's layout."""
    import numpy as np

    import oracle_ref as O

    out = tmp_path / "o"
    r = subprocess.run([str(CLI), "--mcmcgpu-ref", "--simulate", "0.1", "-n", "1000", "--seed", "1", "--repet", "2",
                        "--tailcut", "--outDir", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    O.srand(1)
    off, idx = O.setup_rnd2(1000, 0.1)
    st = O.gpurand_init(1000, 1)
    name = "1000_0.100000_1.000000"
    for i in range(2):
        res = O.mcmc_gpu_run(off, idx, O.max_deg(off), st, tailcut=True)
        got = (out / f"{name}-MCMC_GPU-{i}-colors.txt").read_text().split("\n")
        assert [int(x.split()[1]) for x in got if x] == res.colors.tolist()
        log = (out / f"{name}-MCMC_GPU-{i}.log").read_text()
        assert f"numCol: {O.max_deg(off)}" in log and "COLORAZIONE FINALE" in log
        assert f"conflitti rilevati: {res.traj[0]}" in log
        assert log.count("***** Tentativo numero:") == res.res.sweeps + res.res.tailcutPasses
        assert ("---> TailCutting" in log) == (res.res.tailcutPasses > 0)
        assert f"Max iteration reached {'yes' if res.res.maxIterReached else 'no'}" in log


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--mcmcgpu"]])
def test_cli_mcmccpu_surface(tmp_path, extra):
    """--mcmccpu through the product (ColoringMCMC_CPU's surface, run by the HIP sweep) writes the
    oracle CLI's -MCMC_CPU- files: colours and the whole report except the wall time, for every
    repetition (seed + i, one glibc stream); with --mcmcgpu beside it the CPU colorer runs first."""
    args = ["--simulate", "0.05", "-n", "1500", "--nCol", "20", "--tabooIteration", "1", "--repet", "2", "--seed", "3"]
    po, oo = tmp_path / "gpu", tmp_path / "cpu"
    r1 = subprocess.run([str(CLI), "--mcmccpu", *extra, *args, "--outDir", str(po)], capture_output=True, text=True,
                        timeout=600)
    assert r1.returncode == 0, r1.stdout + r1.stderr
    assert "MCMC_CPU elapsed time" in r1.stdout
    r2 = subprocess.run([str(ORACLE), "--mcmccpu", *args, "--outDir", str(oo)], capture_output=True, text=True,
                        timeout=600)
    assert r2.returncode == 0, r2.stdout + r2.stderr
    name = "1500_0.050000_1.000000"
    strip = lambda t: re.sub(r"Execution time: .*", "", t)
    for i in range(2):
        assert (po / f"{name}-MCMC_CPU-{i}-colors.txt").read_text() == (oo / f"{name}-MCMC_CPU-{i}-colors.txt").read_text()
        assert strip((po / f"{name}-MCMC_CPU-{i}.log").read_text()) == strip((oo / f"{name}-MCMC_CPU-{i}.log").read_text())
        assert (po / f"{name}-MCMC_GPU-{i}.log").exists() == bool(extra)


def _run_cli(out, args):
    r = subprocess.run([str(CLI), "--mcmcgpu", *args, "--outDir", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--tailcut", "--tailcutRepair"]])
def test_cli_gpus_loopback_equals_one_gpu(tmp_path, extra):
    """--gpus 3 --loopback --simulate-fast (every rank generates only its own rows, all three on the
    one device): default nCol, report and colours equal the one-GPU run's -- the whole graph's
    statistics (maxDeg/minDeg/Edges from every rank's rows, not rank 0's), and with
    --tailcut --tailcutRepair the partitioned tail cut."""
    n, p = 70000, 0.002
    args = ["--simulate-fast", str(p), "-n", str(n), "--er-seed", "3", "--seed", "5", *extra]
    out1 = _run_cli(tmp_path / "one", args)
    out3 = _run_cli(tmp_path / "three", [*args, "--gpus", "3", "--loopback"])
    name = f"{n}_{p:.6f}_1.000000_er3"
    for suffix in ("-MCMC_GPU-0-colors.txt",):
        assert (tmp_path / "one" / (name + suffix)).read_text() == (tmp_path / "three" / (name + suffix)).read_text()
    strip = lambda t: [l for l in t.splitlines() if not l.startswith("Execution time")]
    assert strip((tmp_path / "one" / f"{name}-MCMC_GPU-0.log").read_text()) == \
        strip((tmp_path / "three" / f"{name}-MCMC_GPU-0.log").read_text())
    deg = lambda o: re.search(r"Min Degree: (\d+) - Max Degree: (\d+)", o).groups()
    assert deg(out1) == deg(out3)
    assert re.search(r"Edges: (\d+)", out1).group(1) == re.search(r"Edges: (\d+)", out3).group(1)
