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
