"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/mcmc_hip.h
declares, and its host-only entry points (glibc stream jump-ahead) agree with real glibc.
No compute call touches a GPU here."""
import re
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as O
from mcmc_colorer_amd import _lib

ROOT = Path(__file__).resolve().parent.parent
HEADER = (ROOT / "include" / "mcmc_hip.h").read_text()


def declared_symbols():
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(mcmc_\w+)\s*\(", HEADER, re.M)))


def test_header_symbols_are_bound():
    syms = declared_symbols()
    assert len(syms) >= 20
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s


def test_error_reporting_without_gpu():
    L = _lib.lib()
    assert L.mcmc_version() >= 1
    rc = L.mcmc_glibc_window(1, 0, None)
    assert rc == -1 and b"NULL" in L.mcmc_last_error()


@pytest.mark.parametrize("seed,draws", [(1, 0), (1, 7), (1, 310), (1, 99991), (5, 123456), (2**31 + 3, 4000001)])
def test_glibc_jump_matches_real_glibc(seed, draws):
    O.srand(seed)
    O.lib().oracle_rand_skip(draws)
    ref = O.rand(200)
    w = np.zeros(31, dtype=np.uint32)
    _lib.check(_lib.lib().mcmc_glibc_window(seed, draws, _lib.u32ptr(w)))
    out = np.zeros(200, dtype=np.uint32)
    _lib.check(_lib.lib().mcmc_glibc_draw(_lib.u32ptr(w), 200, _lib.u32ptr(out)))
    assert out.tolist() == ref
    # and the window advanced by 200 equals a direct jump to draws + 200
    w2 = np.zeros(31, dtype=np.uint32)
    _lib.check(_lib.lib().mcmc_glibc_window(seed, draws + 200, _lib.u32ptr(w2)))
    assert np.array_equal(w, w2)


def test_oracle_glibc_window_setter():
    """oracle_set_glibc_window (used to start the oracle at a jumped-to stream position)."""
    w = np.zeros(31, dtype=np.uint32)
    _lib.check(_lib.lib().mcmc_glibc_window(1, 5050, _lib.u32ptr(w)))
    O.srand(1)
    O.lib().oracle_rand_skip(5050)
    ref = O.rand(100)
    O.set_glibc_window(w)
    assert O.rand(100) == ref
