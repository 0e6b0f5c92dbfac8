"""The oracle (CPU restatement) pinned against the reference's own outputs.

* golden vectors in tests/golden/ were produced by the REFERENCE sources
  compiled where they lie (oracle/make_golden.py, oracle/_ref);
* known-answer properties of the reference fixtures matrix/test/*.mtx;
* when oracle/_ref is present, random instances against the live reference.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, golden_names, load_golden


def csr_of(g):
    m = int(g["m"])
    return (m,) + oracle.coo_to_csr(m, g["row"], g["col"], g["val"])


@pytest.mark.parametrize("name", golden_names())
def test_crs_matches_reference_bitwise(name):
    g = load_golden(name)
    m, rp, idx, val = csr_of(g)
    y = oracle.csr_spmv(rp, idx, val, g["x"])
    assert np.array_equal(y, g["y_crs"]), "opt_crs restatement differs from the reference"


@pytest.mark.parametrize("name", golden_names())
def test_format_restatements_match_reference(name):
    g = load_golden(name)
    m, n = int(g["m"]), int(g["n"])
    _, rp, idx, val = csr_of(g)
    if "y_ell" in g:
        K, y = oracle.ell_spmv(m, g["row"], g["col"], g["val"], g["x"])
        assert np.array_equal(y, g["y_ell"])
    if "y_dia" in g:
        _, y = oracle.dia_spmv(m, n, g["row"], g["col"], g["val"], g["x"])
        assert np.array_equal(y, g["y_dia"])
    if "y_ss_simple" in g:
        assert np.array_equal(oracle.ss_spmv(rp, idx, val, g["x"], 4, False), g["y_ss_simple"])
    if "y_ss_opt" in g:
        assert np.array_equal(oracle.ss_spmv(rp, idx, val, g["x"], 4, True), g["y_ss_opt"])


F_PLUGINS = ("coo", "jds", "css", "ss_pad")


def _within(y, yref, mag, rel=1e-12):
    return bool(np.all(np.abs(y - yref) <= rel * mag + 1e-300))


@pytest.mark.parametrize("name", golden_names())
def test_f_plugin_vectors_pinned(name):
    """Every fixture carries the outputs of the reference's (f) plugins and of
    opt_ss OPTIMIZED+PADDING (oracle/make_golden.py): opt_jds and opt_css sum
    every row in column order (src/opt_jds.cpp:91-103; opt_css per column
    block, src/opt_css.cpp:226-303, blocks ascending) -- bit-equal to the
    opt_crs restatement; opt_coo's omp atomic scatter (src/opt_coo.cpp:34-46)
    and the PADDING tree fold (src/opt_ss.cpp:305-347) change the order --
    within 1e-12 of sum |a x|, exact on the integer-valued fixture."""
    g = load_golden(name)
    _, rp, idx, val = csr_of(g)
    y = oracle.csr_spmv(rp, idx, val, g["x"])
    mag = oracle.csr_spmv(rp, idx, np.abs(val), np.abs(g["x"]))
    for f in F_PLUGINS:
        assert f"y_{f}" in g, f"{name}: y_{f} missing"
        yf = g[f"y_{f}"]
        if f in ("jds", "css") or name == "syn_integer":
            assert np.array_equal(yf, y), f"{name}: y_{f}"
        else:
            assert _within(yf, y, mag), f"{name}: y_{f}"


@pytest.mark.parametrize("name", ["3x3", "5x5", "10x10", "random"])
def test_loader_and_vectors_match_reference(name):
    """LoadSparseMatrix + srand(3)/CreateRandomVector restated exactly."""
    g = load_golden("mtx_" + name)
    m, n, r, c, v = oracle.load_mtx(os.path.join(GOLDEN, "mtx", name + ".mtx"))
    assert (m, n) == (int(g["m"]), int(g["n"]))
    assert np.array_equal(r, g["row"]) and np.array_equal(c, g["col"]) and np.array_equal(v, g["val"])
    x, y0 = oracle.rand_vectors(n, m, seed=3)
    assert np.array_equal(x, g["x"]) and np.array_equal(y0, g["y0"])


def test_known_answers():
    # 3x3: diag(1,2,3) -> y_i = (i+1) x_i   
    g = load_golden("mtx_3x3")
    assert np.array_equal(g["y_crs"], np.array([1.0, 2.0, 3.0]) * g["x"])
    assert g["y_crs"].tolist() == [0.56138017520372763, 0.44996662552001265, 1.1792753381558114]
    # 5x5: row 5 is empty -> 0
    g = load_golden("mtx_5x5")
    assert g["y_crs"][4] == 0.0
    # 10x10: header says 27 of 28 triplets -> entry (7,10) dropped; rows 8-10 empty
    g = load_golden("mtx_10x10")
    assert len(g["val"]) == 27
    x = g["x"]
    row7 = sum(7.0 * x[c] for c in [0, 1, 2, 3, 4, 5, 7, 8])
    assert g["y_crs"][6] == pytest.approx(row7, rel=1e-15)
    assert (g["y_crs"][7:] == 0).all()


@pytest.mark.parametrize("name", golden_names())
def test_verify_criterion(name):
    """VerifyResult: passes on the reference y, fails on a perturbed row."""
    g = load_golden(name)
    m = int(g["m"])
    assert oracle.verify(m, g["row"], g["col"], g["val"], g["x"], g["y_crs"]) == -1
    nz = np.flatnonzero(np.abs(g["y_crs"]) > 1e-3)
    if len(nz):
        y = g["y_crs"].copy()
        y[nz[0]] *= 1 + 1e-4
        assert oracle.verify(m, g["row"], g["col"], g["val"], g["x"], y) == nz[0]


@pytest.mark.skipif(not oracle.ref_available("crs"), reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", range(6))
def test_random_instances_against_live_reference(seed):
    rng = np.random.default_rng(seed)
    m, n = int(rng.integers(1, 300)), int(rng.integers(1, 300))
    lens = rng.integers(0, 12, size=m)
    row = np.repeat(np.arange(m), lens).astype(np.int32)
    col = rng.integers(0, n, size=row.size).astype(np.int32)
    o = np.lexsort((col, row))
    row, col = row[o], col[o]
    # DIA keeps the last duplicate (src/opt_dia.cpp:55): dedupe for that check
    key = row.astype(np.int64) * n + col
    keep = np.concatenate([[True], key[1:] != key[:-1]]) if len(key) else np.array([], bool)
    row, col = row[keep], col[keep]
    val = rng.standard_normal(row.size)
    x = rng.random(n)
    rp, idx, cv = oracle.coo_to_csr(m, row, col, val)
    y = oracle.csr_spmv(rp, idx, cv, x)
    yr, ok = oracle.ref_spmv("crs", m, n, row, col, val, x)
    assert ok and np.array_equal(y, yr)
    _, yd = oracle.dia_spmv(m, n, row, col, val, x)
    assert np.array_equal(yd, oracle.ref_spmv("dia", m, n, row, col, val, x)[0])
    if n >= (np.bincount(row, minlength=m).max() if len(row) else 0):
        _, ye = oracle.ell_spmv(m, row, col, val, x)
        assert np.array_equal(ye, oracle.ref_spmv("ell", m, n, row, col, val, x)[0])
    assert np.array_equal(oracle.ss_spmv(rp, idx, cv, x, 4, True),
                          oracle.ref_spmv("ss_opt", m, n, row, col, val, x)[0])
    # the (f) plugins and SS PADDING, live: the same pins as the golden test
    mag = oracle.csr_spmv(rp, idx, np.abs(cv), x)
    for f in F_PLUGINS:
        if not oracle.ref_available(f):
            continue
        yf, okf = oracle.ref_spmv(f, m, n, row, col, val, x)
        assert okf, f
        if f in ("jds", "css"):
            assert np.array_equal(yf, y), f
        else:
            assert _within(yf, y, mag), f
