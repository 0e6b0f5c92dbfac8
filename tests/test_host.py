"""Host side of the product path (no GPU): loader, vectors, verify, COO->CSR,
synthetic generators, row partition -- checked against the oracle and the
reference golden fixtures."""
import os

import numpy as np
import pytest

import oracle
import singlespmv_amd as sp
from conftest import GOLDEN, load_golden


@pytest.mark.parametrize("name", ["3x3", "5x5", "10x10", "random"])
def test_loader_matches_reference(name):
    g = load_golden("mtx_" + name)
    A = sp.load_sparse_matrix(os.path.join(GOLDEN, "mtx", name + ".mtx"))
    assert (A.nRow, A.nCol, A.nNnz) == (int(g["m"]), int(g["n"]), len(g["val"]))
    assert np.array_equal(A.row_idx, g["row"]) and np.array_equal(A.col_idx, g["col"])
    assert np.array_equal(A.val, g["val"])


def test_loader_errors(tmp_path):
    with pytest.raises(sp.SpmvError, match="I/O|File not Found"):
        sp.load_sparse_matrix(str(tmp_path / "missing.mtx"))
    p = tmp_path / "trunc.mtx"
    p.write_text("%%MatrixMarket\n3 3 4\n1 1 1\n2 2 2\n")
    with pytest.raises(sp.SpmvError):
        sp.load_sparse_matrix(str(p))
    p.write_text("3 3 1\n4 1 1\n")
    with pytest.raises(sp.SpmvError):
        sp.load_sparse_matrix(str(p))


def test_loader_sorts_and_keeps_duplicates(tmp_path):
    p = tmp_path / "dup.mtx"
    p.write_text("% c\n% d\n3 4 5\n3 1 1.5\n1 4 2\n1 2 -1\n3 1 0.25\n2 2 7e-3\n")
    A = sp.load_sparse_matrix(str(p))
    m, n, r, c, v = oracle.load_mtx(str(p))
    assert np.array_equal(A.row_idx, r) and np.array_equal(A.col_idx, c)
    assert np.array_equal(A.val, v)
    assert A.row_idx.tolist() == [0, 0, 1, 2, 2] and A.val.tolist()[-2:] == [1.5, 0.25]


def test_random_vector_matches_reference():
    g = load_golden("mtx_random")
    sp.srand(3)
    x = sp.create_random_vector(int(g["n"]))
    y0 = sp.create_random_vector(int(g["m"]))
    assert np.array_equal(x, g["x"]) and np.array_equal(y0, g["y0"])


def test_verify_result_clone():
    g = load_golden("syn_powerlaw")
    A = sp.SpMat(int(g["m"]), int(g["n"]), g["row"], g["col"], g["val"])
    assert sp.verify_result(A, g["x"], g["y_crs"])
    y = g["y_crs"].copy()
    y[np.argmax(y)] += 1.0
    assert not sp.verify_result(A, g["x"], y)


def test_coo_to_csr_matches_oracle():
    g = load_golden("syn_edge")
    m = int(g["m"])
    rp = sp.coo_to_csr(m, g["row"])
    rp_o, _, _ = oracle.coo_to_csr(m, g["row"], g["col"], g["val"])
    assert np.array_equal(rp, rp_o)
    with pytest.raises(sp.SpmvError):
        sp.coo_to_csr(3, np.array([2, 1], np.int32))  # unsorted rows


@pytest.mark.parametrize("kind", ["uniform", "powerlaw", "banded"])
def test_generators_deterministic_and_well_formed(kind):
    spec = sp.gen_spec(kind, 5000, per_row=16, max_len=3000, seed=7)
    rp, col, val = sp.generate_csr(spec)
    rp2, col2, val2 = sp.generate_csr(spec)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
    assert rp[0] == 0 and (np.diff(rp) >= 0).all() and rp[-1] == len(col)
    assert col.min() >= 0 and col.max() < 5000
    assert (val > 0).all() and (val <= 1).all()
    # sorted within rows
    for r in range(0, 5000, 97):
        seg = col[rp[r]:rp[r + 1]]
        assert (np.diff(seg) >= 0).all()
    # any row range reproduces the same rows (multi-GPU ranks generate their own)
    rpb, colb, valb = sp.generate_csr(spec, 1234, 2345)
    assert np.array_equal(colb, col[rp[1234]:rp[2345]])
    assert np.array_equal(valb, val[rp[1234]:rp[2345]])
    if kind == "uniform":
        assert (np.diff(rp) == 16).all()
    if kind == "banded":
        assert np.diff(rp).max() == 64
        r = 2500
        assert col[rp[r]:rp[r + 1]].tolist() == list(range(r - 32, r + 32))
    if kind == "powerlaw":
        lens = np.diff(rp)
        assert lens.min() >= 1 and lens.max() <= 3000
        assert 3.0 < lens.mean() < 10.0


def test_integer_generator_and_vectors():
    spec = sp.gen_spec("uniform", 300, per_row=8, integer_values=True)
    _, _, val = sp.generate_csr(spec)
    assert set(np.unique(val)).issubset(set(range(10)))
    x = sp.generate_vector(1000, seed=43)
    assert np.array_equal(x[100:200], sp.generate_vector(100, seed=43, begin=100))
    assert (x >= 0).all() and (x < 1).all()


def test_partition_rows_balanced():
    spec = sp.gen_spec("powerlaw", 20000, max_len=5000, seed=3)
    rp, _, _ = sp.generate_csr(spec)
    for parts in (1, 2, 3, 8):
        cuts = sp.partition_rows(rp, parts)
        assert cuts[0] == 0 and cuts[-1] == 20000 and (np.diff(cuts) >= 0).all()
        nnz = rp[-1]
        for k in range(1, parts):
            assert rp[cuts[k]] >= k * nnz // parts
            assert cuts[k] == 0 or rp[cuts[k] - 1] < k * nnz / parts


def _write_mtx(path, m, n, row, col, val, header="%%MatrixMarket matrix coordinate real general\n% c\n",
               sep="\n"):
    with open(path, "w") as f:
        f.write(header)
        f.write(f"{m} {n} {len(val)}\n")
        f.write(sep.join(f"{r + 1} {c + 1} {float(v)!r}" for r, c, v in zip(row, col, val)))
        f.write("\n")


@pytest.mark.parametrize("sep", ["\n", "\t\n", "  \n\n", " "])
def test_parallel_loader_matches_oracle_loader(tmp_path, sep):
    """Large shuffled file (multi-chunk parallel parse): identical COO to the
    oracle's restatement of LoadSparseMatrix, whatever the line structure."""
    rng = np.random.default_rng(1)
    m, n, k = 40000, 30000, 600000
    row = rng.integers(0, m, k)
    col = rng.integers(0, n, k)
    val = rng.standard_normal(k) * 10.0 ** rng.integers(-5, 5, k)
    p = str(tmp_path / "big.mtx")
    _write_mtx(p, m, n, row, col, val, sep=sep)
    A = sp.load_sparse_matrix(p)
    mo, no, ro, co, vo = oracle.load_mtx(p)
    assert (A.nRow, A.nCol) == (mo, no)
    assert np.array_equal(A.row_idx, ro) and np.array_equal(A.col_idx, co)
    assert np.array_equal(A.val, vo)


def test_loader_ignores_entries_beyond_L(tmp_path):
    p = tmp_path / "x.mtx"
    p.write_text("3 3 2\n1 1 1.5\n2 2\n2.5 3 3 9.0\n")  # triplet split over lines; 3rd ignored
    A = sp.load_sparse_matrix(str(p))
    assert A.row_idx.tolist() == [0, 1] and A.val.tolist() == [1.5, 2.5]


def test_csr_bin_roundtrip(tmp_path):
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", 7777, max_len=400, seed=3))
    p = str(tmp_path / "a.csrbin")
    sp.save_csr_bin(p, 7777, 7777, rp, col, val)
    m, n, rp2, col2, val2 = sp.load_csr_bin(p)
    assert (m, n) == (7777, 7777)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
    with open(p, "r+b") as f:
        f.write(b"NOTMAGIC")
    with pytest.raises(sp.SpmvError):
        sp.load_csr_bin(p)
