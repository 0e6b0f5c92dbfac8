"""Host side of the product path (no GPU): loader, vectors, verify, COO->CSR,
synthetic generators, row partition -- checked against the oracle and the
reference golden fixtures."""
import os

import numpy as np
import pytest

import oracle
import singlespmv_amd as sp
from conftest import GOLDEN, load_golden


@pytest.mark.parametrize("name", ["3x3", "5x5", "10x10", "random", "dups"])
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


def test_loader_duplicate_runs_follow_the_reference_sort():
    """mtx_dups: (row, col) keys repeated in runs of up to 75 in shuffled file
    order.  The reference's std::sort is not stable; the loader reproduces
    its order of equal keys (the fixture is the reference loader's COO), where
    a stable sort (the oracle's restatement) differs."""
    g = load_golden("mtx_dups")
    path = os.path.join(GOLDEN, "mtx", "dups.mtx")
    A = sp.load_sparse_matrix(path)
    assert np.array_equal(A.val, g["val"])
    _, _, r, c, v = oracle.load_mtx(path)
    assert np.array_equal(r, g["row"]) and np.array_equal(c, g["col"])
    assert not np.array_equal(v, g["val"])  # the fixture does exercise the unstable order
    if oracle.ref_available("crs"):  # the reference loader itself, where it is built
        _, _, rr, rc, rv = oracle.ref_load_mtx(path)
        assert np.array_equal(rv, A.val) and np.array_equal(rc, A.col_idx) and np.array_equal(rr, A.row_idx)


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
    # equal (row, col) keys (~150 here): the loader follows the reference's
    # unstable std::sort, the oracle keeps file order -- same values per key
    key = ro.astype(np.int64) * n + co
    first = np.concatenate([[True], key[1:] != key[:-1]])
    grp = np.cumsum(first)
    dup = np.bincount(grp)[grp] > 1
    assert dup.sum() > 0 and np.array_equal(A.val[~dup], vo[~dup])
    assert np.array_equal(A.val[np.lexsort((A.val, grp))], vo[np.lexsort((vo, grp))])


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


MM_CASES = {
    "general_real": ("real general", [(3, 1, 1.5), (1, 2, -2.0), (3, 3, 4.0), (1, 1, 0.5)]),
    "symmetric": ("real symmetric", [(1, 1, 2.0), (3, 1, 1.5), (2, 1, -1.0), (3, 3, 4.0), (3, 2, 0.25)]),
    "hermitian": ("real hermitian", [(2, 1, 7.0), (2, 2, 1.0)]),
    "skew": ("real skew-symmetric", [(2, 1, 7.0), (3, 2, -1.0)]),
    "integer_sym": ("integer symmetric", [(1, 1, 3), (3, 1, 9), (2, 2, -4)]),
    "pattern": ("pattern general", [(1, 3), (3, 1), (2, 2), (1, 1)]),
    "pattern_sym": ("pattern symmetric", [(3, 1), (2, 1), (3, 3)]),
}


@pytest.mark.parametrize("case", sorted(MM_CASES))
def test_load_mtx_csr_matches_csr5_loader(tmp_path, case):
    """spmv_load_mtx_csr vs the restatement of CSR5_cuda/main.cu:157-306:
    identical CSR, including the file-order row contents (parity pinned by
    the restatement only: the reference ships no symmetric/pattern fixture)."""
    kind, entries = MM_CASES[case]
    p = tmp_path / f"{case}.mtx"
    body = "\n".join(" ".join(str(t) for t in e) for e in entries)
    p.write_text(f"%%MatrixMarket matrix coordinate {kind}\n% comment\n3 3 {len(entries)}\n{body}\n")
    m, n, rp, col, val, info = sp.load_mtx_csr(str(p))
    mo, no, rpo, colo, valo = oracle.load_mtx_csr5(str(p))
    assert (m, n) == (mo, no)
    assert np.array_equal(rp, rpo) and np.array_equal(col, colo) and np.array_equal(val, valo)
    assert info["mirrored"] == (kind.split()[1] in ("symmetric", "hermitian"))
    assert info["field"] == kind.split()[0]
    # sorted variant: same multiset per row, columns non-decreasing
    _, _, rps, cols, vals, _ = sp.load_mtx_csr(str(p), sort_columns=True)
    assert np.array_equal(rps, rpo)
    for r in range(m):
        seg = slice(rpo[r], rpo[r + 1])
        assert (np.diff(cols[seg]) >= 0).all()
        assert sorted(zip(colo[seg], valo[seg])) == sorted(zip(cols[seg], vals[seg]))


def test_load_mtx_csr_large_symmetric_parallel(tmp_path):
    """multi-chunk parallel parse + mirrored scatter vs a numpy restatement."""
    rng = np.random.default_rng(7)
    m, k = 20000, 300000
    r = rng.integers(0, m, k)
    c = rng.integers(0, m, k)
    lo, hi = np.maximum(r, c), np.minimum(r, c)  # lower triangle as stored
    v = rng.standard_normal(k)
    p = str(tmp_path / "sym.mtx")
    _write_mtx(p, m, m, lo, hi, v, header="%%MatrixMarket matrix coordinate real symmetric\n")
    mm, nn, rp, col, val, info = sp.load_mtx_csr(p)
    assert info["mirrored"]
    # expanded entry list in file order, then a stable sort by row
    off = lo != hi
    er = np.empty(k + off.sum(), np.int64)
    ec = np.empty_like(er)
    ev = np.empty(len(er))
    idx = np.arange(k) + np.concatenate([[0], np.cumsum(off)[:-1]])
    er[idx], ec[idx], ev[idx] = lo, hi, v
    mir = idx[off] + 1
    er[mir], ec[mir], ev[mir] = hi[off], lo[off], v[off]
    order = np.argsort(er, kind="stable")
    assert np.array_equal(rp, np.concatenate([[0], np.cumsum(np.bincount(er, minlength=m))]))
    assert np.array_equal(col, ec[order]) and np.array_equal(val, ev[order])


def test_load_mtx_csr_errors(tmp_path):
    p = tmp_path / "c.mtx"
    p.write_text("%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1.0 2.0\n")
    with pytest.raises(sp.SpmvError, match="not supported"):
        sp.load_mtx_csr(str(p))
    p.write_text("2 2 1\n1 1 1.0\n")  # no banner
    with pytest.raises(sp.SpmvError, match="banner"):
        sp.load_mtx_csr(str(p))
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n2 3 1\n1 1 1.0\n")
    with pytest.raises(sp.SpmvError, match="m != n"):
        sp.load_mtx_csr(str(p))
    p.write_text("%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1.0\n")
    with pytest.raises(sp.SpmvError, match="truncated"):
        sp.load_mtx_csr(str(p))
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n2 2 1\n2 1 5.0\n")
    _, _, rp, col, val, info = sp.load_mtx_csr(str(p), expand=False)
    assert rp.tolist() == [0, 0, 1] and not info["mirrored"]


def test_load_mtx_csr_reference_banner_file():
    """random.mtx is the one reference fixture with a banner (real general):
    the CSR5-semantics loader gives the same CSR as LoadSparseMatrix once rows
    are column-sorted."""
    g = load_golden("mtx_random")
    m, n, rp, col, val, _ = sp.load_mtx_csr(os.path.join(GOLDEN, "mtx", "random.mtx"), sort_columns=True)
    assert np.array_equal(rp, sp.coo_to_csr(int(g["m"]), g["row"]))
    assert np.array_equal(col, g["col"]) and np.array_equal(val, g["val"])


def test_mtx2bin_cli(tmp_path):
    from singlespmv_amd import mtx2bin
    out = str(tmp_path / "r.csrbin")
    assert mtx2bin.main([os.path.join(GOLDEN, "mtx", "random.mtx"), out]) == 0
    g = load_golden("mtx_random")
    m, n, rp, col, val = sp.load_csr_bin(out)
    assert np.array_equal(rp, sp.coo_to_csr(int(g["m"]), g["row"])) and np.array_equal(val, g["val"])


def test_dist_layout_cuts_and_slices():
    """The row cut of the C-ABI multi-GPU plan (spmv_dist_layout): nnz-
    balanced cuts, monotone, covering [0, m], and the padded
    slice = the longest range; N = 1..8 over uniform, power-law and
    all-empty matrices."""
    for kind in ("uniform", "powerlaw"):
        spec = sp.gen_spec(kind, 100_003, per_row=7, max_len=5000, seed=4)
        rp, _, _ = sp.generate_csr(spec)
        nnz = int(rp[-1])
        for parts in range(1, 9):
            cuts, sl = sp.dist_layout(rp, parts)
            assert cuts[0] == 0 and cuts[-1] == len(rp) - 1 and np.all(np.diff(cuts) >= 0)
            assert sl == max(1, int(np.max(np.diff(cuts))))
            share = np.diff(rp[cuts])
            # no part exceeds its nnz share by more than one row's entries
            assert share.max() <= nnz / parts + np.diff(rp).max()
    cuts, sl = sp.dist_layout(np.zeros(11, np.int64), 4)
    assert cuts[0] == 0 and cuts[-1] == 10 and sl >= 1
