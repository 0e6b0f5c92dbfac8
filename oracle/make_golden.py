#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE's own code (oracle/_ref).

TEST INFRASTRUCTURE ONLY.  Run here, where /root/reference exists:

    make -C oracle all ref && python oracle/make_golden.py

Every fixture is data: inputs (COO as produced by the reference loader, x)
and the outputs of the reference plugins (y per format, VerifyResult flag).

* mtx_<name>.npz   -- the four reference fixtures matrix/test/*.mtx, loaded
                      by the reference LoadSparseMatrix, x/y0 from srand(3) +
                      CreateRandomVector exactly as src/main.cpp:18,31-32.
                      The .mtx data files themselves are copied to
                      tests/golden/mtx/ so loader tests run without the tree.
* syn_<name>.npz   -- small seeded instances of the BASELINE config families
                      (uniform 16/row, power-law, banded 64 diagonals,
                      integer-valued, edge cases), matrices built here with
                      numpy, y from the reference plugins.
Every fixture also carries y_coo, y_jds, y_css and y_ss_pad: the outputs of
the reference's opt_coo, opt_jds, opt_css and opt_ss OPTIMIZED+PADDING
plugins (oracle/Makefile), the (f) rows of SURVEY §8.
"""
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

REF_TEST = "/root/reference/matrix/test"
OUT = os.path.join(ROOT, "tests", "golden")


# the (f) plugins and the SS PADDING variant run on every fixture (SURVEY
# §8(c): they compile here and pass VERIFY): y_coo (omp atomic scatter --
# its summation order follows the thread split, so it is compared within
# 1e-12, not bitwise), y_jds, y_css (3 column blocks), y_ss_pad
F_PLUGINS = ["coo", "jds", "css", "ss_pad"]


def ref_outputs(m, n, row, col, val, x, y0, fmts):
    out = {}
    for f in fmts + [f for f in F_PLUGINS if f not in fmts]:
        y, ok = oracle.ref_spmv(f, m, n, row, col, val, x, y_init=y0, calls=2)
        assert ok, f"reference VerifyResult failed for {f}"
        out[f"y_{f}"] = y
    return out


def save(name, m, n, row, col, val, x, y0, fmts, **extra):
    d = dict(m=np.int64(m), n=np.int64(n), row=row.astype(np.int32),
             col=col.astype(np.int32), val=val.astype(np.float64),
             x=x.astype(np.float64), y0=y0.astype(np.float64))
    d.update(ref_outputs(m, n, row, col, val, x, y0, fmts))
    d.update(extra)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
    print(f"{name}: m={m} n={n} nnz={len(val)} fmts={fmts}")


def sort_coo(row, col, val):
    o = np.lexsort((col, row))
    return row[o], col[o], val[o]


def main():
    os.makedirs(os.path.join(OUT, "mtx"), exist_ok=True)
    all_fmts = ["crs", "ell", "dia", "ss_simple", "ss_opt"]
    # --- reference fixtures ------------------------------------------------
    for name in ["3x3", "5x5", "10x10", "random"]:
        p = os.path.join(REF_TEST, name + ".mtx")
        shutil.copy(p, os.path.join(OUT, "mtx", name + ".mtx"))
        m, n, row, col, val = oracle.ref_load_mtx(p)
        x, y0 = oracle.ref_rand_vectors(n, m, seed=3)
        save("mtx_" + name, m, n, row, col, val, x, y0, all_fmts)

    rng = np.random.default_rng(20261015)
    # --- C2 family: uniform 16 nnz/row, cols uniform, sorted, dups allowed --
    m = n = 1024
    row = np.repeat(np.arange(m), 16)
    col = rng.integers(0, n, size=m * 16)
    val = 1.0 - rng.random(m * 16)              # U(0,1]
    row, col, val = sort_coo(row, col, val)
    x = rng.random(n)
    save("syn_uniform", m, n, row, col, val, x, rng.random(m),
         ["crs", "ell", "ss_opt"])
    # --- C3 family: power law P(k) ~ k^-2 on [1, 2000] + two very long rows -
    m = n = 3000
    k = np.arange(1, 2001)
    p = 1.0 / k**2
    lens = rng.choice(k, size=m, p=p / p.sum())
    lens[17] = 2500
    lens[1234] = 1800
    lens[rng.integers(0, m, 40)] = 0            # empty rows
    row = np.repeat(np.arange(m), lens)
    col = rng.integers(0, n, size=row.size)
    val = 1.0 - rng.random(row.size)
    row, col, val = sort_coo(row, col, val)
    save("syn_powerlaw", m, n, row, col, val, rng.random(n), rng.random(m),
         ["crs", "ss_opt"])
    # --- C4 family: banded, diagonal offsets -32..31 -------------------------
    m = n = 400
    offs = np.arange(-32, 32)
    rr, oo = np.meshgrid(np.arange(m), offs, indexing="ij")
    cc = rr + oo
    keep = (cc >= 0) & (cc < n)
    row, col = rr[keep], cc[keep]
    val = 1.0 - rng.random(row.size)
    row, col, val = sort_coo(row, col, val)
    save("syn_banded", m, n, row, col, val, rng.random(n), rng.random(m),
         ["crs", "dia", "ell"])
    # --- integer-valued (CSR5 trick, CSR5_cuda/main.cu:317-326): exact sums --
    m, n = 700, 900
    row = np.repeat(np.arange(m), 24)
    col = rng.integers(0, n, size=row.size)
    val = rng.integers(0, 10, size=row.size).astype(np.float64)
    row, col, val = sort_coo(row, col, val)
    save("syn_integer", m, n, row, col, val,
         rng.integers(0, 10, size=n).astype(np.float64), rng.random(m),
         ["crs", "ell", "ss_opt"])
    # --- edge cases: empty rows at head/tail, duplicates, rectangular, a row
    #     longer than one 64-lane wave, negative values (cancellation) --------
    m, n = 300, 170
    lens = rng.integers(0, 9, size=m)
    lens[:5] = 0
    lens[-7:] = 0
    lens[100] = 333                             # longer than n: duplicates
    lens[101] = 65
    row = np.repeat(np.arange(m), lens)
    col = rng.integers(0, n, size=row.size)
    val = rng.standard_normal(row.size)
    row, col, val = sort_coo(row, col, val)
    save("syn_edge", m, n, row, col, val, rng.standard_normal(n), rng.random(m),
         ["crs", "ss_opt"])


def make_dups():
    """mtx_dups: a Matrix Market file whose (row, col) keys repeat in runs
    far longer than std::sort's 16-element insertion-sort threshold, entries
    in shuffled file order -- the reference loader's std::sort (not stable,
    src/util.cpp:51) leaves equal keys in an order of its own, which this
    fixture pins (the COO is the REFERENCE loader's, via oracle/_ref)."""
    rng = np.random.default_rng(20261018)
    # n above the longest row: opt_ell pads with column = slot index
    # (src/opt_ell.cpp:46-52), which must stay inside x
    m, n = 90, 400
    keys = [(r, c) for r in range(m) for c in rng.choice(n, size=rng.integers(0, 6), replace=False)]
    ents = []
    for (r, c) in keys:
        reps = int(rng.choice([1, 1, 2, 3, 17, 40, 75]))
        ents += [(r, c, float(1.0 - rng.random())) for _ in range(reps)]
    order = rng.permutation(len(ents))
    path = os.path.join(OUT, "mtx", "dups.mtx")
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n% duplicate-key runs\n")
        f.write(f"{m} {n} {len(ents)}\n")
        for i in order:
            r, c, v = ents[i]
            f.write(f"{r + 1} {c + 1} {v!r}\n")
    m2, n2, row, col, val = oracle.ref_load_mtx(path)
    x, y0 = oracle.ref_rand_vectors(n2, m2, seed=3)
    save("mtx_dups", m2, n2, row, col, val, x, y0, ["crs", "ell", "ss_simple", "ss_opt"])


if __name__ == "__main__":
    if sys.argv[1:] == ["dups"]:
        make_dups()
    else:
        main()
        make_dups()
