"""Parity of the HIP kernels (through the C-ABI) against the oracle and the
reference golden vectors.  Needs an MI355X: `pytest -m gpu`.

Tolerances (BASELINE north star: within 1e-6 relative fp64):
* every result must pass the reference VerifyResult criterion
  (src/util.cpp:67-83: a row fails iff abs > 1e-6 AND rel > 1e-6);
* non-negative inputs: |y - y_ref| <= 1e-12 * |y_ref| + 1e-300 per row;
* integer-valued inputs and sequential-order formats (ELL, DIA, 1-lane CSR,
  BIN): bit-exact against the oracle's sequential row sum -- BIN's long rows
  (the run path, plan info bin_long_len) excepted: deterministic, within
  1e-12 of the sequential sum relative to sum |a_ij x_j|;
* every format is idempotent: two calls over a garbage y give identical y
  (the two-call verification of src/main.cpp:40-56).
"""
import ctypes as C
import os
import time

import numpy as np
import pytest

import oracle
import singlespmv_amd as sp
from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu

FORMATS = ["csr", "ell", "ss", "hyb", "dia", "css", "coo", "jds", "bin", "auto"]
REL = 1e-12


def oracle_y(rp, col, val, x):
    return oracle.csr_spmv(np.ascontiguousarray(rp, np.int64), np.ascontiguousarray(col, np.int32),
                           np.ascontiguousarray(val, np.float64), np.ascontiguousarray(x, np.float64))


def check_close(y, yref, rel=REL, what=""):
    err = np.abs(y - yref)
    tol = rel * np.abs(yref) + 1e-300
    bad = np.flatnonzero(err > np.maximum(tol, 0))
    # allow exact-zero rows with tiny absolute error only for signed inputs
    assert len(bad) == 0, f"{what}: {len(bad)} rows off, first {bad[:5]}: {y[bad[:5]]} vs {yref[bad[:5]]}"


def assert_bin_rows(plan, y, rp, col, val, x, what=""):
    """BIN: rows shorter than the plan's long-row threshold are the
    sequential opt_crs sum bit for bit; long rows (the Mul's run path, summed
    as run pieces) are within 1e-12 of it relative to sum_j |a_ij x_j|."""
    yo = oracle_y(rp, col, val, x)
    ll = plan.info()["bin_long_len"]
    if ll == 0:
        assert np.array_equal(y, yo), f"bin {what}: not bit-exact"
        return
    long_rows = np.diff(np.asarray(rp, np.int64)) >= ll
    assert np.array_equal(y[~long_rows], yo[~long_rows]), f"bin {what}: short rows not bit-exact"
    mag = oracle_y(rp, col, np.abs(val), np.abs(x))
    err = np.abs(y[long_rows] - yo[long_rows])
    assert np.all(err <= 1e-12 * mag[long_rows] + 1e-300), f"bin {what}: long rows off by {err.max()}"


def run_plan(plan, x, m, garbage=1.2345e300):
    y = np.full(m, garbage)
    plan.execute(x, y)
    y2 = np.full(m, -garbage)
    plan.execute(x, y2)
    if plan.info()["format"] == "coo":
        # f64 atomics (as the reference's omp atomic): rows split across wave
        # steps may round differently run to run -- idempotent to 1e-12
        check_close(y2, y, what="coo idempotence")
    else:
        assert np.array_equal(y, y2, equal_nan=True), "not idempotent / depends on prior y"
    return y


def make_plan(m, n, rp, col, val, fmt, **kw):
    try:
        return sp.Plan.from_csr(m, n, rp, col, val, fmt=fmt, **kw)
    except sp.SpmvError as e:
        if fmt == "dia" and "not supported" in str(e):
            return None
        raise


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("fmt", FORMATS)
def test_golden(name, fmt):
    g = load_golden(name)
    m, n = int(g["m"]), int(g["n"])
    rp = sp.coo_to_csr(m, g["row"])
    plan = make_plan(m, n, rp, g["col"], g["val"], fmt)
    if plan is None:
        pytest.skip("DIA refuses this matrix (too many diagonals)")
    y = run_plan(plan, g["x"], m)
    A = sp.SpMat(m, n, g["row"], g["col"], g["val"])
    assert sp.verify_result(A, g["x"], y), "VerifyResult (1e-6) failed"
    yref = g["y_crs"]
    signed = (g["val"] < 0).any() or (g["x"] < 0).any()
    if name == "syn_integer":
        assert np.array_equal(y, yref), "integer-valued inputs must be exact"
    elif not signed:
        check_close(y, yref, what=f"{name}/{fmt}")
    info = plan.info()
    # DIA adds duplicate entries into one slot first (src/opt_dia.cpp:47-56)
    dups = bool(np.any((np.diff(g["row"]) == 0) & (np.diff(g["col"]) == 0)))
    sequential = info["format"] == "ell" or (info["format"] == "dia" and not dups) or (info["format"] == "csr" and info["csr_lanes"] == 1) \
        or (info["format"] == "jds" and info["overflow_nnz"] == 0) \
        or (info["format"] == "css" and info["css_split_rows"] == 0) \
        or (info["format"] == "bin" and info["bin_long_len"] == 0)
    if info["format"] == "bin":
        assert_bin_rows(plan, y, rp, g["col"], g["val"], g["x"], what=name)
    if sequential:
        assert np.array_equal(y, yref), f"{info['format']} is sequential: must be bit-exact"
    # the format's own reference plugin (oracle/make_golden.py): opt_coo,
    # opt_jds, opt_css, opt_ss (OPTIMIZED, and OPTIMIZED+PADDING) -- within
    # 1e-12 of sum |a x| (their summation orders differ from each other)
    own = {"coo": ("y_coo",), "jds": ("y_jds",), "css": ("y_css",), "ss": ("y_ss_opt", "y_ss_pad"),
           "ell": ("y_ell",), "dia": ("y_dia",)}.get(fmt, ())
    mag = oracle_y(rp, g["col"], np.abs(g["val"]), np.abs(g["x"]))
    for key in own:
        if key in g:
            err = np.abs(y - g[key])
            assert np.all(err <= REL * mag + 1e-300), f"{name}/{fmt} vs the reference's {key}: {err.max()}"


@pytest.mark.parametrize("lanes", [1, 2, 4, 8, 16, 32, 64])
def test_csr_lanes(lanes):
    spec = sp.gen_spec("powerlaw", 20000, max_len=3000, seed=11)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(20000, seed=5)
    y = run_plan(sp.Plan.from_csr(20000, 20000, rp, col, val, "csr", csr_lanes=lanes), x, 20000)
    yo = oracle_y(rp, col, val, x)
    check_close(y, yo, what=f"lanes={lanes}")
    if lanes == 1:
        assert np.array_equal(y, yo)


@pytest.mark.parametrize("lanes", [0, 1, 4, 16, 64])
@pytest.mark.parametrize("empty", [False, True])
def test_csr_window_kernel(lanes, empty):
    """Banded rows: the CSR plan keeps an x window per 512-row workgroup and
    runs csr_slabx (x from LDS, the stream one batch ahead) -- lanes 4 with
    81-entry rows take its long-row loop; adding one explicit zero far off the
    band to the last row leaves no window (csr_slab2), and every other row is
    bit-identical between the two kernels (same chunks, same order)."""
    if lanes == 0 and empty:
        pytest.skip("AUTO bins rows of mixed lengths (the adaptive kernel)")
    m = 20077
    rp, col, val = sp.generate_csr(sp.gen_spec("banded", m, band_lo=-40, band_hi=40, seed=21))
    if empty:
        rp, col, val = _with_empty_rows(rp, col, val, 0.1, 3)
    x = sp.generate_vector(m, seed=22)
    kw = {"csr_lanes": lanes} if lanes else {}
    plan = sp.Plan.from_csr(m, m, rp, col, val, "csr", **kw)
    assert plan.info()["kernel"].startswith("csr_slabx_kernel"), plan.info()["kernel"]
    y = run_plan(plan, x, m)
    yo = oracle_y(rp, col, val, x)
    check_close(y, yo, what=f"slabx lanes {lanes}")
    if lanes == 1:
        assert np.array_equal(y, yo)
    # the same matrix with an explicit 0 at column 0 of the last row: no window
    s = int(rp[-2])
    col2 = np.concatenate([col[:s], [0], col[s:]]).astype(np.int32)
    val2 = np.concatenate([val[:s], [0.0], val[s:]])
    rp2 = rp.copy()
    rp2[-1] += 1
    plan2 = sp.Plan.from_csr(m, m, rp2, col2, val2, "csr", **kw)
    assert plan2.info()["kernel"].startswith("csr_slab2_kernel"), plan2.info()["kernel"]
    y2 = run_plan(plan2, x, m)
    assert np.array_equal(y[:-1], y2[:-1])
    check_close(y2, yo, what=f"slab2 lanes {lanes}")


@pytest.mark.parametrize("m,n", [(1, 1), (7, 7), (255, 255), (256, 300), (257, 257), (513, 40), (1000, 5000)])
@pytest.mark.parametrize("lanes", [1, 4])
def test_csr_window_kernel_small_shapes(m, n, lanes):
    """csr_slabx at the edges: fewer rows than a workgroup, a partial last
    granule, rectangular matrices whose windows touch column 0 or n - 1,
    empty rows; y against the oracle (bit for bit with one lane)."""
    rng = np.random.default_rng(m * 7 + n)
    rows, cols = [], []
    for r in range(m):
        c = r * n // max(m, 1)
        cs = sorted({min(n - 1, max(0, c + d)) for d in range(-3, 4) if rng.random() < 0.8})
        if r % 11 == 5:
            cs = []  # empty rows
        rows += [r] * len(cs)
        cols += cs
    rp = np.zeros(m + 1, np.int64)
    np.add.at(rp, np.asarray(rows, np.int64) + 1, 1)
    rp = np.cumsum(rp)
    col = np.asarray(cols, np.int32)
    val = rng.random(len(col)) + 0.5
    x = rng.random(n)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "csr", csr_lanes=lanes)
    assert plan.info()["kernel"].startswith("csr_slabx_kernel"), plan.info()["kernel"]
    y = run_plan(plan, x, m)
    yo = oracle_y(rp, col, val, x)
    if lanes == 1:
        assert np.array_equal(y, yo)
    else:
        check_close(y, yo, what=f"{m}x{n}")


@pytest.mark.parametrize("sigma", [4, 8, 12, 16, 20, 24, 32, 48, 64])
@pytest.mark.parametrize("kind", ["powerlaw", "uniform", "empty_rows", "banded", "short"])
def test_ss_sigma(sigma, kind):
    m = 30011
    if kind == "short":
        # rows of 0-3 entries: a tile finishes 64-4096 rows, so every tile-end
        # path runs -- rows in the one store instruction (<= 62), in whole
        # waves (63-256, staged) and stored directly (> 256)
        rng = np.random.default_rng(100 + sigma)
        lens = rng.integers(0, 4, m)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.sort(rng.choice(m, int(k), replace=False)) for k in lens]).astype(np.int32)
        val = rng.standard_normal(int(rp[-1]))
    elif kind == "empty_rows":
        spec = sp.gen_spec("powerlaw", m, max_len=500, seed=13)
        rp, col, val = sp.generate_csr(spec)
        rng = np.random.default_rng(sigma)
        lens = np.diff(rp)
        zero = rng.random(m) < 0.1
        zero[:7] = True
        zero[-9:] = True
        keep = np.repeat(~zero, lens)
        col, val = np.ascontiguousarray(col[keep]), np.ascontiguousarray(val[keep])
        rp = np.concatenate([[0], np.cumsum(np.where(zero, 0, lens))]).astype(np.int64)
    else:  # banded: every tile's x window fits (ss_stream_kernel reads x from LDS)
        spec = sp.gen_spec(kind, m, per_row=13, max_len=4000, band_lo=-40, band_hi=23, seed=17)
        rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=19)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "ss", ss_sigma=sigma)
    y = run_plan(plan, x, m)
    check_close(y, oracle_y(rp, col, val, x), what=f"ss sigma={sigma} {kind}")


@pytest.mark.parametrize("width", [0, 4, 8, 24, 64])
def test_hyb_widths(width):
    m = 25000
    spec = sp.gen_spec("powerlaw", m, max_len=6000, seed=23)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=29)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "hyb", ell_width=width)
    info = plan.info()
    assert info["n_kernels"] in (1, 2)
    y = run_plan(plan, x, m)
    check_close(y, oracle_y(rp, col, val, x), what=f"hyb K={width}")


def test_dia_banded_bit_exact_and_refusal():
    m = 50000
    spec = sp.gen_spec("banded", m, band_lo=-32, band_hi=31, seed=31)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=37)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "dia")
    assert plan.info()["n_diags"] == 64
    y = run_plan(plan, x, m)
    assert np.array_equal(y, oracle_y(rp, col, val, x))
    # AUTO picks DIA for a banded matrix
    assert sp.Plan.from_csr(m, m, rp, col, val, "auto").info()["format"] == "dia"
    # a uniform random matrix is refused by DIA
    rp2, col2, val2 = sp.generate_csr(sp.gen_spec("uniform", 5000, per_row=8))
    with pytest.raises(sp.SpmvError, match="not supported"):
        sp.Plan.from_csr(5000, 5000, rp2, col2, val2, "dia")


@pytest.mark.parametrize("shift,lag", [(17, 0), (8, 0), (10, 3), (12, -1), (20, 1)])
def test_css_slabs_and_pacing(shift, lag):
    """Column-slab sweep: any slab width / pacing slack gives the sequential
    opt_crs sum bit for bit (rows sorted by column)."""
    m = 70001
    spec = sp.gen_spec("powerlaw", m, max_len=3000, seed=47)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=53)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "css", css_slab_shift=shift, css_lag=lag)
    info = plan.info()
    assert info["css_slabs"] == (m + (1 << shift) - 1) >> shift
    y = run_plan(plan, x, m)
    yo = oracle_y(rp, col, val, x)
    if info["css_split_rows"] == 0:
        assert np.array_equal(y, yo)
    else:
        check_close(y, yo, what="css split rows")


def test_css_split_long_rows_deterministic():
    """Rows longer than half a wave's share are split into pieces merged in
    piece order: 1e-12 relative to opt_crs and bitwise identical run to run;
    the unsplit rows stay bit-exact."""
    m = 200000
    spec = sp.gen_spec("powerlaw", m, max_len=20000, seed=67)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=71)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "css")
    assert plan.info()["css_split_rows"] > 0
    y = run_plan(plan, x, m)
    yo = oracle_y(rp, col, val, x)
    check_close(y, yo, what="css split")
    plan2 = sp.Plan.from_csr(m, m, rp, col, val, "css")
    assert np.array_equal(y, run_plan(plan2, x, m))
    lens = np.diff(rp)
    short = lens < 32
    assert np.array_equal(y[short], yo[short])


def test_css_multi_pass():
    """More rows than #CU x 19968 -> several row passes through LDS."""
    m = 6_000_000
    spec = sp.gen_spec("uniform", m, per_row=2, seed=59)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=61)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "css")
    assert plan.info()["css_passes"] >= 2
    y = run_plan(plan, x, m)
    assert np.array_equal(y, oracle_y(rp, col, val, x))


def test_jds_permutation_and_coo_atomics():
    """JDS (rows sorted by length, y permuted back) is the sequential row sum
    for rows up to its jagged-diagonal cap, within 1e-12 beyond;
    COO (one f64 atomic per row run per 128-entry unit) is within 1e-12 and
    reproducible for every row that sits inside one unit."""
    m = 50000
    spec = sp.gen_spec("powerlaw", m, max_len=1500, seed=73)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=79)
    yo = oracle_y(rp, col, val, x)
    pj = sp.Plan.from_csr(m, m, rp, col, val, "jds")
    yj = run_plan(pj, x, m)
    check_close(yj, yo, what="jds")
    short = np.diff(rp) <= 64
    assert np.array_equal(yj[short], yo[short])
    assert pj.info()["overflow_nnz"] > 0
    pj1 = sp.Plan.from_csr(m, m, rp, col, val, "jds", ell_width=2000)  # no overflow: all sequential
    assert np.array_equal(run_plan(pj1, x, m), yo)
    pc = sp.Plan.from_csr(m, m, rp, col, val, "coo")
    y = np.full(m, np.nan)
    pc.execute(x, y)
    check_close(y, yo, what="coo")
    # a row inside one 128-entry unit gets exactly one atomic: reproducible
    lens = np.diff(rp)
    inside = (rp[:-1] // 128 == (rp[1:] - 1) // 128) & (lens > 0)
    y2 = np.full(m, np.nan)
    pc.execute(x, y2)
    assert np.array_equal(y[inside], y2[inside])


def test_jds_identity_order_is_ell():
    """Rows already in non-increasing length order (equal lengths here): JDS
    keeps matrix order -- no permutation array, ELL's kernel and y, bit for
    bit; the oracle's sequential row sums too."""
    m = 30000
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=5))
    assert len(set(np.diff(rp).tolist())) == 1
    x = sp.generate_vector(m, seed=6)
    pj = sp.Plan.from_csr(m, m, rp, col, val, "jds")
    pe = sp.Plan.from_csr(m, m, rp, col, val, "ell")
    assert pj.info()["kernel"] == "ell_slice_kernel"
    yj, ye = run_plan(pj, x, m), run_plan(pe, x, m)
    assert np.array_equal(yj, ye)
    assert np.array_equal(yj, oracle_y(rp, col, val, x))


def test_integer_exact_all_formats():
    m = 40000
    spec = sp.gen_spec("powerlaw", m, max_len=2000, integer_values=True, seed=41)
    rp, col, val = sp.generate_csr(spec)
    x = sp.generate_vector(m, seed=43, integer_values=True)
    yo = oracle_y(rp, col, val, x)
    for fmt in ["csr", "ell", "ss", "hyb", "css", "coo", "jds", "bin"]:
        plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        if fmt == "bin":  # small integers: the long rows' run partials are exact too
            assert plan.info()["bin_long_rows"] > 0
        y = run_plan(plan, x, m)
        assert np.array_equal(y, yo), fmt


def test_rectangular_and_empty():
    rng = np.random.default_rng(3)
    for m, n in [(1, 1), (7, 1000), (1000, 7), (0, 5), (5, 1)]:
        lens = rng.integers(0, 5, size=m)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = rng.integers(0, n, size=rp[-1]).astype(np.int32)
        val = rng.random(rp[-1])
        x = rng.random(n)
        yo = oracle_y(rp, col, val, x) if m else np.zeros(0)
        for fmt in ["csr", "ell", "ss", "hyb", "css", "coo", "jds"]:
            plan = sp.Plan.from_csr(m, n, rp, col, val, fmt)
            y = np.full(m, 7.0)
            plan.execute(x, y)
            check_close(y, yo, what=f"{m}x{n} {fmt}")
    # all-empty matrix: y = 0
    plan = sp.Plan.from_csr(4, 4, np.zeros(5, np.int64), np.zeros(0, np.int32), np.zeros(0), "ss")
    y = np.full(4, 3.0)
    plan.execute(np.ones(4), y)
    assert (y == 0).all()


def test_no_columns_with_null_device_x():
    """m > 0, n = 0 (so nnz = 0): the API allows a NULL device x; every
    format writes y = 0 without reading x (the CSR row-group
    kernels read x unconditionally)."""
    import torch
    m = 1000
    rp = np.zeros(m + 1, np.int64)
    for fmt in ["csr", "ell", "ss", "hyb", "css", "coo", "jds", "bin", "dia", "auto"]:
        plan = sp.Plan.from_csr(m, 0, rp, np.zeros(0, np.int32), np.zeros(0), fmt)
        y = torch.full((m,), 5.0, dtype=torch.float64, device="cuda")
        st = sp.lib().spmv_execute(plan._h, None, C.c_void_p(y.data_ptr()), sp.X_DEVICE | sp.Y_DEVICE)
        assert st == 0, (fmt, sp.lib().spmv_last_error())
        assert (y.cpu().numpy() == 0).all(), fmt
        plan.destroy()


def test_device_pointers_and_streams():
    import torch
    m = 100000
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=2))
    x = sp.generate_vector(m, seed=3)
    yo = oracle_y(rp, col, val, x)
    for fmt in ["csr", "ell", "ss", "css"]:
        plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        xd = torch.from_numpy(x).cuda()
        yd = torch.full((m,), float("nan"), dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        plan.set_stream(s)
        with torch.cuda.stream(s):
            plan.execute(xd, yd)
        torch.cuda.synchronize()
        check_close(yd.cpu().numpy(), yo, what=fmt)
        ms = plan.time(xd, yd, 3)
        assert ms > 0


@pytest.mark.parametrize("long_len", [-1, 64])
def test_bin_x_staging_paths_agree(long_len):
    """The Mul stages x strips by LDS-DMA when x is 16-byte aligned and
    through registers when it is not (a device x at an 8-byte offset): both
    paths give the same y bit for bit, with and without long rows."""
    import torch
    m, n = 50_000, 90_001
    rp, col, val = _bin_matrix("powerlaw", m, n, seed=5)
    x = sp.generate_vector(n, seed=8)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_long_len=long_len)
    buf = torch.zeros(n + 2, dtype=torch.float64, device="cuda")
    assert buf.data_ptr() % 16 == 0
    out = []
    for off in (0, 1):
        xd = buf[off:off + n]
        xd.copy_(torch.from_numpy(x))
        yd = torch.full((m,), float("nan"), dtype=torch.float64, device="cuda")
        plan.execute(xd, yd)
        torch.cuda.synchronize()
        out.append(yd.cpu().numpy())
    assert np.array_equal(out[0], out[1])
    assert_bin_rows(plan, out[0], rp, col, val, x, what=f"x staging long_len {long_len}")


@pytest.mark.parametrize("fmt,gpus", [("", ""), ("bin", ""), ("css", ""), ("bin", "1"), ("", "1")])
def test_dropin_optimizeproblem_spmv(fmt, gpus, monkeypatch):
    """The reference-signature drop-in (include/opt_hip.h) via libopt_hip.so
    (format from SPMV_HIP_FORMAT, as the -DOPT_HIP_<FMT> build would fix it);
    SPMV_HIP_GPUS routes it through the multi-GPU plan (spmv_dist_*, here
    over the box's one device)."""
    if fmt:
        monkeypatch.setenv("SPMV_HIP_FORMAT", fmt)
    if gpus:
        monkeypatch.setenv("SPMV_HIP_GPUS", gpus)
    class SpMatC(C.Structure):
        _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int),
                    ("row_idx", C.c_void_p), ("col_idx", C.c_void_p), ("val", C.c_void_p)]

    class VecC(C.Structure):
        _fields_ = [("size", C.c_int), ("val", C.c_void_p)]

    class SpMatOptC(C.Structure):
        _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int), ("plan", C.c_void_p),
                    ("format", C.c_int), ("d_x", C.c_void_p), ("x_uploaded", C.c_int), ("dist", C.c_void_p),
                    ("n_gpus", C.c_int)]

    sp.lib()
    L = C.CDLL(sp.OPT_LIB_PATH)
    opt = getattr(L, "_Z15OptimizeProblemRK5SpMatRK3VecR8SpMatOptR6VecOpt")
    g = load_golden("mtx_random")
    m, n = int(g["m"]), int(g["n"])
    row, col, val, x = (np.ascontiguousarray(g[k]) for k in ("row", "col", "val", "x"))
    A = SpMatC(m, n, len(val), row.ctypes.data, col.ctypes.data, val.ctypes.data)
    xv = VecC(n, x.ctypes.data)
    y = np.full(m, 99.0)
    yv = VecC(m, y.ctypes.data)
    Ao, xo = SpMatOptC(), VecC()
    opt(C.byref(A), C.byref(xv), C.byref(Ao), C.byref(xo))
    assert xo.val == x.ctypes.data  # x_opt aliases x (src/opt_crs.cpp:11-12)
    for _ in range(2):
        L.SpMV(C.byref(Ao), C.byref(xo), C.byref(yv))
        assert sp.verify_result(sp.SpMat(m, n, row, col, val), x, y)
    check_close(y, g["y_crs"])
    assert bool(Ao.dist) == bool(gpus) and bool(Ao.plan) != bool(gpus)
    L.SpMVRelease(C.byref(Ao))


class _SpMatC(C.Structure):
    _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int),
                ("row_idx", C.c_void_p), ("col_idx", C.c_void_p), ("val", C.c_void_p)]


class _VecC(C.Structure):
    _fields_ = [("size", C.c_int), ("val", C.c_void_p)]


class _SpMatOptC(C.Structure):
    _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int), ("plan", C.c_void_p),
                ("format", C.c_int), ("d_x", C.c_void_p), ("x_uploaded", C.c_int), ("dist", C.c_void_p),
                ("n_gpus", C.c_int)]


def _dropin_y(row, col, val, x, m, n, calls=2, fetch=False):
    """OptimizeProblem + `calls` SpMV through libopt_hip.so (the drop-in);
    fetch: SpMVFetch after each call (SPMV_HIP_Y_RESIDENT=1).  Returns (y,
    the resolved layout)."""
    sp.lib()
    L = C.CDLL(sp.OPT_LIB_PATH)
    opt = getattr(L, "_Z15OptimizeProblemRK5SpMatRK3VecR8SpMatOptR6VecOpt")
    fetch_fn = getattr(L, "_Z9SpMVFetchRK8SpMatOptR3Vec", None) or getattr(L, "SpMVFetch")
    row, col, val, x = (np.ascontiguousarray(a) for a in (row, col, val, x))
    A = _SpMatC(m, n, len(val), row.ctypes.data, col.ctypes.data, val.ctypes.data)
    xv = _VecC(n, x.ctypes.data)
    y = np.full(m, 99.0)
    yv = _VecC(m, y.ctypes.data)
    Ao, xo = _SpMatOptC(), _VecC()
    opt(C.byref(A), C.byref(xv), C.byref(Ao), C.byref(xo))
    for _ in range(calls):
        y.fill(99.0)
        L.SpMV(C.byref(Ao), C.byref(xo), C.byref(yv))
        if fetch:
            fetch_fn(C.byref(Ao), C.byref(yv))
    fmt = sp.FORMAT_NAMES[Ao.format]
    L.SpMVRelease(C.byref(Ao))
    return y, fmt


@pytest.mark.parametrize("fetch", [False, True])
def test_dropin_crs_is_opt_crs_bit_for_bit(fetch, monkeypatch):
    """The drop-in's CRS (-DOPT_HIP_CRS / SPMV_HIP_FORMAT=crs) keeps opt_crs's
    semantics on the fastest layout that does so (spmv_options_t.crs_exact):
    y is the reference opt_crs y bit for bit on every golden fixture, and a
    config-2-like matrix (1 M x 1 M, 16 per row: x beyond L2) gets the BIN
    layout, bit-exact against the oracle.  With SPMV_HIP_Y_RESIDENT=1 y stays
    on the device until SpMVFetch."""
    monkeypatch.setenv("SPMV_HIP_FORMAT", "crs")
    if fetch:
        monkeypatch.setenv("SPMV_HIP_Y_RESIDENT", "1")
    for name in golden_names():
        g = load_golden(name)
        m, n = int(g["m"]), int(g["n"])
        y, fmt = _dropin_y(g["row"], g["col"], g["val"], g["x"], m, n, fetch=fetch)
        assert np.array_equal(y, g["y_crs"]), f"{name}: drop-in CRS ({fmt}) differs from opt_crs"
    m = 1_000_000
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=31))
    x = sp.generate_vector(m, seed=32)
    row = np.repeat(np.arange(m, dtype=np.int32), np.diff(rp))
    y, fmt = _dropin_y(row, col, val, x, m, m, fetch=fetch)
    assert fmt == "bin"
    assert np.array_equal(y, oracle_y(rp, col, val, x))
    # SPMV_HIP_CRS_EXACT=0: the CSR kernels themselves (butterfly sums)
    monkeypatch.setenv("SPMV_HIP_CRS_EXACT", "0")
    y, fmt = _dropin_y(row, col, val, x, m, m, fetch=fetch)
    assert fmt == "csr"
    check_close(y, oracle_y(rp, col, val, x))


@pytest.mark.parametrize("exact", ["", "1"])
def test_dropin_exact_switch(exact, monkeypatch):
    """SPMV_HIP_EXACT=1 keeps the drop-in's BIN plan off the run path: a
    power-law matrix's long rows are then the sequential opt_crs sum bit for
    bit; without it they are within 1e-12."""
    monkeypatch.setenv("SPMV_HIP_FORMAT", "bin")
    if exact:
        monkeypatch.setenv("SPMV_HIP_EXACT", exact)

    class SpMatC(C.Structure):
        _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int),
                    ("row_idx", C.c_void_p), ("col_idx", C.c_void_p), ("val", C.c_void_p)]

    class VecC(C.Structure):
        _fields_ = [("size", C.c_int), ("val", C.c_void_p)]

    class SpMatOptC(C.Structure):
        _fields_ = [("nRow", C.c_int), ("nCol", C.c_int), ("nNnz", C.c_int), ("plan", C.c_void_p),
                    ("format", C.c_int), ("d_x", C.c_void_p), ("x_uploaded", C.c_int), ("dist", C.c_void_p),
                    ("n_gpus", C.c_int)]

    sp.lib()
    L = C.CDLL(sp.OPT_LIB_PATH)
    opt = getattr(L, "_Z15OptimizeProblemRK5SpMatRK3VecR8SpMatOptR6VecOpt")
    m = 30_000
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", m, max_len=3000, seed=29))
    row = np.ascontiguousarray(np.repeat(np.arange(m, dtype=np.int32), np.diff(rp)))
    col = np.ascontiguousarray(col)
    x = sp.generate_vector(m, seed=31)
    A = SpMatC(m, m, len(val), row.ctypes.data, col.ctypes.data, val.ctypes.data)
    xv = VecC(m, x.ctypes.data)
    y = np.full(m, 99.0)
    yv = VecC(m, y.ctypes.data)
    Ao, xo = SpMatOptC(), VecC()
    opt(C.byref(A), C.byref(xv), C.byref(Ao), C.byref(xo))
    L.SpMV(C.byref(Ao), C.byref(xo), C.byref(yv))
    yo = oracle_y(rp, col, val, x)
    long_rows = np.diff(rp) >= 128
    assert long_rows.any()
    if exact:
        assert np.array_equal(y, yo)
    else:
        assert np.array_equal(y[~long_rows], yo[~long_rows])
        check_close(y, yo, what="drop-in bin, run path")
    L.SpMVRelease(C.byref(Ao))


@pytest.mark.parametrize("fmt,name", [("ss", "SS"), ("css", "CSS"), ("jds", "JDS"), ("coo", "COO"), ("bin", "BIN")])
def test_driver_binary_reports_block(fmt, name):
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mtx = os.path.join(root, "tests", "golden", "mtx", "random.mtx")
    out = subprocess.run([os.path.join(root, "bin", "spmv"), mtx, "--format", fmt],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "++++" in out.stdout and "Performance(GFLOPS)" in out.stdout
    assert f"MatrixFormat\t{name}" in out.stdout.replace(" ", "")
    # the block parses the way the reference's log tooling reads it
    # (log/format.cpp:32-49: a line of 40 '+' opens a record, each line is
    # "key value" split on whitespace, a line of 40 '-' closes it)
    records, cur = [], None
    for line in out.stdout.splitlines():
        if line == "+" * 40:
            cur = {}
        elif line == "-" * 40:
            records.append(cur)
            cur = None
        elif cur is not None:
            kv = line.split()
            if len(kv) >= 2:
                cur[kv[0]] = kv[1]
    assert len(records) == 1, out.stdout
    rec = records[0]
    assert (rec["Architecture"], rec["MatrixFormat"]) == ("GPU", name)
    assert (int(rec["nRow"]), int(rec["nCol"]), int(rec["nNnz"])) == (10, 10, 95)
    assert rec["Matrix"].startswith("random") and float(rec["Performance(GFLOPS)"]) > 0


def _with_empty_rows(rp, col, val, frac, seed):
    m = len(rp) - 1
    rng = np.random.default_rng(seed)
    lens = np.diff(rp)
    zero = rng.random(m) < frac
    zero[:3] = True
    zero[-5:] = True
    keep = np.repeat(~zero, lens)
    rp2 = np.concatenate([[0], np.cumsum(np.where(zero, 0, lens))]).astype(np.int64)
    return rp2, np.ascontiguousarray(col[keep]), np.ascontiguousarray(val[keep])


def _device_csr(rp, col, val):
    import torch
    return (torch.from_numpy(np.ascontiguousarray(rp, np.int64)).cuda(),
            torch.from_numpy(np.ascontiguousarray(col, np.int32)).cuda(),
            torch.from_numpy(np.ascontiguousarray(val, np.float64)).cuda())


DEVICE_FORMATS = [("csr", {}), ("csr", {"csr_lanes": 1}), ("ss", {"ss_sigma": 4}), ("ss", {"ss_sigma": 16}),
                  ("ss", {"ss_sigma": 32}), ("ss", {"ss_sigma": 64}), ("ss", {}), ("ell", {}), ("hyb", {}), ("hyb", {"ell_width": 4}),
                  ("jds", {}), ("jds", {"ell_width": 8}), ("dia", {}), ("coo", {}), ("css", {}),
                  ("css", {"css_slab_shift": 12}), ("bin", {}), ("bin", {"bin_long_len": 40}),
                  ("bin", {"bin_strip_cols": 3001}), ("bin", {"bin_product_order": 2}), ("auto", {})]


def _device_build_cases():
    cases = []
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", 30011, max_len=700, seed=5))
    cases.append(("powerlaw", 30011, 30011, rp, col, val))
    cases.append(("empty_rows", 30011, 30011) + _with_empty_rows(rp, col, val, 0.2, 1))
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", 4096, per_row=16, seed=6))
    cases.append(("nnz%T==0", 4096, 4096, rp, col, val))  # 65536 nnz: whole tiles
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", 2_100_000, per_row=3, seed=8))
    cases.append(("3-level scan", 2_100_000, 2_100_000) + _with_empty_rows(rp, col, val, 0.05, 2))
    cases.append(("rect", 7, 1000, np.array([0, 2, 2, 5, 5, 6, 9, 9], np.int64),
                  np.array([1, 999, 3, 4, 500, 0, 7, 8, 9], np.int32), np.arange(1.0, 10.0)))
    cases.append(("all-empty", 4, 4, np.zeros(5, np.int64), np.zeros(0, np.int32), np.zeros(0)))
    rp, col, val = sp.generate_csr(sp.gen_spec("banded", 70001, band_lo=-9, band_hi=6, seed=7))
    cases.append(("banded", 70001, 70001, rp, col, val))
    cases.append(("banded+empty", 70001, 70001) + _with_empty_rows(rp, col, val, 0.1, 4))
    # duplicates, unsorted columns and -0.0 values inside a band: the DIA
    # slots add duplicates in entry order from +0.0 (the host build's
    # val[at] += v), every other format keeps the entries as they are
    rng = np.random.default_rng(11)
    m = 5003
    lens = rng.integers(0, 9, m)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    rows = np.repeat(np.arange(m), lens)
    col = np.clip(rows + rng.integers(-3, 4, rows.size), 0, m - 1).astype(np.int32)
    val = rng.random(rows.size) + 0.01
    val[rng.random(rows.size) < 0.05] = -0.0
    cases.append(("banded dup/unsorted/-0", m, m, rp, col, val))
    return cases


def test_host_csr_build_routing():
    """spmv_options_t::build: a host CSR of >= 2^24 entries (AUTO) or any
    size (DEVICE) is staged into HBM and built by the device builders -- the
    host builder's layout byte for byte and the same y (BIN rows out of
    column order sorted by strip on the device first); small CSRs under AUTO
    stay on the host builders."""
    import torch
    # large: 1 M rows x 17 entries = 17 M entries, AUTO -> BIN (x too wide
    # for a window) built on the device
    m = 1_000_000
    spec = sp.gen_spec("uniform", m, per_row=17, seed=5)
    rp, col, val = sp.generate_csr(spec)
    assert int(rp[-1]) >= 1 << 24
    x = sp.generate_vector(m, seed=6)
    yo = oracle_y(rp, col, val, x)
    for fmt in ("auto", "ell", "csr", "css"):
        pa = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        assert pa.built_on_device(), fmt
        ph = sp.Plan.from_csr(m, m, rp, col, val, fmt, build="host")
        assert not ph.built_on_device()
        assert pa.info()["format"] == ph.info()["format"] and pa.info()["kernel"] == ph.info()["kernel"], fmt
        assert pa.digest() == ph.digest(), fmt
        ya, yh = run_plan(pa, x, m), run_plan(ph, x, m)
        assert np.array_equal(ya, yh), fmt
        check_close(ya, yo, what=f"routed {fmt}")
        pa.destroy()
        ph.destroy()
    # small: AUTO keeps the host builders, DEVICE forces the device ones
    cases = _device_build_cases()
    for name, mm, n, rp2, col2, val2 in cases[:4] + cases[-1:]:
        x2 = sp.generate_vector(n, seed=9)
        for fmt in ("auto", "dia", "hyb", "ss", "jds", "coo", "css", "bin"):
            try:
                ph = sp.Plan.from_csr(mm, n, rp2, col2, val2, fmt, build="host")
            except sp.SpmvError as e:
                assert "not supported" in str(e), (name, fmt, e)
                continue
            assert not sp.Plan.from_csr(mm, n, rp2, col2, val2, fmt).built_on_device()
            pd = sp.Plan.from_csr(mm, n, rp2, col2, val2, fmt, build="device")
            assert pd.built_on_device(), (name, fmt)  # every format, AUTO resolved alike
            assert pd.digest() == ph.digest(), (name, fmt)
            yd2, yh2 = run_plan(pd, x2, mm), run_plan(ph, x2, mm)
            if ph.info()["format"] == "coo":  # f64 atomics: unordered adds
                check_close(yd2, yh2, what=f"routed coo {name}")
            else:
                assert np.array_equal(yd2, yh2), (name, fmt)
            pd.destroy()
            ph.destroy()
    with pytest.raises(KeyError):
        sp.make_options("auto", build="sideways")


def test_device_conversion_matches_host_build():
    """spmv_plan_create_csr_device: every format built on the GPU (CSR, SS,
    ELL, HYB, JDS, DIA, COO, and AUTO resolved from device data) gives the
    host builder's layout byte for byte (spmv_plan_digest, array by array)
    and so the same y; a format the host refuses is refused on the device."""
    import torch
    for name, m, n, rp, col, val in _device_build_cases():
        x = sp.generate_vector(n, seed=9)
        yo = oracle_y(rp, col, val, x)
        drp, dcol, dval = _device_csr(rp, col, val)
        for fmt, kw in DEVICE_FORMATS:
            try:
                ph = sp.Plan.from_csr(m, n, rp, col, val, fmt, build="host", **kw)
            except sp.SpmvError as e:
                assert "not supported" in str(e), (name, fmt, e)
                with pytest.raises(sp.SpmvError, match="not supported"):
                    sp.Plan.from_device_csr(m, n, drp, dcol, dval, fmt, **kw)
                continue
            pd = sp.Plan.from_device_csr(m, n, drp, dcol, dval, fmt, **kw)
            ih, idv = ph.info(), pd.info()
            for k in ("format", "kernel", "empty_rows", "stored_slots", "algo_bytes", "n_kernels", "ell_width",
                      "n_diags", "overflow_nnz", "csr_lanes", "ss_sigma"):
                assert idv[k] == ih[k], f"{name} {fmt} {kw}: info {k} {idv[k]} != {ih[k]}"
            dh, dd = ph.digest(), pd.digest()
            assert list(dd) == list(dh), (name, fmt, list(dd), list(dh))
            bad = [a for a in dh if dh[a] != dd[a]]
            assert not bad, f"{name} {fmt} {kw}: device layout differs in {bad}"
            yh = run_plan(ph, x, m)
            yd = run_plan(pd, x, m)
            if ih["format"] == "coo":
                check_close(yd, yh, what=f"{name} coo")
            else:
                assert np.array_equal(yh, yd), f"{name} {fmt} {kw}: device build differs from host build"
            if m:
                check_close(yd, yo, what=f"{name} {fmt} {kw}")
            ph.destroy()
            pd.destroy()
    # the device-side validation refuses what the host path refuses
    rp = np.array([0, 2, 3], np.int64)
    bad_col = torch.tensor([0, 5, 1], dtype=torch.int32, device="cuda")
    v = torch.ones(3, dtype=torch.float64, device="cuda")
    with pytest.raises(sp.SpmvError, match="column index"):
        sp.Plan.from_device_csr(2, 5, torch.from_numpy(rp).cuda(), bad_col, v, "ss")
    with pytest.raises(sp.SpmvError, match="non-decreasing"):
        sp.Plan.from_device_csr(3, 6, torch.tensor([0, 2, 1, 3], device="cuda"), bad_col, v, "csr")
    with pytest.raises(sp.SpmvError, match=r"row_ptr\[m\]"):
        sp.Plan.from_device_csr(2, 6, torch.tensor([0, 2, 2], device="cuda"), bad_col, v, "ss")
    with pytest.raises(ValueError):
        sp.Plan.from_device_csr(2, 6, rp, bad_col, v, "csr")  # host row_ptr


def _fuzz_csr(seed):
    """A random CSR: mixed row lengths (empty rows, short rows, a few long
    ones), columns uniform, banded or clustered, duplicates possible, rows
    sorted or (some) shuffled."""
    rng = np.random.default_rng(seed)
    m = int(rng.integers(1, 4000))
    n = int(rng.choice([1, 7, 300, 5000, 70_000]))
    lens = rng.integers(0, int(rng.choice([2, 9, 40])), m)
    lens[rng.random(m) < 0.15] = 0
    if rng.random() < 0.5:  # a few long rows
        k = max(1, m // 200)
        lens[rng.choice(m, k, replace=False)] = rng.integers(100, 3000, k)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(rp[-1])
    rows = np.repeat(np.arange(m), lens)
    mode = seed % 3
    if mode == 0:
        col = rng.integers(0, n, nnz)
    elif mode == 1:  # banded around the diagonal
        col = np.clip(rows * n // max(m, 1) + rng.integers(-5, 6, nnz), 0, n - 1)
    else:  # clustered in a few column ranges
        c0 = rng.integers(0, n, 4)
        col = np.clip(c0[rng.integers(0, 4, nnz)] + rng.integers(0, 50, nnz), 0, n - 1)
    col = col.astype(np.int32)
    for r in range(m):  # sorted rows, except some shuffled ones
        a, z = rp[r], rp[r + 1]
        if z - a > 1:
            col[a:z] = np.sort(col[a:z]) if rng.random() > 0.1 else rng.permutation(col[a:z])
    val = rng.random(nnz) + 0.01
    return m, n, rp, col, val


FUZZ_FORMATS = [("csr", {}), ("ss", {}), ("ss", {"ss_sigma": 8}), ("ell", {}), ("hyb", {}), ("jds", {}), ("dia", {}),
                ("coo", {}), ("css", {}), ("bin", {}), ("bin", {"bin_long_len": 16}),
                ("bin", {"bin_strip_cols": 1000}), ("auto", {})]


@pytest.mark.parametrize("seed", range(40))
def test_device_build_fuzz(seed):
    """Random CSRs (mixed row lengths, duplicates, unsorted rows, several
    column patterns): every format built on the GPU from the device CSR is the
    host builder's layout byte for byte (spmv_plan_digest) with the same y;
    a format the host refuses is refused on the device too."""
    m, n, rp, col, val = _fuzz_csr(seed)
    x = sp.generate_vector(n, seed=seed + 100)
    yo = oracle_y(rp, col, val, x)
    drp, dcol, dval = _device_csr(rp, col, val)
    for fmt, kw in FUZZ_FORMATS:
        try:
            ph = sp.Plan.from_csr(m, n, rp, col, val, fmt, build="host", **kw)
        except sp.SpmvError as e:
            assert "not supported" in str(e), (seed, fmt, e)
            with pytest.raises(sp.SpmvError, match="not supported"):
                sp.Plan.from_device_csr(m, n, drp, dcol, dval, fmt, **kw)
            continue
        pd = sp.Plan.from_device_csr(m, n, drp, dcol, dval, fmt, **kw)
        assert pd.built_on_device() and pd.info()["format"] == ph.info()["format"], (seed, fmt, kw)
        dh, dd = ph.digest(), pd.digest()
        bad = [a for a in dh if dh[a] != dd.get(a)]
        assert list(dd) == list(dh) and not bad, f"seed {seed} {fmt} {kw}: layout differs in {bad}"
        yh, yd = run_plan(ph, x, m), run_plan(pd, x, m)
        if ph.info()["format"] == "coo":
            check_close(yd, yh, what=f"fuzz {seed} coo")
        else:
            assert np.array_equal(yd, yh), (seed, fmt, kw)
        check_close(yd, yo, what=f"fuzz {seed} {fmt} {kw}")
        ph.destroy()
        pd.destroy()


def test_profile_phases():
    """spmv_profile: the per-phase split (reference g_profile Mul/Sum)."""
    import torch
    m = 200000
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", m, max_len=2000, seed=4))
    x = torch.from_numpy(sp.generate_vector(m, seed=5)).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    want = {"csr": ["csr"], "ell": ["ell"], "jds": ["ell", "overflow"], "hyb": ["ell", "overflow"],
            "ss": ["tile", "fixup"], "css": ["sweep"], "coo": ["zero_y", "segment"]}
    for fmt, names in want.items():
        plan = sp.Plan.from_csr(m, m, rp, col, val, fmt, ell_width=8 if fmt == "hyb" else 0)
        prof = plan.profile(x, y, 5)
        assert list(prof) == names, (fmt, prof)
        assert all(v >= 0 for v in prof.values()) and sum(prof.values()) > 0
        yo = oracle_y(rp, col, val, x.cpu().numpy())
        check_close(y.cpu().numpy(), yo, what=f"profile {fmt}")


@pytest.mark.parametrize("args", [[], ["-", "1.0", "16"], ["-", "-0.5", "7"], ["-", "1.0", "40"], ["-", "2.0", "64"],
                                  [os.path.join(os.path.dirname(__file__), "golden", "mtx", "random.mtx")]])
def test_csr5_handle_api(args):
    """include/csr5_hip.h: the CSR5 benchmark's anonymouslibHandle flow
    (CSR5_cuda/main.cu call_anonymouslib) -- refuses spmv in CSR mode,
    y = alpha*A*x within 1e-10 of the benchmark's own check, identical on
    repeated calls, caller's arrays untouched; an explicit setSigma takes the
    nearest sigma of the SS kernel's set (7 -> 8, 40 -> 48, 64 -> 64)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([os.path.join(root, "bin", "csr5_api")] + args, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "-> OK" in out.stdout
    if len(args) == 3:
        assert f"sigma={ {'16': 16, '7': 8, '40': 48, '64': 64}[args[2]] } " in out.stdout, out.stdout


def test_execute_alpha():
    """spmv_execute_alpha: y = alpha * (A x), alpha applied to the finished row
    sums (one rounded multiply), every format, host and device buffers."""
    import torch
    m = 30000
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", m, max_len=900, seed=81))
    x = sp.generate_vector(m, seed=83)
    yo = oracle_y(rp, col, val, x)
    for fmt in ["csr", "ell", "ss", "css", "jds"]:
        plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        y1 = np.full(m, np.nan)
        plan.execute(x, y1)
        for alpha in (2.5, -1.0, 0.0):
            y = np.full(m, np.nan)
            plan.execute(x, y, alpha=alpha)
            assert np.array_equal(y, alpha * y1), (fmt, alpha)
        yd = torch.empty(m, dtype=torch.float64, device="cuda")
        plan.execute(torch.from_numpy(x).cuda(), yd, alpha=3.0)
        assert np.array_equal(yd.cpu().numpy(), 3.0 * y1)
        check_close(y1, yo, what=fmt)


@pytest.mark.parametrize("lanes", [1, 4, 32])
def test_csr_64bit_row_pointers(lanes):
    """The int64 row-pointer kernel instance (used from 2^31 nnz on), forced
    on a small matrix (option csr_row_ptr64): same y as the int32 instance,
    host and device builds."""
    import torch
    m = 40000
    rp, col, val = sp.generate_csr(sp.gen_spec("powerlaw", m, max_len=1200, seed=91))
    x = sp.generate_vector(m, seed=93)
    y32 = run_plan(sp.Plan.from_csr(m, m, rp, col, val, "csr", csr_lanes=lanes), x, m)
    p64 = sp.Plan.from_csr(m, m, rp, col, val, "csr", csr_lanes=lanes, csr_row_ptr64=True)
    assert p64.info()["row_ptr_bytes"] == 8
    assert np.array_equal(run_plan(p64, x, m), y32)
    pd = sp.Plan.from_device_csr(m, m, torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda(),
                                 torch.from_numpy(val).cuda(), "csr", csr_lanes=lanes, csr_row_ptr64=True)
    assert pd.info()["row_ptr_bytes"] == 8
    assert np.array_equal(run_plan(pd, x, m), y32)


def test_auto_format_choice():
    """AUTO follows the measured crossovers (profiles/round1/probe/
    auto_sweep.jsonl; round 2: bin_small/auto_cross.jsonl): banded -> DIA;
    x beyond ~6 MB and >= 8 M entries -> BIN; x beyond ~6 MB, fewer
    entries -> CSS; below that, near-uniform rows -> CSR, skewed rows -> SS."""
    cases = [(sp.gen_spec("banded", 300000, band_lo=-8, band_hi=8), "dia"),
             (sp.gen_spec("uniform", 4_000_000, per_row=6, seed=6), "bin"),
             (sp.gen_spec("uniform", 1_000_000, per_row=8, seed=1), "bin"),
             (sp.gen_spec("uniform", 1_000_000, per_row=4, seed=1), "css"),
             (sp.gen_spec("powerlaw", 1_000_000, max_len=500, seed=2), "css"),
             (sp.gen_spec("uniform", 400_000, per_row=8, seed=3), "csr"),
             (sp.gen_spec("powerlaw", 300_000, max_len=500, seed=4), "ss")]
    for spec, want in cases:
        rp, col, val = sp.generate_csr(spec)
        m = len(rp) - 1
        plan = sp.Plan.from_csr(m, m, rp, col, val, "auto")
        assert plan.info()["format"] == want, (spec.kind, m, plan.info()["format"])
        if m <= 400_000:
            x = sp.generate_vector(m, seed=5)
            check_close(run_plan(plan, x, m), oracle_y(rp, col, val, x), what=f"auto {want}")


# ---------------------------------------------------------------- BIN
# plan info fields that fix a BIN layout (host and device builds must agree)
BIN_LAYOUT_KEYS = ("format", "stored_slots", "bin_bins", "bin_strips", "bin_pad", "bin_groups", "bin_product_order",
                   "bin_sum_entries", "bin_long_len", "bin_long_rows", "bin_long_pieces", "bin_long_entries",
                   "bin_products")


def _bin_matrix(kind, m, n, seed):
    if kind == "empty_rows":
        spec = sp.gen_spec("powerlaw", m, n, max_len=700, seed=seed)
        rp, col, val = sp.generate_csr(spec)
        rng = np.random.default_rng(seed)
        lens = np.diff(rp)
        zero = rng.random(m) < 0.2
        zero[:11] = True
        zero[-13:] = True
        keep = np.repeat(~zero, lens)
        col, val = np.ascontiguousarray(col[keep]), np.ascontiguousarray(val[keep])
        rp = np.concatenate([[0], np.cumsum(np.where(zero, 0, lens))]).astype(np.int64)
        return rp, col, val
    spec = sp.gen_spec(kind, m, n, per_row=11, max_len=5000, seed=seed)
    return sp.generate_csr(spec)


@pytest.mark.parametrize("shape", [(40_000, 40_000), (30_011, 100_003), (70_001, 9_000), (5, 3), (1, 70_000)])
@pytest.mark.parametrize("kind", ["uniform", "powerlaw", "empty_rows"])
@pytest.mark.parametrize("opts", [{}, {"bin_strip_cols": 16384}, {"bin_strip_cols": 3001}, {"bin_groups": 3}])
def test_bin_bit_exact(shape, kind, opts):
    """BIN (binned Mul/Sum): every row is the sequential opt_crs sum bit for
    bit (one wave per bin adds its products in column order), for partial
    strips, rectangular shapes, empty rows, long rows and row groups."""
    m, n = shape
    rp, col, val = _bin_matrix(kind, m, n, seed=m % 97 + len(opts))
    x = sp.generate_vector(n, seed=31)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", **opts)
    y = run_plan(plan, x, m)
    assert_bin_rows(plan, y, rp, col, val, x, what=f"{shape} {kind} {opts}")
    if kind == "powerlaw" and m > 5:
        # the same rows with the run path off: every row bit-exact
        plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_long_len=-1, **opts)
        assert plan.info()["bin_long_len"] == 0
        assert np.array_equal(run_plan(plan, x, m), oracle_y(rp, col, val, x)), f"bin exact {shape} {opts}"


@pytest.mark.parametrize("long_len,opts", [(6, {}), (64, {}), (1000, {}), (64, {"bin_strip_cols": 3001}),
                                           (200, {"bin_sum_waves": 2, "bin_pad": 8}), (64, {"bin_sum_waves": 8})])
def test_bin_long_rows_run_path(long_len, opts):
    """The run path at explicit thresholds: rows with >=
    long_len entries are reduced per strip run in the Mul (pieces cut at
    64-entry blocks -- rows of 5000 entries over 2-17 strips give runs far
    longer than a block), the rest stay bit-exact; two plans agree bit for
    bit; plan info counts the long rows and at least one piece per run."""
    m, n = 60_000, 50_000
    rp, col, val = _bin_matrix("powerlaw", m, n, seed=long_len)
    x = sp.generate_vector(n, seed=3)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_long_len=long_len, **opts)
    info = plan.info()
    lens = np.diff(rp)
    assert info["bin_long_len"] == long_len
    assert info["bin_long_rows"] == int(np.sum(lens >= long_len)) > 0
    C = opts.get("bin_strip_cols", 20480)
    runs = sum(len(np.unique(col[rp[r]:rp[r + 1]] // C)) for r in np.flatnonzero(lens >= long_len))
    assert info["bin_long_pieces"] >= runs
    y = run_plan(plan, x, m)
    assert_bin_rows(plan, y, rp, col, val, x, what=f"long_len {long_len} {opts}")
    # the same plan from a device CSR: the long blocks laid out from the
    # rows' runs (k_bin_build.hip), the same layout, y bit-identical
    import torch
    pd = sp.Plan.from_device_csr(m, n, torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda(),
                                 torch.from_numpy(val).cuda(), "bin", bin_long_len=long_len, **opts)
    assert pd.built_on_device()
    idv = pd.info()
    for k in BIN_LAYOUT_KEYS:
        assert idv[k] == info[k], (long_len, opts, k, info[k], idv[k])
    assert pd.digest() == plan.digest(), (long_len, opts)
    assert np.array_equal(run_plan(pd, x, m), y), f"device long_len {long_len} {opts}"
    again = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_long_len=long_len, **opts)
    assert np.array_equal(run_plan(again, x, m), y)
    # signed values: the partials still meet the 1e-12 bound of sum |a x|
    sval = val * np.where(np.arange(len(val)) % 3 == 0, -1.0, 1.0)
    xs = x - 0.5
    ps = sp.Plan.from_csr(m, n, rp, col, sval, "bin", bin_long_len=long_len, **opts)
    assert_bin_rows(ps, run_plan(ps, xs, m), rp, col, sval, xs, what=f"signed long_len {long_len}")


@pytest.mark.parametrize("opts", [{"bin_pad": 8}, {"bin_pad": 16}, {"bin_pad": 32}, {"bin_sum_waves": 2},
                                  {"bin_sum_waves": 4}, {"bin_sum_waves": 8}, {"placement": "plain"},
                                  {"placement": "vmm"}])
def test_bin_layout_options(opts):
    """The layout options (product-line padding, Sum waves / bin rows) and the
    product-buffer placements (plain hipMalloc / 2-MB VMM handles) change
    speed only."""
    m = 120_000
    rp, col, val = _bin_matrix("powerlaw", m, m, seed=41)
    x = sp.generate_vector(m, seed=43)
    plan = sp.Plan.from_csr(m, m, rp, col, val, "bin", bin_groups=2, **opts)
    info = plan.info()
    if "bin_pad" in opts:
        assert info["bin_pad"] == opts["bin_pad"]
    if "bin_sum_waves" in opts:
        assert info["bin_sum_waves"] == opts["bin_sum_waves"]
    assert_bin_rows(plan, run_plan(plan, x, m), rp, col, val, x, what=str(opts))


@pytest.mark.parametrize("kind", ["uniform", "powerlaw", "banded", "empty_rows"])
@pytest.mark.parametrize("opts", [{}, {"bin_pad": 16}, {"bin_sum_waves": 4}, {"bin_strip_cols": 3001}])
def test_bin_product_orders(kind, opts):
    """Products in Mul order (the Mul writes its entries' products in place,
    unpadded; the Sum gathers each bin's segments in 8-entry chunks through
    the chunk table, k_bin.hip bin_sum_mo_kernel) and in Sum order (the Mul
    scatters them into padded segments) give the same y, bit for bit: the
    sequential opt_crs row sums."""
    m, n = 150_000, 170_003
    rp, col, val = _bin_matrix(kind, m, n, seed=5)
    x = sp.generate_vector(n, seed=6)
    ys = {}
    for order in (1, 2):
        plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_product_order=order, bin_long_len=-1, **opts)
        info = plan.info()
        assert info["bin_product_order"] == order
        if order == 2:  # the Mul's entries are not padded
            assert info["stored_slots"] == len(val) == info["bin_products"]
            assert info["bin_sum_entries"] >= len(val)
        ys[order] = run_plan(plan, x, m)
        assert_bin_rows(plan, ys[order], rp, col, val, x, what=f"order {order} {kind} {opts}")
    assert np.array_equal(ys[1], ys[2])
    # Mul order falls back to Sum order with long rows
    if kind == "powerlaw":
        lr = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_long_len=64, bin_product_order=2, **opts)
        assert lr.info()["bin_long_rows"] > 0 and lr.info()["bin_product_order"] == 1


def test_bin_auto_product_order():
    """AUTO picks the Mul order for short (bin, strip) segments -- a wide
    matrix like the multi-GPU rank shapes (here 20 K x 60 M, 16 per row:
    ~55 entries per segment) -- and the Sum order for long ones."""
    m, n = 20_000, 60_000_000
    spec = sp.gen_spec("uniform", m, n, per_row=16, seed=9)
    rp, col, val = sp.generate_csr(spec, 0, m)
    x = sp.generate_vector(n, seed=10)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "bin")
    assert plan.info()["bin_product_order"] == 2
    assert np.array_equal(run_plan(plan, x, m), oracle_y(rp, col, val, x))
    rp2, col2, val2 = _bin_matrix("uniform", 150_000, 170_003, seed=5)
    assert sp.Plan.from_csr(150_000, 170_003, rp2, col2, val2, "bin").info()["bin_product_order"] == 1


def _create_peak_drop(make):
    """(plan, peak drop of free device memory while `make()` runs): a thread
    polls hipMemGetInfo (torch.cuda.mem_get_info) during the create call."""
    import threading
    import torch
    torch.cuda.synchronize()
    base = torch.cuda.mem_get_info()[0]
    low = [base]
    stop = threading.Event()

    def poll():
        while not stop.is_set():
            low[0] = min(low[0], torch.cuda.mem_get_info()[0])

    t = threading.Thread(target=poll)
    t.start()
    try:
        plan = make()
    finally:
        stop.set()
        t.join()
    low[0] = min(low[0], torch.cuda.mem_get_info()[0])
    return plan, base - low[0]


@pytest.mark.parametrize("fmt,kind", [("bin", "uniform"), ("dia", "banded")])
def test_plan_create_holds_only_the_plan(fmt, kind):
    """AUTO placement: while a large BIN / DIA plan is created, free device
    memory never drops by more than the plan's own bytes (+128 MB of runtime
    slack); ten plans built in a row behave the same.  The placement search
    (an explicit opt-in) times its candidates and gives the same y bit for
    bit."""
    m = 4_000_000
    spec = sp.gen_spec(kind, m, per_row=16, band_lo=-20, band_hi=20, seed=21)
    rp, col, val = sp.generate_csr(spec)
    csr_bytes = 8 * (m + 1) + 12 * int(rp[-1])
    for i in range(10 if fmt == "bin" else 2):
        # the host builders (the device builders stage the CSR in HBM: below)
        plan, drop = _create_peak_drop(lambda: sp.Plan.from_csr(m, m, rp, col, val, fmt, build="host"))
        info = plan.info()
        # AUTO: BIN's product buffer (>= 32 MB) and DIA's values (>= 256 MB)
        # from 2-MB VMM handles
        assert info["format"] == fmt and info["placement"] == "vmm"
        assert drop <= info["device_bytes"] + (128 << 20), (i, drop, info["device_bytes"])
        if i == 0:
            x = sp.generate_vector(m, seed=22)
            y_auto = run_plan(plan, x, m)
        plan.destroy()
    # built on the device: the staged CSR (and the builders' scratch) on top
    plan, drop = _create_peak_drop(lambda: sp.Plan.from_csr(m, m, rp, col, val, fmt, build="device"))
    info = plan.info()
    assert plan.built_on_device() and info["placement"] == "vmm"
    assert drop <= info["device_bytes"] + 2 * csr_bytes + (128 << 20), (drop, info["device_bytes"], csr_bytes)
    assert np.array_equal(run_plan(plan, x, m), y_auto)
    plan.destroy()
    plan = sp.Plan.from_csr(m, m, rp, col, val, fmt, placement="search")
    info = plan.info()
    assert info["placement"] == "search" and info["placement_candidates"] >= 1
    assert 0 < info["placement_best_ms"] <= info["placement_worst_ms"]
    assert np.array_equal(run_plan(plan, x, m), y_auto)


def test_experiment_switches_do_not_reach_the_product_library(monkeypatch):
    """Every ablation / tuning variable of the probe build, set to a value that
    (in the probe build) skips stores, drops LDS adds or re-lays the data:
    the product library ignores them -- y stays bit-exact."""
    bad = {"SPMV_BIN_DEBUG": "6", "SPMV_BIN_PADLOG": "5", "SPMV_BIN_SUMWAVES": "8", "SPMV_BIN_SLOT_LINEAR": "1",
           "SPMV_BIN_REUSE": "1", "SPMV_BIN_SB": "2", "SPMV_BIN_CUS": "3", "SPMV_BIN_PLACEMENT": "3",
           "SPMV_BIN_HOST_BUILD": "1", "SPMV_CSS_DEBUG": "3", "SPMV_CSS_LAYOUT": "0", "SPMV_CSS_PIECE_DIV": "7",
           "SPMV_CSS_WGS": "5", "SPMV_DIA_DEBUG": "1", "SPMV_DIA_PLACEMENT": "2", "SPMV_ELL_UNROLL": "3",
           "SPMV_CSR_FORCE_RP64": "1", "SPMV_PLACEMENT_MODE": "9", "SPMV_VMM_CHUNK_MB": "1", "SPMV_BIN_ORDER": "1",
           "SPMV_LAUNCH_DEBUG": "16", "SPMV_LAUNCH_SS": "0", "SPMV_LAUNCH_SS_SPLIT": "136", "SPMV_LAUNCH_ELL_DBG": "1",
           "SPMV_LAUNCH_SS_WIN": "0", "SPMV_SS_KERNEL": "0"}
    for k, v in bad.items():
        monkeypatch.setenv(k, v)
    m = 60_000
    for kind, fmts in (("powerlaw", ["bin", "css", "csr", "ell", "ss"]), ("banded", ["dia", "bin", "ss"])):
        spec = sp.gen_spec(kind, m, max_len=900, band_lo=-5, band_hi=9, seed=12)
        rp, col, val = sp.generate_csr(spec)
        x = sp.generate_vector(m, seed=13)
        yo = oracle_y(rp, col, val, x)
        for fmt in fmts:
            plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
            info = plan.info()
            assert info["n_kernels"] >= 1 and info["row_ptr_bytes"] == 4
            y = run_plan(plan, x, m)
            if fmt == "bin":
                assert_bin_rows(plan, y, rp, col, val, x, what=f"{kind} with switches set")
            elif fmt in ("dia", "ell"):
                assert np.array_equal(y, yo), (kind, fmt)
            else:
                check_close(y, yo, what=f"{kind} {fmt} with switches set")


def test_lds_add_lane_order():
    """The named guard of BIN's and CSS's exactness (k_bin.hip, k_css.hip):
    lanes of ONE ds_add_f64 that hit the same LDS slot are applied in lane
    order.  Values are chosen so that any other order (reverse, pairwise
    tree, or a different lane permutation) rounds differently."""
    rng = np.random.default_rng(5)

    def lane_order(slots, vals):
        out = np.zeros(64)
        for r in range(len(slots) // 64):
            for lane in range(64):
                k = slots[r * 64 + lane]
                out[k] = out[k] + vals[r * 64 + lane]
        return out

    # 1) all 64 lanes on one slot: 1e16, 31 small values, -1e16, 31 small values
    v = np.concatenate([[1e16], 1.0 + rng.integers(0, 4, 31) * 0.25, [-1e16], 1.0 + rng.integers(0, 4, 31) * 0.25])
    s = np.zeros(64, np.int32)
    want = lane_order(s, v)
    rev = 0.0
    for t in v[::-1]:
        rev = rev + t
    assert want[0] != rev, "test values are not order-sensitive"
    assert np.array_equal(sp.lds_order_probe(s, v), want)
    # 2) k-major-like patterns: 4 slots interleaved, magnitudes spread, 16 rounds
    s = np.tile(np.arange(64, dtype=np.int32) % 4, 16)
    v = rng.choice([1e16, -1e16, 3.0, 0.1, 1e-3, 7e15], size=s.size) * rng.random(s.size)
    assert np.array_equal(sp.lds_order_probe(s, v), lane_order(s, v))
    # 3) random slots, runs of equal slots within one instruction
    s = np.sort(rng.integers(0, 64, size=64 * 32).reshape(32, 64), axis=1).astype(np.int32).ravel()
    v = rng.standard_normal(s.size) * 10.0 ** rng.integers(-8, 17, s.size)
    assert np.array_equal(sp.lds_order_probe(s, v), lane_order(s, v))


def test_bin_edge_cases():
    """No entries (y = 0), a single column, signed values (VerifyResult), the
    Mul/Sum profile split, and the option check."""
    m = 5000
    rp0 = np.zeros(m + 1, np.int64)
    plan = sp.Plan.from_csr(m, 10, rp0, np.zeros(0, np.int32), np.zeros(0), "bin")
    y = run_plan(plan, np.ones(10), m)
    assert not y.any()
    rp = np.arange(m + 1, dtype=np.int64)
    col = np.zeros(m, np.int32)
    val = np.linspace(-1.0, 1.0, m)
    plan = sp.Plan.from_csr(m, 1, rp, col, val, "bin")
    assert np.array_equal(run_plan(plan, np.array([3.0]), m), val * 3.0)
    rng = np.random.default_rng(7)
    spec = sp.gen_spec("uniform", 50_000, per_row=9, seed=3)
    rp, col, val = sp.generate_csr(spec)
    val = val * np.where(rng.random(len(val)) < 0.5, -1.0, 1.0)
    x = sp.generate_vector(50_000, seed=9) - 0.5
    plan = sp.Plan.from_csr(50_000, 50_000, rp, col, val, "bin")
    y = run_plan(plan, x, 50_000)
    assert np.array_equal(y, oracle_y(rp, col, val, x))
    import torch
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty(50_000, dtype=torch.float64, device="cuda")
    ph = plan.profile(xd, yd, 3)
    assert list(ph) == ["mul", "sum"], ph
    with pytest.raises(sp.SpmvError):
        sp.Plan.from_csr(50_000, 50_000, rp, col, val, "bin", bin_strip_cols=20481)


@pytest.mark.parametrize("sum_waves", [0, 2])
def test_bin_empty_bins_between_full_ones(sum_waves):
    """Bins without products among a wave's bins (runs of empty rows longer
    than a bin, 2+ bins per Sum wave): the Sum walks all of a wave's bins with
    one batch cursor (the next bin's loads in flight during the write-back),
    so an empty bin must still get its zeros -- y starts as garbage here."""
    m, n = 6_000_000, 1_000_000
    rng = np.random.default_rng(17)
    lens = np.zeros(m, np.int64)
    lens[100_000:3_000_000] = 2
    lens[3_200_000:m] = 1
    lens[4_000_000:4_040_000] = 0  # an empty stretch in the middle of the wave sequence
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(rp[-1])
    col = np.sort(rng.integers(0, n, size=nnz).astype(np.int32).reshape(-1, 1), axis=1).ravel()
    # columns ascending within each row (2-entry rows: sort pairs)
    two = np.flatnonzero(lens == 2)
    starts = rp[two]
    a, b = col[starts], col[starts + 1]
    col[starts], col[starts + 1] = np.minimum(a, b), np.maximum(a, b)
    val = rng.random(nnz) + 0.5
    x = sp.generate_vector(n, seed=5)
    plan = sp.Plan.from_csr(m, n, rp, col, val, "bin", bin_sum_waves=sum_waves)
    info = plan.info()
    assert info["bin_bins"] >= 1024  # two or more bins per Sum wave
    y = run_plan(plan, x, m)
    assert np.array_equal(y, oracle_y(rp, col, val, x))
    assert not y[:100_000].any() and not y[4_000_000:4_040_000].any()


@pytest.mark.parametrize("opts", [{}, {"bin_strip_cols": 3001}, {"bin_groups": 3}, {"bin_product_order": 1}])
def test_bin_device_build(opts, monkeypatch):
    """spmv_plan_create_csr_device with BIN: the segments (and the long rows'
    run path) are counted, laid out and filled on the GPU (k_bin_build.hip).
    The host builder's layout byte for byte (spmv_plan_digest) and y
    bit-identical to it and to the oracle; rows whose column strips are not
    ascending are sorted by strip on the device first, same layout."""
    import torch
    cases = [("uniform", 40_000, 40_000), ("powerlaw", 30_011, 100_003), ("empty_rows", 70_001, 9_000),
             ("uniform", 5, 3), ("powerlaw", 1, 70_000)]
    for kind, m, n in cases:
        rp, col, val = _bin_matrix(kind, m, n, seed=m % 89)
        x = sp.generate_vector(n, seed=17)
        yo = oracle_y(rp, col, val, x)
        ph = sp.Plan.from_csr(m, n, rp, col, val, "bin", **opts)
        pd = sp.Plan.from_device_csr(m, n, torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda(),
                                     torch.from_numpy(val).cuda(), "bin", **opts)
        ih, idv = ph.info(), pd.info()
        assert pd.built_on_device() and not ph.built_on_device()
        for k in BIN_LAYOUT_KEYS:
            assert ih[k] == idv[k], (kind, m, n, k, ih[k], idv[k])
        assert pd.digest() == ph.digest(), (kind, m, n, opts)
        yd = run_plan(pd, x, m)
        assert np.array_equal(yd, run_plan(ph, x, m)), f"{kind} {m}x{n} {opts}"
        assert_bin_rows(pd, yd, rp, col, val, x, what=f"device {kind} {m}x{n} {opts}")
    # unsorted rows (strips descending inside some rows) -> host builder
    rp, col, val = _bin_matrix("powerlaw", 50_000, 50_000, seed=3)
    col = col.copy()
    for r in range(0, 50_000, 7):
        col[rp[r]:rp[r + 1]] = col[rp[r]:rp[r + 1]][::-1]
    x = sp.generate_vector(50_000, seed=5)
    pd = sp.Plan.from_device_csr(50_000, 50_000, torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda(),
                                 torch.from_numpy(val).cuda(), "bin", **opts)
    ph = sp.Plan.from_csr(50_000, 50_000, rp, col, val, "bin", build="host", **opts)
    assert pd.built_on_device() and pd.digest() == ph.digest()
    yd = run_plan(pd, x, 50_000)
    assert np.array_equal(yd, run_plan(ph, x, 50_000))
    # BIN adds a row's strips in strip order: with unsorted columns that is
    # not the CSR order the oracle follows, so rounding may differ
    check_close(yd, oracle_y(rp, col, val, x), what="unsorted rows")
    # all-empty
    pd = sp.Plan.from_device_csr(6, 6, torch.zeros(7, dtype=torch.int64, device="cuda"),
                                 torch.zeros(0, dtype=torch.int32, device="cuda"),
                                 torch.zeros(0, dtype=torch.float64, device="cuda"), "bin")
    assert not run_plan(pd, np.ones(6), 6).any()


# ---------------------------------------------------------------- full size
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_full_size_headline_bit_exact(config):
    """BASELINE configs 2 and 3 at their full size (160 M / 29.6 M entries):
    the AUTO plan (BIN) against the oracle's opt_crs restatement -- bit for
    bit -- plus linearity A(x1 + x2) = A x1 + A x2 to fp64 rounding; at
    config 2 also CSR, ELL, SS and CSS (the formats the bench line times beside
    AUTO), at config 3 HYB, CSR, SS and CSS: 1e-12, ELL (column order) bit for
    bit."""
    import torch
    if config == "c2":
        spec = sp.gen_spec("uniform", 10_000_000, per_row=16, seed=42)
    else:
        spec = sp.gen_spec("powerlaw", 5_000_000, max_len=10000, alpha=2.0, seed=42)
    rp, col, val = sp.generate_csr(spec)
    m = len(rp) - 1
    plan = sp.Plan.from_csr(m, m, rp, col, val, "auto")
    assert plan.info()["format"] == "bin"
    x1 = sp.generate_vector(m, seed=43)
    x2 = sp.generate_vector(m, seed=44)
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    outs = []
    for xv in (x1, x2, x1 + x2):
        plan.execute(torch.from_numpy(xv).cuda(), y)
        outs.append(y.cpu().numpy().copy())
    assert_bin_rows(plan, outs[0], rp, col, val, x1, what=config)
    if config == "c3":  # power-law rows: the long ones take the run path
        assert plan.info()["bin_long_rows"] > 0
    lin = np.abs(outs[2] - (outs[0] + outs[1]))
    assert np.all(lin <= 1e-12 * np.abs(outs[2]) + 1e-300)
    plan.destroy()
    # c3: the named ELL + CSR hybrid and the other skew-tolerant formats; c2:
    # every format the bench line times beside AUTO -- at full size against the
    # same oracle (each folds in its own fixed order: 1e-12 relative)
    yo = oracle_y(rp, col, val, x1)
    xd = torch.from_numpy(x1).cuda()
    for fmt in (("csr", "ell", "ss", "css") if config == "c2" else ("hyb", "csr", "ss", "css")):
        p2 = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        y.fill_(float("nan"))
        p2.execute(xd, y)
        if fmt == "ell":
            assert np.array_equal(y.cpu().numpy(), yo), f"{config} {fmt}"
        else:
            check_close(y.cpu().numpy(), yo, what=f"{config} {fmt}")
        p2.destroy()



def test_full_size_c5_rank_shape():
    """Rank 0 of BASELINE config 5 (80 M x 80 M, 16 nnz/row, row-partitioned
    over 8 GPUs): its 10 M rows over all 80 M columns with the 640 MB x, the
    AUTO plan (BIN with 2 Sum waves), bit for bit against the oracle's opt_crs
    restatement, plus linearity A(x1 + x2) = A x1 + A x2."""
    import torch
    world, rows = 8, 10_000_000
    spec = sp.gen_spec("uniform", world * rows, per_row=16, seed=42)
    rp, col, val = sp.generate_csr(spec, 0, rows)
    n = world * rows
    plan = sp.Plan.from_csr(rows, n, rp, col, val, "auto")
    info = plan.info()
    assert info["format"] == "bin" and info["n"] == n and info["nnz"] == 16 * rows
    x1 = sp.generate_vector(n, seed=43)
    x2 = sp.generate_vector(n, seed=44)
    y = torch.empty(rows, dtype=torch.float64, device="cuda")
    outs = []
    for xv in (x1, x2, x1 + x2):
        plan.execute(torch.from_numpy(xv).cuda(), y)
        outs.append(y.cpu().numpy().copy())
    assert np.array_equal(outs[0], oracle_y(rp, col, val, x1))
    lin = np.abs(outs[2] - (outs[0] + outs[1]))
    assert np.all(lin <= 1e-12 * np.abs(outs[2]) + 1e-300)
    plan.destroy()


def test_full_size_c4_banded():
    """BASELINE config 4 at full size: 20 M rows, diagonals -32..+31 (64),
    1.28 G entries -- the largest index range in the product.  The DIA, ELL
    and JDS plans bit for bit and the CSR (16 lanes per row) and SS plans to
    1e-12 against the oracle's opt_crs restatement."""
    import torch
    m = 20_000_000
    spec = sp.gen_spec("banded", m, band_lo=-32, band_hi=31, seed=42)
    rp, col, val = sp.generate_csr(spec)
    assert int(rp[-1]) == 64 * m - 1024  # rows 0..31 and the last 31 rows are clipped
    x = sp.generate_vector(m, seed=43)
    yo = oracle_y(rp, col, val, x)
    xd = torch.from_numpy(x).cuda()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    plan = sp.Plan.from_csr(m, m, rp, col, val, "dia", build="host")
    assert plan.info()["n_diags"] == 64 and not plan.built_on_device()
    plan.execute(xd, y)
    assert np.array_equal(y.cpu().numpy(), yo)
    # the same DIA plan built on the device from the CSR in HBM (f2): byte-
    # identical layout, bit-exact y, and AUTO resolves to DIA there too
    dh = plan.digest()
    plan.destroy()
    del plan
    drp, dcol, dval = _device_csr(rp, col, val)
    for fmt in ("dia", "auto"):
        t0 = time.perf_counter()
        pd = sp.Plan.from_device_csr(m, m, drp, dcol, dval, fmt)
        t_build = time.perf_counter() - t0
        assert pd.info()["format"] == "dia"
        assert pd.digest() == dh, f"device {fmt}: layout differs from the host build"
        y.fill_(float("nan"))
        pd.execute(xd, y)
        assert np.array_equal(y.cpu().numpy(), yo)
        print(f"c4 device {fmt} plan built in {t_build:.3f} s")
        pd.destroy()
    del drp, dcol, dval, pd
    torch.cuda.empty_cache()
    # the other config-4 formats, built through the host-CSR routing (>= 2^24
    # entries: the device builders): ELL / JDS sum each row in column order
    # (bit for bit), CSR / SS fold in their own fixed order (1e-12)
    for fmt in ("csr", "ell", "jds", "ss"):
        plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
        assert plan.built_on_device(), fmt
        y.fill_(float("nan"))
        plan.execute(xd, y)
        if fmt in ("ell", "jds"):
            assert np.array_equal(y.cpu().numpy(), yo), f"c4 {fmt}"
        else:
            check_close(y.cpu().numpy(), yo, what=f"c4 {fmt}")
        plan.destroy()


def test_bin_refuses_huge_sparse_grid_and_auto_avoids_it():
    """A very sparse, very wide matrix: BIN's (bin, strip) segments would be
    nearly empty (all padding) -- AUTO does not pick BIN; a segment grid
    beyond 2^28 is refused with NOT_SUPPORTED."""
    rng = np.random.default_rng(3)
    # short segments -> 2 Sum waves, 10239-row bins: 3584 bins x 97657 strips > 2^28
    m, n, per = 32_000_000, 2_000_000_000, 2
    rp = np.arange(0, per * m + 1, per, dtype=np.int64)
    col = np.sort(rng.integers(0, n, size=(m, per)), axis=1).astype(np.int32).ravel()
    val = rng.random(per * m)
    with pytest.raises(sp.SpmvError, match="not supported"):
        sp.Plan.from_csr(m, n, rp, col, val, "bin")
    m2, n2, per2 = 4_000_000, 400_000_000, 6  # 782 bins x 19532 strips: 1.6 entries per segment
    rp2 = np.arange(0, per2 * m2 + 1, per2, dtype=np.int64)
    col2 = np.sort(rng.integers(0, n2, size=(m2, per2)), axis=1).astype(np.int32).ravel()
    plan = sp.Plan.from_csr(m2, n2, rp2, col2, rng.random(per2 * m2), "auto")
    assert plan.info()["format"] != "bin"


def test_bandwidth_probes_report_plausible_rates():
    """The live ceilings bench.py prices its roofline fields with: STREAM
    read, nontemporal write, mixed read+write (3/4 written back) -- each a
    positive rate below the 8 TB/s HBM spec; argument errors are refused."""
    r = sp.stream_probe(0, 512 << 20, 3)
    w = sp.stream_write_probe(0, 512 << 20, 3)
    m = sp.mixed_probe(0, 512 << 20, 3, 3)
    for v in (r, w, m):
        assert 500.0 < v < 8000.0, (r, w, m)
    with pytest.raises(sp.SpmvError):
        sp.mixed_probe(0, 512 << 20, 5, 3)


@pytest.mark.parametrize("fmt", ["csr", "ell", "ss", "hyb", "dia", "coo", "jds", "bin"])
def test_graph_replays_the_execute(fmt):
    """spmv_graph_*: reps executes captured in one HIP graph give the
    spmv_execute y bit for bit on every launch (COO: its f64 atomics, 1e-12),
    on the null stream and on a side stream; CSS is refused."""
    import torch
    m = 60_013
    if fmt == "dia":
        rp, col, val = sp.generate_csr(sp.gen_spec("banded", m, band_lo=-5, band_hi=6, seed=4))
    else:
        rp, col, val = _bin_matrix("powerlaw" if fmt in ("hyb", "jds", "ss") else "uniform", m, m, 4)
    x = sp.generate_vector(m, seed=5)
    plan = sp.Plan.from_csr(m, m, rp, col, val, fmt)
    xd = torch.from_numpy(x).cuda()
    ye = torch.full((m,), float("nan"), dtype=torch.float64, device="cuda")
    plan.execute(xd, ye)
    torch.cuda.synchronize()
    y_exec = ye.cpu().numpy()
    if fmt == "bin":
        assert_bin_rows(plan, y_exec, rp, col, val, x, "exec")
    else:
        check_close(y_exec, oracle_y(rp, col, val, x), what=fmt)
    yg = torch.full((m,), float("nan"), dtype=torch.float64, device="cuda")
    g = plan.graph(xd, yg, reps=3)
    for stream in (None, torch.cuda.Stream()):
        plan.set_stream(stream)
        for _ in range(2):
            yg.fill_(float("nan"))
            torch.cuda.synchronize()
            g.launch()
            y = yg.cpu().numpy()
            if fmt == "coo":
                check_close(y, y_exec, what="coo graph")
            else:
                assert np.array_equal(y, y_exec), f"{fmt}: graph y differs from execute"
        assert g.time(2) > 0
    plan.set_stream(None)
    g.destroy()
    css = sp.Plan.from_csr(m, m, rp, col, val, "css")
    with pytest.raises(sp.SpmvError, match="not supported"):
        css.graph(xd, yg)


def test_device_build_oom_falls_back_to_host_builders():
    """A host CSR of >= 2^24 entries is staged into HBM and built there (build
    AUTO); when the device builders' own scratch does not fit, the plan must
    still come from the host builders (status OUT_OF_MEMORY -> host route,
    HIP's sticky error cleared), never fail with a HIP error.  HBM is filled
    with a blocker so that only the staging copy plus a small margin stays
    free; the margins sweep across the SS builder's scratch (16 B per row)."""
    import torch
    spec = sp.gen_spec("uniform", 1_100_000, per_row=16, seed=21)
    rp, col, val = sp.generate_csr(spec)
    m, nnz = len(rp) - 1, int(rp[-1])
    assert nnz >= 1 << 24  # the AUTO build routes this host CSR through the device builders
    x = sp.generate_vector(m, seed=22)
    yo = oracle_y(rp, col, val, x)
    staging = 8 * (m + 1) + 12 * nnz
    outcomes, host_built = [], False
    for margin_mb in (4, 12, 20, 28, 40, 64, 128):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        free, _ = torch.cuda.mem_get_info()
        blocker = torch.empty(free - staging - (margin_mb << 20), dtype=torch.uint8, device="cuda")
        try:
            p = sp.Plan.from_csr(m, m, rp, col, val, "ss")
        except sp.SpmvError as e:  # the host plan may not fit either: then the error must say so
            assert "out of memory" in str(e), f"margin {margin_mb} MB: {e}"
            outcomes.append((margin_mb, "oom"))
            continue
        finally:
            del blocker
            torch.cuda.empty_cache()
        on_dev = p.built_on_device()
        outcomes.append((margin_mb, "device" if on_dev else "host"))
        y = np.full(m, np.nan)
        p.execute(x, y)
        check_close(y, yo, what=f"ss, margin {margin_mb} MB, built on {'device' if on_dev else 'host'}")
        p.destroy()
        host_built |= not on_dev
        if on_dev:  # the scratch fits from here on
            break
    print("device-build OOM sweep:", outcomes)
    assert host_built, f"no margin exercised the host fallback: {outcomes}"


def test_fetch_y_serves_only_the_latest_staged_execute():
    """spmv_fetch_y returns the y of the latest execute when that execute was
    SPMV_Y_STAGED; after any other execute it refuses instead of handing back
    an older y."""
    import torch
    m = 20_000
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=8, seed=3))
    x = sp.generate_vector(m, seed=4)
    p = sp.Plan.from_csr(m, m, rp, col, val, "csr")
    L = sp.lib()
    y = np.full(m, np.nan)
    assert L.spmv_execute(p._h, x.ctypes.data, None, sp.Y_STAGED) == 0
    assert L.spmv_fetch_y(p._h, y.ctypes.data) == 0
    check_close(y, oracle_y(rp, col, val, x))
    yd = torch.empty(m, dtype=torch.float64, device="cuda")
    p.execute(torch.from_numpy(x).cuda(), yd)  # device y: the staged y is no longer the latest
    assert L.spmv_fetch_y(p._h, y.ctypes.data) == 1  # SPMV_ERROR_INVALID_VALUE
    yh = np.empty(m)
    p.execute(x, yh)  # host y (staging buffer + D2H): not a staged execute either
    assert L.spmv_fetch_y(p._h, y.ctypes.data) == 1
    assert L.spmv_execute(p._h, x.ctypes.data, None, sp.Y_STAGED) == 0
    assert L.spmv_fetch_y(p._h, y.ctypes.data) == 0 and np.array_equal(y, yh)
    p.destroy()


def test_crs_exact_skips_bin_for_rows_out_of_column_order():
    """crs_exact promises the sequential column-order sum bit for bit: BIN
    sums a row strip by strip, so a matrix whose rows are not strictly
    ascending (here every 7th row reversed, which AUTO would still route to
    BIN) must get a layout that sums in CSR order (ELL at 16 per row), and y
    must equal the oracle's opt_crs restatement bit for bit."""
    m = 1_000_000
    rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=31))
    col = col.copy()
    for r in range(0, m, 7):
        col[rp[r]:rp[r + 1]] = col[rp[r]:rp[r + 1]][::-1]
    x = sp.generate_vector(m, seed=32)
    pa = sp.Plan.from_csr(m, m, rp, col, val, "auto")
    assert pa.info()["format"] == "bin"
    pa.destroy()
    p = sp.Plan.from_csr(m, m, rp, col, val, "csr", crs_exact=True)
    assert p.info()["format"] in ("ell", "csr"), p.info()["format"]
    y = np.full(m, np.nan)
    p.execute(x, y)
    assert np.array_equal(y, oracle_y(rp, col, val, x))
    p.destroy()
