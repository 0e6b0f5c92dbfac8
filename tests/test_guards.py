"""CPU-side guards of the product library (no GPU needed):

* the experiment switches (SPMV_<FMT>_* environment variables, ablation
  kernels) exist only in the probe build -- the product library cannot be
  steered into a wrong or slow mode by a stray variable;
* the LDS adds that BIN's and CSS's bit-exact sums rest on compile to ONE
  ds_add_f64 per wave instruction (no CAS loop, whose lane order would be
  unspecified); the hardware ordering itself is checked on the GPU
  (test_gpu_parity.py::test_lds_add_lane_order);
* the Python mirror refuses vectors of the wrong dtype / length / layout /
  device before any address reaches the C-ABI;
* bench.py --gpus N self-launches N ranks through torch.distributed.run.
"""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

import singlespmv_amd as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "singlespmv_amd", "csrc")
PROBE_VARS = ["SPMV_BIN_DEBUG", "SPMV_BIN_PADLOG", "SPMV_BIN_SUMWAVES", "SPMV_BIN_REUSE",
              "SPMV_BIN_SB", "SPMV_BIN_CUS", "SPMV_BIN_PLACEMENT", "SPMV_BIN_HOST_BUILD", "SPMV_CSS_DEBUG",
              "SPMV_CSS_LAYOUT", "SPMV_CSS_PIECE_DIV", "SPMV_CSS_WGS", "SPMV_DIA_DEBUG", "SPMV_DIA_PLACEMENT",
              "SPMV_ELL_UNROLL", "SPMV_CSR_FORCE_RP64", "SPMV_PLACEMENT_MODE", "SPMV_VMM_CHUNK_MB", "SPMV_BIN_ORDER",
              "SPMV_LAUNCH_DEBUG", "SPMV_VMM_ALIGN_MB", "SPMV_VMM_STRIDE", "SPMV_VMM_SHUFFLE", "SPMV_DIA_GROUP",
              "SPMV_DIA_LDS_KB", "SPMV_LAUNCH_DIA_LDS_KB", "SPMV_ARENA_VMM_MB", "SPMV_LAUNCH_CSR",
              "SPMV_LAUNCH_CSR_U", "SPMV_LAUNCH_CSR_LDS_KB", "SPMV_LAUNCH_CSR_S", "SPMV_LAUNCH_ELL_O32", "SPMV_LAUNCH_ELL_UNROLL", "SPMV_LAUNCH_ELL_LDS_KB",
              "SPMV_BIN_MUL_PERM", "SPMV_BIN_PLACEMENT_GAP_MB", "SPMV_CSR_VAL_PLAIN", "SPMV_LAUNCH_COO_U",
              "SPMV_LAUNCH_COO_BLOCKS", "SPMV_LAUNCH_SS_WIN"]


def _strings(path):
    return subprocess.check_output(["strings", "-a", path], text=True)


def test_product_library_reads_no_experiment_switch():
    s = _strings(os.path.join(ROOT, "singlespmv_amd", "libspmv_hip.so"))
    present = [v for v in PROBE_VARS if v in s]
    assert not present, f"product library still reads {present}"
    # the drop-in's two documented switches are the only SPMV_ variables left
    assert set(re.findall(r"SPMV_[A-Z0-9_]+", _strings(sp.OPT_LIB_PATH))) >= {"SPMV_HIP_FORMAT"}


def test_probe_build_reads_them():
    subprocess.check_call(["make", "-s", "-j8", "probes"], cwd=ROOT)
    s = _strings(os.path.join(ROOT, "probes_build", "libspmv_hip.so"))
    assert all(v in s for v in ("SPMV_BIN_DEBUG", "SPMV_CSS_DEBUG", "SPMV_DIA_DEBUG", "SPMV_PLACEMENT_MODE"))


def test_product_library_holds_no_probe_kernel_instances():
    """The probe-only kernels and launch variants (round 4's ss_tile_kernel,
    the SS prefetch depths 1 / 4 and unstaged rows, csr_vec4) are compiled
    into the probe build only: the product library instantiates the launch
    shapes it runs and nothing else (12.7 MiB before)."""
    lib = os.path.join(ROOT, "singlespmv_amd", "libspmv_hip.so")
    syms = subprocess.check_output(["nm", "-C", lib], text=True)
    assert "ss_tile_kernel" not in syms and "csr_vec4_kernel" not in syms
    ss = re.findall(r"ss_stream_kernel<(\d+), (true|false), (\d+), (true|false)>", syms)
    assert ss and all(pf == "2" and st == "true" for _, _, pf, st in ss), sorted(set(ss))
    assert os.path.getsize(lib) < 10 << 20


def _device_asm(src):
    return subprocess.check_output(
        ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-Iinclude", "-Isinglespmv_amd/csrc", "--offload-arch=gfx950",
         "-munsafe-fp-atomics", "-ffp-contract=off", "--cuda-device-only", "-S", "-o", "-", src],
        cwd=ROOT, text=True, stderr=subprocess.DEVNULL)


def _kernel_bodies(asm, name_part):
    """Device assembly of every kernel whose mangled name contains name_part."""
    out = []
    for m in re.finditer(r"^(_Z\S*" + name_part + r"\S*):", asm, flags=re.M):
        end = asm.find("s_endpgm", m.end())
        out.append(asm[m.end():end])
    return out


@pytest.mark.parametrize("src,kernel", [("k_probe.hip", "lds_order_kernel"), ("k_bin.hip", "bin_sum_kernel"),
                                        ("k_bin.hip", "bin_sum_bin_kernel"), ("k_css.hip", "css_sweep_kernel")])
def test_lds_adds_are_single_ds_add_f64(src, kernel):
    bodies = _kernel_bodies(_device_asm(os.path.join("singlespmv_amd", "csrc", src)), kernel)
    assert bodies, f"no {kernel} in {src}"
    for b in bodies:
        assert "ds_add_f64" in b or "ds_add_rtn_f64" in b, f"{kernel}: LDS f64 add is not ds_add_f64"
        assert "ds_cmpst" not in b and "ds_cmpswap" not in b, f"{kernel}: CAS loop"


def test_lds_dma_strips_drained_before_the_barrier():
    """The Mul's x strips staged by LDS-DMA (global_load_lds) are read by the
    other waves after the workgroup barrier: every such body waits for
    vmcnt(0) between its last DMA load and the next s_barrier (the source
    asks for it explicitly; this keeps a compiler change from dropping it)."""
    bodies = [b for b in _kernel_bodies(_device_asm(os.path.join("singlespmv_amd", "csrc", "k_bin.hip")),
                                        "bin_mul_kernel") if "global_load_lds" in b]
    assert bodies, "no LDS-DMA bin_mul_kernel instance"
    for b in bodies:
        last = b.rfind("global_load_lds")
        bar = b.find("s_barrier", last)
        assert bar > 0 and re.search(r"s_waitcnt vmcnt\(0\)", b[last:bar]), "DMA strip not drained before the barrier"


def test_product_bin_kernels_carry_no_ablation():
    """k_bin.hip holds the product kernels only: the probe ablations (wrong-y
    modes) of rounds 1-3 are gone from its source (their results stay under
    profiles/)."""
    src = open(os.path.join(CSRC, "k_bin.hip")).read()
    assert "ablation" not in src.lower() and "wrong y" not in src


def test_vector_checks():
    chk = sp._check_vec
    chk(np.zeros(10), 10, "x", 0, False)
    chk(np.zeros(12), 10, "x", 0, False)  # longer is fine
    chk(None, 0, "x", 0, False)
    with pytest.raises(ValueError, match="float64"):
        chk(np.zeros(10, np.float32), 10, "x", 0, False)
    with pytest.raises(ValueError, match="needs 10"):
        chk(np.zeros(9), 10, "y", 0, True)
    with pytest.raises(ValueError, match="contiguous"):
        chk(np.zeros(20)[::2], 10, "x", 0, False)
    ro = np.zeros(10)
    ro.flags.writeable = False
    chk(ro, 10, "x", 0, False)
    with pytest.raises(ValueError, match="read-only"):
        chk(ro, 10, "y", 0, True)
    with pytest.raises(ValueError, match="numpy"):
        chk([0.0] * 10, 10, "x", 0, False)
    with pytest.raises(ValueError, match="float64"):
        chk(torch.zeros(10, dtype=torch.float32), 10, "x", 0, False)
    with pytest.raises(ValueError, match="numpy array"):
        chk(torch.zeros(10, dtype=torch.float64), 10, "x", 0, False)  # CPU tensor
    with pytest.raises(ValueError, match="contiguous"):
        chk(torch.zeros(20, dtype=torch.float64)[::2], 10, "x", 0, False)


def test_bench_self_launch(monkeypatch):
    """`bench.py --gpus N` outside torchrun starts torch.distributed.run with N
    ranks on 127.0.0.1 (one process per GPU) and returns its exit code; inside
    a matching launcher (or at N = 1) it runs in-process."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 7)
    monkeypatch.setenv("BENCH_DIST_BACKEND", "gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--rows", "1000", "--verify"])
    args = bench.parse()
    assert bench.self_launch(args) == 7
    cmd, env = calls[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=2" in cmd and "127.0.0.1" in cmd
    assert cmd[-5:] == ["--gpus", "2", "--rows", "1000", "--verify"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(args) is None  # the child: run in-process
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.self_launch(bench.parse()) is None  # N = 1
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(bench.parse()) == 2  # mismatched launcher: refuse


def test_bench_self_launch_parent_stays_off_hip(tmp_path):
    """The self-launching parent counts GPUs from the KFD topology and spawns
    the launcher without loading HIP: in a fresh interpreter, a fake launcher
    reads the parent's /proc/self/maps at the spawn -- no libamdhip64 (nor
    torch) may be mapped.  The fake topology holds one CPU node and two GPU
    nodes (simd_count > 0); HIP_VISIBLE_DEVICES caps the count."""
    topo = tmp_path / "nodes"
    for i, simds in enumerate((0, 256, 256)):
        (topo / str(i)).mkdir(parents=True)
        (topo / str(i) / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simds}\n")
    prog = (
        "import sys, json; sys.path.insert(0, %r); import bench\n"
        "seen = {}\n"
        "def fake(cmd, env=None):\n"
        "    maps = open('/proc/self/maps').read()\n"
        "    seen.update(hip='libamdhip64' in maps, torch='libtorch' in maps, cmd=cmd)\n"
        "    return 5\n"
        "sys.argv = ['bench.py', '--gpus', '2', '--rows', '1000']\n"
        "rc = bench.self_launch(bench.parse(), runner=fake)\n"
        "print(json.dumps(dict(rc=rc, n=bench.visible_gpu_count(), **seen)))\n" % ROOT)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                            "CUDA_VISIBLE_DEVICES", "BENCH_DIST_BACKEND")}
    env["BENCH_KFD_TOPOLOGY"] = str(topo)
    out = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["rc"] == 5 and res["n"] == 2 and "--nproc-per-node=2" in res["cmd"]
    assert res["hip"] is False and res["torch"] is False
    # one visible device: --gpus 2 is refused before any spawn
    env["HIP_VISIBLE_DEVICES"] = "0"
    out = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=120)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["rc"] == 2 and res["n"] == 1 and "cmd" not in res


def test_traffic_keys_name_the_shape():
    """roofline.traffic is looked up by (config, m x n, kernel): a rank shape
    without its own profile reports null instead of another shape's bytes."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    t = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic_calibrated.json")))
    assert bench.traffic_key("c2", 10_000_000, 10_000_000, "bin_mul_kernel+bin_sum_kernel") in t
    # N = 8 rank shape (AUTO: Mul-ordered products)
    assert bench.traffic_key("c2", 10_000_000, 80_000_000, "bin_mul_kernel+bin_sum_bin_kernel") in t
    assert bench.traffic_key("c2", 10_000_000, 30_000_000, "bin_mul_kernel+bin_sum_kernel") not in t  # unprofiled


def test_host_code_under_asan_ubsan():
    """the host code (loaders, generators, format builders, BIN
    layout, dist layout, C-ABI validation) built with AddressSanitizer +
    UBSan (`make asan`, host objects only) runs the BIN layout check and the
    host/oracle test files clean."""
    subprocess.check_call(["make", "-s", "-j8", "asan"], cwd=ROOT)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1")
    # 12 of the plain run's 60 random matrices (4 of each kind): the plain
    # build checks all 60 (tests/test_bin_layout.py)
    out = subprocess.run([os.path.join(ROOT, "build", "asan", "bin_layout_check"), "12"], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stderr[-3000:]
    rt = subprocess.check_output(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"], text=True).strip()
    env.update(LD_PRELOAD=rt, SPMV_HIP_LIBRARY=os.path.join(ROOT, "build", "asan", "libspmv_hip.so"))
    out = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                          os.path.join(ROOT, "tests", "test_host.py"), os.path.join(ROOT, "tests", "test_abi.py")],
                         env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "passed" in out.stdout


def test_bench_shard_check_flags_a_wrong_slice():
    """bench.shard_check: the oracle's opt_crs y of a rank's shard (its rows,
    global columns, the replicated x) -- exact y scores 0, a y off in one
    entry by 1e-9 relative scores ~1e-9, so every bench line's
    max_rel_err_vs_cpu would expose a wrong slice (no GPU needed: CPU
    tensors stand in for the device ones)."""
    import bench
    import oracle
    spec = sp.gen_spec("powerlaw", 4000, 6000, max_len=300, seed=5)
    rp, col, val = sp.generate_csr(spec, 1000, 2500)  # rows [1000, 2500) of a 4000 x 6000 matrix
    x = torch.from_numpy(sp.generate_vector(6000, seed=6))
    M = {"rp": rp, "col": col, "val": val, "x": x}
    y_check, ms = bench.shard_check(M)
    assert ms >= 0
    yo = oracle.csr_spmv(rp, col, val, x.numpy())
    assert len(yo) == 1500
    assert y_check(torch.from_numpy(yo.copy()))["max_rel_err_vs_cpu"] == 0.0
    bad = yo.copy()
    k = int(np.argmax(np.abs(bad)))
    bad[k] *= 1 + 1e-9
    err = y_check(torch.from_numpy(bad))["max_rel_err_vs_cpu"]
    assert 5e-10 < err < 2e-9
