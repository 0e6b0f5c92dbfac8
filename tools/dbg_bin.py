# Reproduce test_bin_layout_knobs in one process: every knob, several plans,
# repeated executes; report executes whose y differs from the oracle.
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import singlespmv_amd as sp, oracle
m = 120_000
spec = sp.gen_spec("powerlaw", m, m, per_row=11, max_len=5000, seed=41)
rp, col, val = sp.generate_csr(spec)
x = sp.generate_vector(m, seed=43)
yo = oracle.csr_spmv(rp, col, val, x)
knobs = [{"SPMV_BIN_PADLOG": "3"}, {"SPMV_BIN_PADLOG": "5"}, {"SPMV_BIN_SUMWAVES": "2"},
         {"SPMV_BIN_SUMWAVES": "8"}, {"SPMV_BIN_REUSE": "1"}, {"SPMV_BIN_DEBUG": "1"}, {}]
for rnd in range(3):
    for env in knobs:
        for k in ("SPMV_BIN_PADLOG", "SPMV_BIN_SUMWAVES", "SPMV_BIN_REUSE", "SPMV_BIN_DEBUG"):
            os.environ.pop(k, None)
        os.environ.update(env)
        p = sp.Plan.from_csr(m, m, rp, col, val, "bin", bin_groups=2)
        out = []
        for rep in range(20):
            y = np.full(m, 1.2345e300 * (-1) ** rep)
            p.execute(x, y)
            bad = np.flatnonzero(y != yo)
            if len(bad):
                out.append((rep, len(bad), bad[:4].tolist(), (y[bad[:2]] - yo[bad[:2]]).tolist()))
        print(rnd, env, "bad executes:", out[:5], flush=True)
        p.destroy()
