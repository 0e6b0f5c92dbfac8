# correctness of a BIN plan variant (SPMV_BIN_DEBUG from the environment) over
# several plans and executes: prints executes whose y differs from the oracle
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import singlespmv_amd as sp, oracle
m = 300_000
spec = sp.gen_spec("powerlaw", m, m, per_row=11, max_len=5000, seed=41)
rp, col, val = sp.generate_csr(spec)
x = sp.generate_vector(m, seed=43)
yo = oracle.csr_spmv(rp, col, val, x)
bad = 0
for rnd in range(4):
    p = sp.Plan.from_csr(m, m, rp, col, val, "bin")
    for rep in range(10):
        y = np.full(m, 1.2345e300 * (-1) ** rep)
        p.execute(x, y)
        bad += int((y != yo).sum())
    p.destroy()
print("bad entries", bad, flush=True)
