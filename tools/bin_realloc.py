# Does the Mul time follow the product buffer's placement?  One plan, the
# product buffer re-allocated between timings.
import ctypes as C, json, os, sys
sys.path.insert(0, os.getcwd())
import torch, singlespmv_amd as sp
m = 10_000_000
spec = sp.gen_spec("uniform", m, m, per_row=16, seed=42)
rp, col, val = sp.generate_csr(spec)
x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
y = torch.empty(m, dtype=torch.float64, device="cuda")
L = sp.lib()
for rep in range(2):
    p = sp.Plan.from_csr(m, m, rp, col, val, "bin")
    for k in range(8):
        p.time(x, y, 3)
        ph = p.profile(x, y, 10)
        print(json.dumps({"plan": rep, "prod_alloc": k, **{a: round(b, 4) for a, b in ph.items()}}), flush=True)
        L.spmv_bin_realloc_prod(p._h)
    p.destroy()
