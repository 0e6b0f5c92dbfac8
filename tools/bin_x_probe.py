import sys, json, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, numpy as np, singlespmv_amd as sp
m = 5_000_000
spec = sp.gen_spec("powerlaw", m, m, max_len=10000, alpha=2.0, seed=42)
rp, col, val = sp.generate_csr(spec)
xr = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
xz = torch.zeros(m, dtype=torch.float64, device="cuda")
xc = torch.full((m,), 4.8e-4, dtype=torch.float64, device="cuda")
y = torch.empty(m, dtype=torch.float64, device="cuda")
plans = {k: sp.Plan.from_csr(m, m, rp, col, val, "bin", placement="search", **o) for k, o in
         (("long", {}), ("exact", {"bin_long_len": -1}))}
for r in range(3):
    for k, p in plans.items():
        for xn, x in (("real", xr), ("zero", xz), ("const", xc)):
            ph = p.profile(x, y, 20)
            print(json.dumps({"r": r, "plan": k, "x": xn, **{a: round(b, 4) for a, b in ph.items()},
                              "search": [round(p.info()["placement_best_ms"], 4), round(p.info()["placement_worst_ms"], 4)]}), flush=True)
