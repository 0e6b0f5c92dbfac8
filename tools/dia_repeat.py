# DIA at config 4: several identical plans in one process (placement effect?)
# plus the stream probe on buffers of 2 / 10 GB.
import json, os, sys
sys.path.insert(0, os.getcwd())
import torch, singlespmv_amd as sp
m = 20_000_000
spec = sp.gen_spec("banded", m, m, band_lo=-32, band_hi=31, seed=42)
rp, col, val = sp.generate_csr(spec)
x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
y = torch.empty(m, dtype=torch.float64, device="cuda")
plans = [sp.Plan.from_csr(m, m, rp, col, val, "dia") for _ in range(int(os.environ.get("NPLANS", "3")))]
for rnd in range(2):
    for i, p in enumerate(plans):
        p.time(x, y, 3)
        print(json.dumps({"plan": i, "round": rnd, "ms": round(p.time(x, y, 20) / 20, 4)}), flush=True)
del plans
for gb in (2, 10):
    print(json.dumps({"stream_gb": gb, "gbs": round(sp.stream_probe(0, gb << 30, 5))}), flush=True)
