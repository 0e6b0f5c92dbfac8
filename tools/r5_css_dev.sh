#!/bin/bash
# the CSS device builder: its GPU tests, then config-2 CSS plan build times
# (device vs host builders) and y equality.
#   bash tools/r5_css_dev.sh <tag>
set -o pipefail
T=$1; R=gpurun_out/$T; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -k "routing or device_conversion or css or golden" --timeout 600 --timeout-method thread > $R/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u - > $R/css_c2_build.json 2> $R/css_c2_build.err <<'PY' || exit 2
import json, time, torch, numpy as np, singlespmv_amd as sp
m = 10_000_000
rp, col, val = sp.generate_csr(sp.gen_spec("uniform", m, per_row=16, seed=42))
x = torch.from_numpy(sp.generate_vector(m, seed=43)).cuda()
out = {}
ys = {}
for b in ("host", "device"):
    t = time.perf_counter()
    p = sp.Plan.from_csr(m, m, rp, col, val, "css", build=b)
    out[b + "_build_s"] = round(time.perf_counter() - t, 3)
    out[b + "_on_device"] = p.built_on_device()
    y = torch.empty(m, dtype=torch.float64, device="cuda")
    p.execute(x, y)
    ys[b] = y.cpu().numpy()
    out[b + "_digest"] = p.digest()
    out[b + "_ms"] = round(p.time(x, y, 20) / 20, 4)
    p.destroy()
out["digest_equal"] = out.pop("host_digest") == out.pop("device_digest")
out["y_equal"] = bool(np.array_equal(ys["host"], ys["device"]))
print(json.dumps(out))
PY
echo done
