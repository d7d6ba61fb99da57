#!/bin/bash
# FFT64 P-GATE: PBS time per batch for the latency kernel vs the batch kernel (crossover for lat_max).
cd "${GRAFT_REPO_ROOT:-.}"
python - <<'PY'
import time, numpy as np, tfhe_amd
ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT), 0x7F4E0001)
eng = tfhe_amd.Engine(ck.params, 0); eng.load_keys(sk)
lut = eng.gate_lut()
for B in (1, 8, 64, 256, 512, 768, 1024, 1536, 2048):
    cts = ck.encrypt_bool(np.ones(B, dtype=bool), seed=7)
    res = {}
    for name, lm in (("lat", 1 << 20), ("batch", 0)):
        eng.set_latency_batch(lm)
        eng.pbs(cts, lut)
        t = time.time(); reps = 3
        for _ in range(reps): out = eng.pbs(cts, lut)
        res[name] = (time.time() - t) / reps * 1e3
        assert ck.decrypt_bool(out).all()
    print(f"B={B:5d} lat {res['lat']:8.2f} ms  batch {res['batch']:8.2f} ms", flush=True)
PY
