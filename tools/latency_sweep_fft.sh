#!/bin/bash
# FFT64: PBS time per batch for the latency kernel vs the batch kernel (crossover for lat_max).
#   PRESET=gate (default) | fhevm, BATCHES=1,64,256 (default: the full grid), TFHE_HIP_LIB=<variant .so>
cd "${GRAFT_REPO_ROOT:-.}"
PRESET=${PRESET:-gate} python - <<'PY'
import os, time, numpy as np, tfhe_amd
fhevm = os.environ["PRESET"] == "fhevm"
ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT if fhevm else tfhe_amd.PRESET_GATE_FFT),
                           0x7F4E0001)
eng = tfhe_amd.Engine(ck.params, 0); eng.load_keys(sk)
lut = eng.generate_accumulator(lambda m: m, 16) if fhevm else eng.gate_lut()
Bs = os.environ.get("BATCHES")
for B in (tuple(int(x) for x in Bs.split(",")) if Bs else
          (1, 8, 64, 128, 256, 384, 512, 640, 768, 1024) if fhevm else
          (1, 8, 64, 128, 192, 256, 320, 384, 512, 768, 1024, 1536, 2048)):
    cts = ck.encrypt(np.arange(B) % 16, 16, seed=7) if fhevm else ck.encrypt_bool(np.ones(B, dtype=bool), seed=7)
    res = {}
    for name, lm in (("lat", 1 << 20), ("batch", 0)):
        eng.set_latency_batch(lm)
        eng.pbs(cts, lut)
        t = time.time(); reps = 3
        for _ in range(reps): out = eng.pbs(cts, lut)
        res[name] = (time.time() - t) / reps * 1e3
        assert (np.array_equal(ck.decrypt(out, 16), np.arange(B) % 16) if fhevm else ck.decrypt_bool(out).all())
    print(f"B={B:5d} lat {res['lat']:8.2f} ms  batch {res['batch']:8.2f} ms", flush=True)
PY
