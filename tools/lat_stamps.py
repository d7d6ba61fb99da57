"""Phase times of the P-GATE latency kernel (diagnostic build only: make -C tfhe_amd B=../build_diag/ls/obj
LIB=../build_diag/ls/libtfhe_hip.so EXTRA=-DFFT_LATSTAMP=1; run with TFHE_HIP_LIB=build_diag/ls/libtfhe_hip.so).
Per wave of workgroup 0, the mean over the 630 CMUXes of the time from the CMUX start to: its phase-A work done,
barrier 1 passed, phase-B work done, barrier 2 passed, phase-C work done, barrier 3 passed (us).
  python tools/lat_stamps.py [--batch 64]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    eng = tfhe_amd.Engine(params, 0).load_keys(sk)
    cts = ck.encrypt_bool(np.random.default_rng(1).integers(0, 2, a.batch).astype(bool), seed=0xC0FFEE01)
    for _ in range(3):
        eng.pbs(cts, eng.gate_lut())
    buf = np.zeros(8 * 8 * 6, dtype=np.uint64)
    f = tfhe_amd.lib().tfhe_hip_debug_latstamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert f(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(8, 8, 6).astype(np.float64) / 100.0 / params.n   # us per CMUX
    res = {"batch": a.batch, "marks": ["A done", "bar1", "B done", "bar2", "C done", "bar3"],
           "wg0_per_wave_us": [[round(x, 3) for x in row] for row in t[0]],
           "mean_over_wg0_7_wave0_us": [round(x, 3) for x in t[:, 0].mean(axis=0)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
