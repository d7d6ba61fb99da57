"""Phase shares of the P-FHEVM FFT64 batch kernel from a diagnostic build:
    tools/ab_build.sh stamps -DF2_STAMPS=1
    TFHE_HIP_LIB=build_ab/stamps/libtfhe_hip.so python tools/stamps.py
(The P-GATE stamps of round 2 instrumented the retired 8-ciphertext kernel; they left with it.)
Runs one 4096-PBS launch and prints, per phase of the CMUX loop, the mean cycles per CMUX over the
sampled waves (every 64th workgroup) and the share of the loop.  Read the shares, not the total (the
stamps' waits forbid overlaps the shipped kernel has)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402

PHASES = ["top barrier", "rotate+decomp A", "fwd A", "rotate+decomp B", "vmcnt col0", "fwd B",
          "MAC0 (+col1 issue)", "vmcnt+barrier col1", "MAC1 + barrier", "inverse 0 + acc", "barrier", "inverse 1 + acc"]


def main():
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT)
    ck, sk = tfhe_amd.gen_keys(p, 0x7F4E0001)
    B = 4096
    msgs = np.random.default_rng(1).integers(0, 16, B).astype(np.uint64)
    cts = ck.encrypt(msgs, 16, seed=3)
    with tfhe_amd.Engine(p, 0) as eng:
        eng.load_keys(sk)
        lut = eng.generate_accumulator(lambda m: m, 16)
        out = eng.pbs(cts, lut)
        assert np.array_equal(ck.decrypt(out, 16), msgs)
        buf = np.zeros(16 * 8 * 12 + 16 * 8, dtype=np.uint64)
        L = tfhe_amd.lib()
        rc = L.tfhe_hip_debug_fft2k_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        assert rc == 0, rc
    pw = buf[16 * 8 * 12:].reshape(16, 8)
    buf = buf[:16 * 8 * 12].reshape(16, 8, 12)
    tot = buf.astype(np.float64).sum(axis=(0, 1))
    waves = np.count_nonzero(buf.sum(axis=2))
    per = tot / max(waves, 1) / p.n
    for k, name in enumerate(PHASES):
        print(f"{name:24s} {per[k]:10.0f} cycles/CMUX  {100 * tot[k] / tot.sum():5.1f} %")
    print(f"total {per.sum():.0f} cycles per CMUX per wave ({waves} waves sampled)")
    pwt = pw.astype(np.float64).sum() / max(waves, 1) / p.n
    print(f"of which in the 6 pair-exchange barriers: {pwt:.0f} cycles/CMUX ({100 * pwt / per.sum():.1f} %)")


if __name__ == "__main__":
    main()
