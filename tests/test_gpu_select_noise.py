"""Measured noise margins of the one-level select (tfhe_amd.integer.g_select).

g_select returns OR(t, f) = t + f + 1/8 as a linear combination of two gate outputs, so a select output carries
twice a PBS output's noise variance.  Its consumers must bootstrap it (every gate does); the worst consumers are
MAJ of three select outputs (margin 1/8) and XOR / XOR3 of select outputs (margin 1/4 on the doubled phase) --
XOR3 of three select bits is what g_mul by a plaintext builds from rows a, a<<1, a<<2 of a select result.

Measured here on the MI355X, P-GATE FFT64: the phase error of each combination over 3 x 4096 select outputs
against its margin, then the combinations bootstrapped and decrypted.  Bar: every decision correct, the largest
error below half the margin, and margin / measured sigma >= 10 (DESIGN §7b estimates ~13 sigma)."""
import numpy as np
import pytest

from tfhe_amd import integer as I

pytestmark = pytest.mark.gpu
MU = 1 << 61  # 1/8


def _signed(x: np.ndarray) -> np.ndarray:
    return x.astype(np.uint64).view(np.int64).astype(np.float64) / 2.0**64   # torus value in [-1/2, 1/2)


def test_select_outputs_keep_downstream_margins(gate_fft_engine, gate_fft_keys):
    ck, _ = gate_fft_keys
    eng = gate_fft_engine
    B = 4096
    rng = np.random.default_rng(0x5E1)
    cond, x, y = (rng.integers(0, 2, (3, B)).astype(bool) for _ in range(3))
    c = I.Circuit(eng)
    # gate outputs (bootstrapped once) as the select's operands, like any intermediate of a circuit
    fresh = ck.encrypt_bool(np.concatenate([cond, x, y]).reshape(-1), seed=0x5E1)
    ops = eng.pbs(fresh, eng.gate_lut()).reshape(3, 3 * B, -1)   # cond | x | y, each 3 x B
    dim = ops.shape[-1]
    s = c.run(I.g_select(ops[0], ops[1][:, None], ops[2][:, None])).reshape(3, B, dim)  # 3 x B select outputs
    sbits = np.where(cond, x, y)                                   # (3, B)
    assert np.array_equal(ck.decrypt_bool(s.reshape(-1, s.shape[-1])), sbits.reshape(-1))
    v = np.where(sbits, 0.125, -0.125)
    cases = {
        # name: (combination, ideal phase, margin, decision)
        "MAJ": (I.MAJ(s[0], s[1], s[2]), v[0] + v[1] + v[2], 0.125,
                (sbits.sum(axis=0) >= 2)),
        "XOR": (I.XOR(s[0], s[1]), 2 * (v[0] + v[1]) + 0.25, 0.25, sbits[0] ^ sbits[1]),
        "XOR3": (I.XOR3(s[0], s[1], s[2]), -2 * (v[0] + v[1] + v[2]), 0.25, sbits[0] ^ sbits[1] ^ sbits[2]),
    }
    for name, (lin, ideal, margin, want) in cases.items():
        err = _signed(ck.phase(lin) - (np.round(np.asarray(ideal) * 2.0**64) % 2.0**64).astype(np.uint64))
        sd, mx = float(err.std()), float(np.abs(err).max())
        print(f"{name}: sigma 2^{np.log2(sd):.2f}, max |err| 2^{np.log2(mx):.2f}, margin / sigma {margin / sd:.1f}")
        assert mx < margin / 2, (name, mx)
        assert margin / sd >= 10, (name, sd)
        out = eng.pbs(lin, eng.gate_lut())                          # the consumer's bootstrap
        assert np.array_equal(ck.decrypt_bool(out), want), name
