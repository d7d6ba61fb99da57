"""The FFT64 external product's rounding error against EXACT arithmetic: the derived worst-case bound and the
variance model that tests/test_exact.py (oracle) and tests/test_gpu_exact.py (device) check.  Derivation in
DESIGN.md §5b; the arbiter is oracle/exact_oracle.c (no floating point).

Notation for one CMUX and one output column j:  R = (k+1) L digit polynomials d_r (signed SignedDecomposer digits),
key polynomials w_{r,j} read as signed int64 (the operand the FFT transforms), M = N/2 complex points,
    S1 = sum_r ||d_r||_2 ||w_{r,j}||_2,      rho^2 = sum_r ||d_r||_2^2 ||w_{r,j}||_2^2 / N
(rho = the rms size of the exact integer product's coefficients for random-phase operands).  u = 2^-53.

Worst case (rigorous, Higham-style stage analysis): every transform is s = 15 stages, each either a radix-2
butterfly level (a scaled unitary matrix, one rounding per component: relative error <= u) or a diagonal of
computed twiddles (|w^ - w| <= mu, complex fma product: relative error <= mu + 2 sqrt(2) u (1 + mu)), so
    alpha = (1 + eta)^s - 1,  eta = mu + 2 sqrt(2) u (1 + mu)          (forward and inverse transforms)
    beta  = alpha (2 + alpha) + sqrt(2) gamma_{2R+1} (1 + alpha)^2      (spectrum products + fma MAC chain)
    |FFT64 - exact| <= sqrt(M) S1 (beta + alpha (1 + beta)) + 1/2       (inverse, then rint)
using ||D||_inf <= sqrt(M) ||d||_2, ||K||_inf <= ||w||_2 / sqrt(M), ||.||_inf <= ||.||_2.

Variance model (independent roundings, relative variance u^2/3 per rounding): per-stage weights c (butterfly level 1,
twiddle product 1.5 + 3 m^2 with m = the twiddle tables' rms error / u, fractions of entries that are exact
multiplies dropped), summed over the digit transform, the key transform, the MAC chain and the inverse:
    sigma = sqrt(kappa / 3) u rho.
"""
import math

import numpy as np

U = 2.0 ** -53
STAGES = 15          # fft512: twist + 3 x (dft8: 3 levels + 1 rotation stage) + 2 tables; fft1k: twist + 2 dft16 (5)
                     # + ta + radix-4 (2) + tb; the inverses mirror them (fft_oracle.c)
MU_BOUND = 4 * U     # twiddle-table error bound used in the bound (measured max 3.2 u: test_twiddle_accuracy)


def gamma(n: int) -> float:
    return n * U / (1 - n * U)


def worst_case_bound(N: int, R: int, s1, mu: float = MU_BOUND):
    """max |FFT64 result - exact result| per output coefficient, for norm sums s1 (array-like)."""
    M = N // 2
    eta = mu + 2 * math.sqrt(2) * U * (1 + mu)
    alpha = (1 + eta) ** STAGES - 1
    beta = alpha * (2 + alpha) + math.sqrt(2) * gamma(2 * R + 1) * (1 + alpha) ** 2
    return math.sqrt(M) * np.asarray(s1, dtype=np.float64) * (beta + alpha * (1 + beta)) + 0.5


def twiddle_rms(oracle_mod, Ms=(512, 2048, 4096)) -> float:
    """rms |w^ - w| / u of the oracle's (= the device's) twiddle tables, against long double cos / sin."""
    two_pi = np.longdouble("6.283185307179586476925286766559")
    acc, cnt = 0.0, 0
    for M in Ms:
        t = np.arange(M)
        x = two_pi * t.astype(np.longdouble) / np.longdouble(M)
        got = np.array([oracle_mod.fft_twiddle(int(i), M) for i in t], dtype=np.float64).astype(np.longdouble)
        acc += float((((got[:, 0] - np.cos(x)) ** 2 + (got[:, 1] - np.sin(x)) ** 2)).sum())
        cnt += M
    return math.sqrt(acc / cnt) / U


def kappa(N: int, R: int, m: float) -> float:
    c_tw = 1.5 + 3 * m * m
    if N == 1024:   # fft512: 3 x dft8 (3 levels + w8 on 2 of 8 outputs, weight 2) + slot twist 7/8 + tables 1, 7/8
        k_t = 3 * 3.5 + (7 / 8 + 1 + 7 / 8) * c_tw
        k_mac = 4.5  # two 3-term chains (6 fma per component each) then one add
    elif N == 2048:  # fft1k: 2 x dft16 (4 levels + 8/16 twiddled, 0.84) + radix-4 (2) + twist 15/16, ta 1, tb 0.7
        k_t = 2 * 4.84 + 2 + (15 / 16 + 1 + 0.7) * c_tw
        k_mac = 2.5  # one 2-term chain (4 fma per component)
    else:
        raise ValueError(N)
    return 3 * k_t + k_mac


def sigma_model(N: int, R: int, s2, m: float):
    """model rms of |FFT64 - exact| per coefficient (s2 = sum_r ||d_r||^2 ||w_r||^2)."""
    rho = np.sqrt(np.asarray(s2, dtype=np.float64) / N)
    return math.sqrt(kappa(N, R, m) / 3) * U * rho


def signed(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, dtype=np.uint64).view(np.int64).astype(np.float64)


def negacyclic_mul_key(a: np.ndarray, s: np.ndarray) -> np.ndarray:
    """a (*) s mod X^N + 1 for float a and binary s (phase of an error term), exact enough for statistics."""
    N = a.shape[-1]
    out = np.zeros_like(a)
    for j in np.nonzero(s)[0]:
        out += np.concatenate([-a[..., N - j:], a[..., :N - j]], axis=-1) if j else a
    return out


def check_steps(oracle_mod, prm, got_next, exact_next, s1, s2, m=None):
    """Compare device/oracle states after a CMUX with the exact CMUX of the same input.  Returns a stats dict;
    asserts max <= worst-case bound and 0.5 <= rms / model <= 2."""
    N, R = prm.N, (prm.k + 1) * prm.pbs_level
    if m is None:
        m = twiddle_rms(oracle_mod)
    d = signed(np.asarray(got_next, dtype=np.uint64) - np.asarray(exact_next, dtype=np.uint64))
    d = d.reshape(-1, prm.k + 1, N)
    bound = worst_case_bound(N, R, s1)                     # [steps][k+1]
    err = np.abs(d).max(axis=2)
    sig = sigma_model(N, R, s2, m)
    live = s1 > 0                                          # a skipped CMUX (a~ = 0) is exactly zero on both sides
    assert np.all(err[~live] == 0), "a zero-rotation CMUX must be exact"
    assert np.all(err <= bound), f"FFT error above the derived bound: {np.max(err / bound):.3g} x"
    ms = (d[live] ** 2).mean(axis=1)                       # per (step, column) mean square
    rms_ratio = math.sqrt(float((ms / sig[live] ** 2).mean()))
    assert 0.5 <= rms_ratio <= 2.0, f"rms error {rms_ratio:.2f} x the variance model"
    return dict(max_err_log2=math.log2(max(float(err.max()), 1.0)),
                bound_log2=math.log2(float(bound[live].min())),
                max_over_bound_log2=math.log2(max(float((err[live] / bound[live]).max()), 2.0 ** -60)),
                rms_over_model=rms_ratio,
                max_over_model_sigma=float((err[live] / sig[live]).max()), steps=int(live.sum()))
