"""Rounding semantics of v_mfma_f64_16x16x4_f64 from tools/microbench/mfma_f64.hip's dump.

For every D element, D[m][n] = C[m][n] + sum_k A[m][k] B[k][n] (k < 4) is compared against
candidate evaluation orders, computed exactly with Fractions and rounded where each candidate rounds:
  fma_chain_0123   c = fma(a_k, b_k, c) for k = 0, 1, 2, 3 (one rounding per step)
  fma_chain_3210   the same, k descending
  exact_once       the exact sum rounded once
  pairwise         (c + (p0 + p1)) + (p2 + p3) with exact products, each sum rounded
Prints the match count per candidate."""
import struct
import sys
from fractions import Fraction

import numpy as np


def rnd(x: Fraction) -> float:
    """Round a Fraction to the nearest double (ties to even) via Python's correctly rounded division."""
    return x.numerator / x.denominator if x != 0 else 0.0


def main(path):
    raw = open(path, "rb").read()
    reps, lanes = struct.unpack_from("ii", raw, 0)
    n = reps * lanes
    off = 8
    A = np.frombuffer(raw, np.float64, n, off); off += 8 * n
    B = np.frombuffer(raw, np.float64, n, off); off += 8 * n
    C = np.frombuffer(raw, np.float64, 4 * n, off).reshape(reps, lanes, 4); off += 32 * n
    D = np.frombuffer(raw, np.float64, 4 * n, off).reshape(reps, lanes, 4)
    A = A.reshape(reps, lanes)
    B = B.reshape(reps, lanes)
    names = ["fma_chain_0123", "fma_chain_3210", "exact_once", "pairwise"]
    hits = dict.fromkeys(names, 0)
    total = 0
    for t in range(reps):
        Am = [[Fraction(A[t, m + 16 * k]) for k in range(4)] for m in range(16)]
        Bm = [[Fraction(B[t, n + 16 * k]) for n in range(16)] for k in range(4)]
        for lane in range(lanes):
            for r in range(4):
                m, nn = (lane >> 4) + 4 * r, lane & 15
                c = Fraction(C[t, lane, r])
                p = [Am[m][k] * Bm[k][nn] for k in range(4)]
                got = D[t, lane, r]
                acc = c
                for k in range(4):
                    acc = Fraction(rnd(acc + p[k]))
                cand = {"fma_chain_0123": float(acc)}
                acc = c
                for k in (3, 2, 1, 0):
                    acc = Fraction(rnd(acc + p[k]))
                cand["fma_chain_3210"] = float(acc)
                cand["exact_once"] = rnd(c + sum(p))
                s01 = Fraction(rnd(p[0] + p[1]))
                s23 = Fraction(rnd(p[2] + p[3]))
                cand["pairwise"] = rnd(Fraction(rnd(c + s01)) + s23)
                for k in names:
                    hits[k] += cand[k] == got
                total += 1
    for k in names:
        print(f"{k:16s} {hits[k]:6d} / {total}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mfma_f64_probe.bin")
