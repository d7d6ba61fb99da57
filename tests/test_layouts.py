"""LDS layout properties of the N = 2048 transpose areas (tfhe_amd/csrc/fft1k.h, F1_SWZ): every layout must be a
bijection of the 1024 (hi, s, l0) elements onto its area and conflict-free for each 16-lane group of the two access
patterns -- row side (lane (hi, l0) touches (hi, s, l0) at step s) and column side (lane (hi, l0) touches
(hi, l0, c) at step c).  A 16-byte element at index a sits in bank group a mod 16 (64 banks x 4 B = 16 x 16 B)."""
import pytest


def skew(hi, s, l0):            # F1_SWZ = 2 (default): 256 hi + 16 s + ((l0 + s) & 15)
    return 256 * hi + 16 * s + ((l0 + s) & 15)


def skew_row(lane, s):          # TAddr::row: one of two lane bases + an immediate
    hi, l0 = lane >> 4, lane & 15
    w1 = 256 * hi + l0
    return (w1 if s < 16 - l0 else w1 - 16) + 17 * s


def skew_col(lane, c):          # TAddr::col
    hi, l0 = lane >> 4, lane & 15
    r1 = 256 * hi + 17 * l0
    return (r1 if c < 16 - l0 else r1 - 16) + c


def xor(hi, s, l0):             # F1_SWZ = 1
    return 256 * hi + 16 * s + (l0 ^ s)


def padded(hi, s, l0):          # F1_SWZ = 0: rows of 17
    return 272 * hi + 17 * s + l0


@pytest.mark.parametrize("layout,size", [(skew, 1024), (xor, 1024), (padded, 1088)])
def test_transpose_layout_bijective_and_conflict_free(layout, size):
    idx = {layout(hi, s, l0) for hi in range(4) for s in range(16) for l0 in range(16)}
    assert len(idx) == 1024 and max(idx) < size
    for step in range(16):
        for hi in range(4):
            row = [layout(hi, step, l0) % 16 for l0 in range(16)]      # row side: step = s
            col = [layout(hi, l0, step) % 16 for l0 in range(16)]      # column side: step = c
            assert len(set(row)) == 16 and len(set(col)) == 16


def test_skew_two_base_form_equals_layout():
    for lane in range(64):
        hi, l0 = lane >> 4, lane & 15
        for k in range(16):
            assert skew_row(lane, k) == skew(hi, k, l0)
            assert skew_col(lane, k) == skew(hi, l0, k)
