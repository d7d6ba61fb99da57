// gl64.h — arithmetic in Z_p, p = 2^64 - 2^32 + 1 ("Goldilocks"), for gfx950 and the host.
//
// Why this prime: the blind-rotate external product needs an exact negacyclic product of a
// digit polynomial and a BSK polynomial (ml/extensions/rust/src/computations.rs:50-54 is the
// reference's exact wrapping product); an NTT over this prime gives it with integer arithmetic,
// so GPU == CPU oracle bit-for-bit.  2^64 == 2^32 - 1 and 2^96 == -1 (mod p), so reductions are
// shifts/adds, and every 64th / 32nd root of unity is a power of two (2^3, 2^6): the 32-point
// sub-transforms of the NTT need no multiplies at all (see ntt16.h).
//
// All functions return canonical values in [0, p) given canonical inputs (gl_reduce128 and
// gl_mul accept any 64-bit words).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfhe {

typedef uint64_t u64;  // == the C ABI's uint64_t (unsigned long on LP64)
typedef uint32_t u32;

constexpr u64 GL_P = 0xFFFFFFFF00000001ull;
constexpr u64 GL_EPS = 0xFFFFFFFFull;  // 2^64 mod p

__host__ __device__ __forceinline__ u64 gl_mulhi(u64 a, u64 b) {
  return (u64)(((unsigned __int128)a * b) >> 64);
}

// (hi * 2^64 + lo) mod p, canonical.  hi = hh * 2^32 + hl:  == lo - hh + hl * (2^32 - 1).
__host__ __device__ __forceinline__ u64 gl_reduce128(u64 hi, u64 lo) {
  const u64 hh = hi >> 32, hl = hi & GL_EPS;
  u64 t0 = lo - hh;
  t0 = (lo < hh) ? t0 - GL_EPS : t0;
  const u64 t1 = (hl << 32) - hl;
  u64 t2 = t0 + t1;
  t2 = (t2 < t1) ? t2 + GL_EPS : t2;
  return (t2 >= GL_P) ? t2 - GL_P : t2;
}

// (hi * 2^64 + lo) mod p for hi < 2^32.
__host__ __device__ __forceinline__ u64 gl_reduce96(u64 hi, u64 lo) {
  const u64 t1 = (hi << 32) - hi;
  u64 t2 = lo + t1;
  t2 = (t2 < t1) ? t2 + GL_EPS : t2;
  return (t2 >= GL_P) ? t2 - GL_P : t2;
}

__host__ __device__ __forceinline__ u64 gl_add(u64 a, u64 b) {
  const u64 s = a + b;
  const u64 t = s + GL_EPS;  // s - p mod 2^64
  return (s < a || s >= GL_P) ? t : s;
}

__host__ __device__ __forceinline__ u64 gl_sub(u64 a, u64 b) {
  const u64 d = a - b;
  return (a < b) ? d + GL_P : d;
}

__host__ __device__ __forceinline__ u64 gl_neg(u64 a) { return a ? GL_P - a : 0; }

__host__ __device__ __forceinline__ u64 gl_mul(u64 a, u64 b) { return gl_reduce128(gl_mulhi(a, b), a * b); }

// x * 2^s mod p.  s is a compile-time constant after unrolling (every call site below is in a
// fully unrolled loop), so the branches fold away.  2^192 == 1, 2^96 == -1.
__host__ __device__ __forceinline__ u64 gl_mul_pow2(u64 x, int s) {
  s %= 192;
  if (s < 0) s += 192;
  const bool neg = s >= 96;
  const int r = neg ? s - 96 : s;
  u64 v;
  if (r == 0) {
    v = x;
  } else if (r <= 32) {
    v = gl_reduce96(x >> (64 - r), x << r);
  } else if (r < 64) {
    v = gl_reduce128(x >> (64 - r), x << r);
  } else {  // 64 <= r < 96: two steps
    const u64 y = gl_reduce96(x >> 32, x << 32);
    const int r2 = r - 32;
    v = gl_reduce128(y >> (64 - r2), y << r2);
  }
  return neg ? gl_neg(v) : v;
}

// small signed digit -> Z_p
__host__ __device__ __forceinline__ u64 gl_from_i32(int d) { return d >= 0 ? (u64)d : GL_P - (u64)(-d); }

// Z_p -> torus 2^64 after sample extraction: round(x * 2^64 / p) == x + round(x / 2^32).
__host__ __device__ __forceinline__ u64 gl_to_torus(u64 x) { return x + ((x + 0x80000000ull) >> 32); }

// torus 2^64 -> Z_p embedding for LUT values: v - round(v / 2^32).
__host__ __device__ __forceinline__ u64 torus_to_gl(u64 v) { return v - ((v >> 32) + ((v >> 31) & 1)); }

__host__ __device__ __forceinline__ u64 gl_pow(u64 a, u64 e) {
  u64 r = 1;
  while (e) {
    if (e & 1) r = gl_mul(r, a);
    a = gl_mul(a, a);
    e >>= 1;
  }
  return r;
}

}  // namespace tfhe
