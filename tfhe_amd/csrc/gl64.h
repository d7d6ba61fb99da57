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

// a * b + z as a 128-bit (hi, lo) pair — never overflows: 4 chained v_mad_u64_u32 (32x32 + 64),
// every partial sum bounded below 2^64 (the 64-bit addend rides in the first two).
__host__ __device__ __forceinline__ void gl_mac128(u64 a, u64 b, u64 z, u64& hi, u64& lo) {
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
  const u64 t = (u64)a0 * b0 + (u32)z;                   // <= 2^64 - 2^32
  const u64 u = (u64)a1 * b0 + ((t >> 32) + (z >> 32));  // <= 2^64 - 1
  const u64 v = (u64)a0 * b1 + (u32)u;                   // <  2^64
  hi = (u64)a1 * b1 + ((u >> 32) + (v >> 32));           // <= 2^64 - 1
  lo = (v << 32) | (u32)t;
}

// Reductions of hi * 2^64 + lo (hi = hh * 2^32 + hl):  == lo - hh + hl * (2^32 - 1)  (mod p).
// t = lo - hh (+p on borrow: t >= 2^64 - 2^32 + 1 there, so t - EPS does not wrap); then
// r = hl * EPS + t in one mad.  On carry the true value is r + EPS and r <= 2^64 - 2^33, so
// r + EPS < p; without carry r may still be >= p.  Exact for every (hi, lo).
__host__ __device__ __forceinline__ u64 gl_reduce128_lazy(u64 hi, u64 lo) {  // any 64-bit word
  const u64 hh = hi >> 32, hl = hi & GL_EPS;
  u64 t = lo - hh;
  t = (lo < hh) ? t + GL_P : t;
  const u64 r = hl * GL_EPS + t;
  return (r < t) ? r + GL_EPS : r;
}
__host__ __device__ __forceinline__ u64 gl_reduce128(u64 hi, u64 lo) {  // canonical
  const u64 hh = hi >> 32, hl = hi & GL_EPS;
  u64 t = lo - hh;
  t = (lo < hh) ? t + GL_P : t;
  const u64 r = hl * GL_EPS + t;
  return (r < t || r >= GL_P) ? r + GL_EPS : r;  // carry: r + EPS < p;  r >= p: r + EPS == r - p
}

// (hi * 2^64 + lo) mod p for hi < 2^32: r = hi * EPS + lo (one mad), same carry argument.
__host__ __device__ __forceinline__ u64 gl_reduce96_lazy(u64 hi, u64 lo) {
  const u64 r = hi * GL_EPS + lo;
  return (r < lo) ? r + GL_EPS : r;
}
__host__ __device__ __forceinline__ u64 gl_reduce96(u64 hi, u64 lo) {
  const u64 r = hi * GL_EPS + lo;
  return (r < lo || r >= GL_P) ? r + GL_EPS : r;
}

__host__ __device__ __forceinline__ u64 gl_canon(u64 x) { return (x >= GL_P) ? x + GL_EPS : x; }

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

__host__ __device__ __forceinline__ u64 gl_mul(u64 a, u64 b) {
  u64 hi, lo;
  gl_mac128(a, b, 0, hi, lo);
  return gl_reduce128(hi, lo);
}

// z + a * b mod p, lazily reduced (any 64-bit word in, any 64-bit word out): the MAC of the
// external product accumulates with this and canonicalizes once per output (gl_canon).
__host__ __device__ __forceinline__ u64 gl_mac_lazy(u64 z, u64 a, u64 b) {
  u64 hi, lo;
  gl_mac128(a, b, z, hi, lo);
  return gl_reduce128_lazy(hi, lo);
}

// x * 2^r mod p for 0 <= r < 96 (r a compile-time constant after unrolling: the branches fold
// away).  Canonical output for r > 0 and any 64-bit x; r = 0 returns x.  Steps of at most 32 bits
// keep the high part below 2^32, so each step is one mad + a carry fix (gl_reduce96).
__host__ __device__ __forceinline__ u64 gl_shl_mod(u64 x, int r) {
  if (r == 0) return x;
  while (r > 32) {
    x = gl_reduce96_lazy(x >> 32, x << 32);
    r -= 32;
  }
  return gl_reduce96(x >> (64 - r), x << r);
}

// x * 2^-t mod p for 1 <= t <= 32, any 64-bit x, canonical output.  With x = xh 2^t + xl and
// 2^-t = -2^(96-t):  x 2^-t == xh - xl 2^(32-t) 2^64 == xh + y - y 2^32,  y = xl 2^(32-t) < 2^32.
// s = xh + y < 2^63 + 2^32 (no wrap); s - y 2^32 >= -(p - 1), so one conditional +p lands in [1, p).
__host__ __device__ __forceinline__ u64 gl_shr_mod(u64 x, int t) {
  const u64 xh = x >> t;
  const u32 y = (u32)x << (32 - t);
  const u64 s = xh + y;
  const u64 yy = (u64)y << 32;
  const u64 d = s - yy;
  return (s < yy) ? d + GL_P : d;
}

// 2^z * x == (neg ? -v : v) for a compile-time z: the cheapest of shl by r = z mod 96 (r <= 64)
// or shr by 96 - r (r > 64, one fold instead of three), with the sign of 2^96 = -1 reported back
// so callers fold it into an add/sub.  v is canonical unless r == 0 (then v = x).
__host__ __device__ __forceinline__ u64 gl_pow2_twiddle(u64 x, int z, bool& neg) {
  z %= 192;
  if (z < 0) z += 192;
  const bool s = z >= 96;
  const int r = z % 96;
  if (r > 64) {
    neg = !s;
    return gl_shr_mod(x, 96 - r);
  }
  neg = s;
  return gl_shl_mod(x, r);
}

// x * 2^s mod p for any integer s (2^192 == 1, 2^96 == -1); canonical for canonical x.
__host__ __device__ __forceinline__ u64 gl_mul_pow2(u64 x, int s) {
  s %= 192;
  if (s < 0) s += 192;
  if (s >= 96) return gl_neg(gl_shl_mod(x, s - 96));
  return gl_shl_mod(x, s);
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
