// fft512.hpp — one-wavefront 512-point complex FFT for the N = 1024 negacyclic product.
//
// One wave64 owns one polynomial: lane t holds 8 complex points (16 f64 registers).
// 512 = 8 x 8 x 8: three in-register radix-8 passes, two intra-wave LDS transposes.
// Forward (DIF, natural in -> digit-permuted out):
//   in : lane t holds x[t + 64 m], m = 0..7 (untwisted: the negacyclic twist is folded in)
//   out: lane (k0 = t>>3, k1 = t&7) holds Z[k0 + 8 k1 + 64 k2], k2 = 0..7, where
//        Z = DFT_512(x_j * zeta^j), zeta = exp(i pi / 1024), DFT sign exp(-2 pi i jk / 512)
// Inverse (the transposed DIT, conjugate twiddles, unnormalised) maps that layout back and
// applies conj(zeta^j), so inverse(forward(x)) = 512 x.
// The pointwise product never needs natural frequency order, so no reordering pass exists.
//
// Twist folding: zeta^{t + 64 m} = zeta^t * psi^m with psi = zeta^64 = exp(i pi / 16).  psi^m
// (8 constants) multiplies the pass-1 inputs; zeta^t is merged into the pass-1 output twiddle,
// giving one per-lane table T1[k0][t] = zeta^t * w512^{t k0} used by both directions.
//
// LDS transpose slot (complex index within the wave's 575-slot / 9.2 KB scratch):
//   S(a, b, c) = 72 a + 9 b + c
// Affine in every index, so each of the three access patterns is one per-lane base VGPR plus
// ds_read/ds_write immediate offsets (an XOR swizzle is conflict-free but costs 24 live address
// VGPRs).  Found by exhaustive search over padded strides against the gfx950 ds_read_b128 /
// ds_write_b128 lane groups (MI355X_MICROARCH.md §LDS): all writes conflict-free, reads at most
// 2-way on one of the three patterns.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chip {

struct __attribute__((aligned(16))) cplx {
  double re, im;
};

__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx cmul(cplx a, cplx w) {
  return {__builtin_fma(a.re, w.re, -a.im * w.im), __builtin_fma(a.re, w.im, a.im * w.re)};
}
// a * conj(w)
__device__ __forceinline__ cplx cmulc(cplx a, cplx w) {
  return {__builtin_fma(a.re, w.re, a.im * w.im), __builtin_fma(a.im, w.re, -a.re * w.im)};
}
// a * (-i) (forward) or a * (+i) (inverse)
template <bool INV>
__device__ __forceinline__ cplx mul_mi(cplx a) {
  if constexpr (INV) return {-a.im, a.re};
  else return {a.im, -a.re};
}
// a * w8^1 with w8 = exp(-+ i pi/4)
template <bool INV>
__device__ __forceinline__ cplx mul_w8(cplx a) {
  constexpr double r = 0.70710678118654752440084436210485;
  if constexpr (INV) return {(a.re - a.im) * r, (a.re + a.im) * r};
  else return {(a.re + a.im) * r, (a.im - a.re) * r};
}
// a * w8^3
template <bool INV>
__device__ __forceinline__ cplx mul_w83(cplx a) {
  constexpr double r = 0.70710678118654752440084436210485;
  if constexpr (INV) return {(-a.re - a.im) * r, (a.re - a.im) * r};
  else return {(a.im - a.re) * r, (-a.re - a.im) * r};
}

// Negate a complex value when `sign` is 1ull << 63 (sign-bit XOR on both parts, no branch).
__device__ __forceinline__ cplx cneg_if(cplx a, uint64_t sign) {
  return {__longlong_as_double((long long)((uint64_t)__double_as_longlong(a.re) ^ sign)),
          __longlong_as_double((long long)((uint64_t)__double_as_longlong(a.im) ^ sign))};
}

// In-register 8-point DFT, natural order in and out: X[k] = sum_m x[m] w8^{+-mk}.
// Uniform relabelings used by the wave of a pair that owns the upper frequency half
// (sign = 1ull << 63, else 0):
//   OUT_XOR4: outputs permuted k -> k ^ 4 (negate b1, b3, b5, b7 before the last stage);
//   IN_XOR4:  inputs given in order m ^ 4 (the DFT of the permuted input is (-1)^k X[k]:
//             negate b4..b7, the terms of the odd outputs).
template <bool INV, int RELABEL = 0>
__device__ __forceinline__ void dft8(cplx (&v)[8], uint64_t sign = 0) {
  cplx a0 = cadd(v[0], v[4]), a4 = csub(v[0], v[4]);
  cplx a1 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
  cplx a2 = cadd(v[2], v[6]), a6 = csub(v[2], v[6]);
  cplx a3 = cadd(v[3], v[7]), a7 = csub(v[3], v[7]);
  a5 = mul_w8<INV>(a5);
  a6 = mul_mi<INV>(a6);
  a7 = mul_w83<INV>(a7);
  cplx b0 = cadd(a0, a2), b2 = csub(a0, a2);
  cplx b1 = cadd(a1, a3), b3 = mul_mi<INV>(csub(a1, a3));
  cplx b4 = cadd(a4, a6), b6 = csub(a4, a6);
  cplx b5 = cadd(a5, a7), b7 = mul_mi<INV>(csub(a5, a7));
  if constexpr (RELABEL == 1) {  // OUT_XOR4
    b1 = cneg_if(b1, sign), b3 = cneg_if(b3, sign), b5 = cneg_if(b5, sign), b7 = cneg_if(b7, sign);
  } else if constexpr (RELABEL == 2) {  // IN_XOR4
    b4 = cneg_if(b4, sign), b5 = cneg_if(b5, sign), b6 = cneg_if(b6, sign), b7 = cneg_if(b7, sign);
  }
  v[0] = cadd(b0, b1);
  v[4] = csub(b0, b1);
  v[2] = cadd(b2, b3);
  v[6] = csub(b2, b3);
  v[1] = cadd(b4, b5);
  v[5] = csub(b4, b5);
  v[3] = cadd(b6, b7);
  v[7] = csub(b6, b7);
}

__device__ __forceinline__ int xslot(int a, int b, int c) { return 72 * a + 9 * b + c; }
constexpr int XCH_SLOTS = 72 * 7 + 9 * 7 + 7 + 1;  // 575 complex slots per wave

// Ordering point for intra-wave LDS traffic: LDS operations of one wave execute in issue
// order, so only the compiler has to be kept from moving them across this point.
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Register-only transpose of lane bits 3..5 with the element index (the "hi" transpose of both
// directions: lane (h, lo) element b  ->  lane (b, lo) element h), done as three butterfly
// swaps with cross-lane moves instead of an LDS round trip:
//   lane bit 5 <-> element bit 2: v_permlane32_swap (upper half of v[e] <-> lower half of v[e|4])
//   lane bit 4 <-> element bit 1: v_permlane16_swap (odd rows of v[e] <-> even rows of v[e|2])
//   lane bit 3 <-> element bit 0: DPP row_shr:8 / row_shl:8 under a bank mask (v[e] <-> v[e|1])
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) {
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void swap16(uint32_t& a, uint32_t& b) {
  auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void swap8(uint32_t& a, uint32_t& b) {
  // a keeps lanes with bit 3 = 0 and takes b's (lane - 8) where bit 3 = 1; b the converse
  const uint32_t na = (uint32_t)__builtin_amdgcn_update_dpp((int)a, (int)b, 0x118, 0xF, 0xC, false);
  const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp((int)b, (int)a, 0x108, 0xF, 0x3, false);
  a = na;
  b = nb;
}
template <int MODE>
__device__ __forceinline__ void swap_cplx(cplx& x, cplx& y) {
  uint32_t xa[4], ya[4];
  const uint64_t x0 = (uint64_t)__double_as_longlong(x.re), x1 = (uint64_t)__double_as_longlong(x.im);
  const uint64_t y0 = (uint64_t)__double_as_longlong(y.re), y1 = (uint64_t)__double_as_longlong(y.im);
  xa[0] = (uint32_t)x0, xa[1] = (uint32_t)(x0 >> 32), xa[2] = (uint32_t)x1, xa[3] = (uint32_t)(x1 >> 32);
  ya[0] = (uint32_t)y0, ya[1] = (uint32_t)(y0 >> 32), ya[2] = (uint32_t)y1, ya[3] = (uint32_t)(y1 >> 32);
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if constexpr (MODE == 32) swap32(xa[d], ya[d]);
    else if constexpr (MODE == 16) swap16(xa[d], ya[d]);
    else swap8(xa[d], ya[d]);
  }
  x.re = __longlong_as_double((long long)(((uint64_t)xa[1] << 32) | xa[0]));
  x.im = __longlong_as_double((long long)(((uint64_t)xa[3] << 32) | xa[2]));
  y.re = __longlong_as_double((long long)(((uint64_t)ya[1] << 32) | ya[0]));
  y.im = __longlong_as_double((long long)(((uint64_t)ya[3] << 32) | ya[2]));
}
__device__ __forceinline__ void xpose_hi(cplx (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) swap_cplx<32>(v[e], v[e | 4]);
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (!(e & 2)) swap_cplx<16>(v[e], v[e | 2]);
#pragma unroll
  for (int e = 0; e < 8; e += 2) swap_cplx<8>(v[e], v[e | 1]);
}

// psi^m = exp(i pi m / 16), m = 0..7 (correctly rounded)
__device__ __forceinline__ cplx psi_pow(int m) {
  constexpr double C[8] = {1.0,
                           0.98078528040323044912618223613424,
                           0.92387953251128675612818318939679,
                           0.83146961230254523707878837761791,
                           0.70710678118654752440084436210485,
                           0.55557023301960222474283081394853,
                           0.38268343236508977172845998403040,
                           0.19509032201612826784828486847702};
  return {C[m], C[(8 - m) & 7] * (m == 0 ? 0.0 : 1.0)};
}

// LDS tables shared by the workgroup:
//   T1[k0 * T1_STRIDE + t] = zeta^t * w512^{t k0}   (8 rows of 64, padded to 72 entries)
//   T2[k1 * 8 + t0] = w64^{t0 k1}                   (64 entries, symmetric in (k1, t0))
// The row padding makes the inverse pass-2 read T1[hi * 72 + 8 t1 + lo] conflict-free on the
// ds_read_b128 lane groups (2-way with a 64 stride); the forward read T1[k0 * 72 + lane] stays
// contiguous.  The inverse pass-1 read uses T2's symmetry, T2[t0 * 8 + lo], for the same reason
// (T2[lo * 8 + t0] is 4-way conflicted).
constexpr int T1_STRIDE = 72;
constexpr int FFT512_TABLE_ENTRIES = 8 * T1_STRIDE + 64;
struct Fft512Tables {
  const cplx* T1;
  const cplx* T2;
};

__device__ __forceinline__ void build_fft512_tables(cplx* T1, cplx* T2, int tid, int nthreads) {
  for (int e = tid; e < 512; e += nthreads) {
    const int k0 = e >> 6, t = e & 63;
    double s, c;
    // angle / pi = t / 1024 - 2 t k0 / 512, reduced mod 2
    const int num = (t - 4 * ((t * k0) & 511)) & 2047;  // in units of pi / 1024
    sincospi((double)num / 1024.0, &s, &c);
    T1[k0 * T1_STRIDE + t] = {c, s};
  }
  for (int e = tid; e < 64; e += nthreads) {
    const int k1 = e >> 3, t0 = e & 7;
    double s, c;
    sincospi(-2.0 * (double)((t0 * k1) & 63) / 64.0, &s, &c);
    T2[e] = {c, s};
  }
}

// Forward: v[m] = x[t + 64 m] (real-and-imaginary folded digits, untwisted).
// Stages: P1 (twist, pass 1, twiddles) | W1 R1 (transpose 1) | P2 (pass 2, twiddles) | W2 R2 | P3.
__device__ __forceinline__ void fwd_p1(cplx (&v)[8], const Fft512Tables& T, int lane) {
#pragma unroll
  for (int m = 1; m < 8; ++m) v[m] = cmul(v[m], psi_pow(m));
  dft8<false>(v);
#pragma unroll
  for (int k0 = 0; k0 < 8; ++k0) v[k0] = cmul(v[k0], T.T1[k0 * T1_STRIDE + lane]);
}
// transpose 1: writer lane (t1 = hi, t0 = lo) element k0 ; reader lane (k0 = hi, t0 = lo) element t1
__device__ __forceinline__ void fwd_w1(const cplx (&v)[8], cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) xch[xslot(e, hi, lo)] = v[e];
}
__device__ __forceinline__ void fwd_r1(cplx (&v)[8], const cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = xch[xslot(hi, e, lo)];
}
__device__ __forceinline__ void fwd_p2(cplx (&v)[8], const Fft512Tables& T, int lo) {
  dft8<false>(v);
#pragma unroll
  for (int k1 = 1; k1 < 8; ++k1) v[k1] = cmul(v[k1], T.T2[k1 * 8 + lo]);
}
// transpose 2: writer lane (k0 = hi, t0 = lo) element k1 ; reader lane (k0 = hi, k1 = lo) element t0
__device__ __forceinline__ void fwd_w2(const cplx (&v)[8], cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) xch[xslot(hi, e, lo)] = v[e];
}
__device__ __forceinline__ void fwd_r2(cplx (&v)[8], const cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = xch[xslot(hi, lo, e)];
}

#ifndef XPOSE_HI_REGS
#define XPOSE_HI_REGS 1  // lane-bits-3..5 transposes with cross-lane moves instead of LDS
#endif

__device__ __forceinline__ void fft512_fwd(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane,
                                           uint64_t out_xor4 = 0) {
  const int hi = lane >> 3, lo = lane & 7;
  fwd_p1(v, T, lane);
#if XPOSE_HI_REGS
  xpose_hi(v);
#else
  fwd_w1(v, xch, hi, lo);
  wave_lds_fence();
  fwd_r1(v, xch, hi, lo);
  wave_lds_fence();
#endif
  fwd_p2(v, T, lo);
  fwd_w2(v, xch, hi, lo);
  wave_lds_fence();
  fwd_r2(v, xch, hi, lo);
  wave_lds_fence();
  dft8<false, 1>(v, out_xor4);  // out_xor4 = 1 << 63: slots come out in order k2 ^ 4
}

// Two independent forward transforms through ONE scratch, software-pipelined: each
// transpose's LDS round trip is covered by the other transform's butterflies.  LDS operations
// of a wave execute in issue order, so b's writes cannot overtake a's earlier reads.
__device__ __forceinline__ void fft512_fwd2(cplx (&a)[8], cplx (&b)[8], cplx* xch, const Fft512Tables& T,
                                            int lane) {
  const int hi = lane >> 3, lo = lane & 7;
  fwd_p1(a, T, lane);
  fwd_w1(a, xch, hi, lo);
  wave_lds_fence();
  fwd_r1(a, xch, hi, lo);
  wave_lds_fence();
  fwd_p1(b, T, lane);
  wave_lds_fence();
  fwd_w1(b, xch, hi, lo);
  wave_lds_fence();
  fwd_r1(b, xch, hi, lo);
  wave_lds_fence();
  fwd_p2(a, T, lo);
  wave_lds_fence();
  fwd_w2(a, xch, hi, lo);
  wave_lds_fence();
  fwd_r2(a, xch, hi, lo);
  wave_lds_fence();
  fwd_p2(b, T, lo);
  wave_lds_fence();
  fwd_w2(b, xch, hi, lo);
  wave_lds_fence();
  fwd_r2(b, xch, hi, lo);
  wave_lds_fence();
  dft8<false>(a);
  dft8<false>(b);
}

// Inverse: v[k2] = Y[k0 + 8 k1 + 64 k2] in lane (k0, k1) -> v[m] = sum_k Y_k w^{-jk} * conj(zeta^j),
// j = t + 64 m in lane t.  Stages: P1 | W1 R1 | P2 | W2 R2 | P3 (the kernel interleaves them
// with other work, so each is callable on its own).
__device__ __forceinline__ void inv_p1(cplx (&v)[8], const Fft512Tables& T, int lo, uint64_t in_xor4 = 0) {
  dft8<true, 2>(v, in_xor4);  // over k2 -> t0 ; lane (k0 = hi, k1 = lo); in_xor4: inputs in k2 ^ 4 order
#pragma unroll
  for (int t0 = 1; t0 < 8; ++t0) v[t0] = cmulc(v[t0], T.T2[t0 * 8 + lo]);
}
// transpose 2': writer lane (k0, k1) element t0 ; reader lane (k0 = hi, t0 = lo) element k1
__device__ __forceinline__ void inv_w1(const cplx (&v)[8], cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) xch[xslot(hi, lo, e)] = v[e];
}
__device__ __forceinline__ void inv_r1(cplx (&v)[8], const cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = xch[xslot(hi, e, lo)];
}
__device__ __forceinline__ void inv_p2(cplx (&v)[8], const Fft512Tables& T, int hi, int lo) {
  dft8<true>(v);  // over k1 -> t1 ; lane (k0 = hi, t0 = lo)
#pragma unroll
  for (int t1 = 0; t1 < 8; ++t1) v[t1] = cmulc(v[t1], T.T1[hi * T1_STRIDE + 8 * t1 + lo]);
}
// transpose 1': writer lane (k0 = hi, t0 = lo) element t1 ; reader lane (t1 = hi, t0 = lo) element k0
__device__ __forceinline__ void inv_w2(const cplx (&v)[8], cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) xch[xslot(hi, e, lo)] = v[e];
}
__device__ __forceinline__ void inv_r2(cplx (&v)[8], const cplx* xch, int hi, int lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = xch[xslot(e, hi, lo)];
}
__device__ __forceinline__ void inv_p3(cplx (&v)[8]) {
  dft8<true>(v);  // over k0 -> m ; lane t holds x[t + 64 m] * zeta^t ... times psi^m still to remove
#pragma unroll
  for (int m = 1; m < 8; ++m) v[m] = cmulc(v[m], psi_pow(m));
}

__device__ __forceinline__ void fft512_inv(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane,
                                           uint64_t in_xor4 = 0) {
  const int hi = lane >> 3, lo = lane & 7;
  inv_p1(v, T, lo, in_xor4);
  inv_w1(v, xch, hi, lo);
  wave_lds_fence();
  inv_r1(v, xch, hi, lo);
  wave_lds_fence();
  inv_p2(v, T, hi, lo);
#if XPOSE_HI_REGS
  xpose_hi(v);
#else
  inv_w2(v, xch, hi, lo);
  wave_lds_fence();
  inv_r2(v, xch, hi, lo);
  wave_lds_fence();
#endif
  inv_p3(v);
}

// Frequency index held in (lane, slot) after fft512_fwd.
__host__ __device__ constexpr int fft512_freq(int lane, int slot) { return (lane >> 3) + 8 * (lane & 7) + 64 * slot; }

}  // namespace chip
