// fft512.hpp — one-wavefront 512-point complex FFT for the N = 1024 negacyclic product.
//
// One wave64 owns one polynomial: lane t holds 8 complex points (16 f64 registers).
// 512 = 8 x 8 x 8: three in-register radix-8 passes, two intra-wave transposes (lane bits 3..5
// in registers, lane bits 0..2 through LDS).
// Forward (natural in -> digit-permuted out):
//   in : lane t holds x[t + 64 m], m = 0..7 (untwisted: the negacyclic twist is folded in)
//   out: lane (k0 = t>>3, k1 = t&7) holds Z[k0 + 8 k1 + 64 k2], k2 = 0..7, where
//        Z = DFT_512(x_j * zeta^j), zeta = exp(i pi / 1024), DFT sign exp(-2 pi i jk / 512)
// Inverse (conjugate twiddles, unnormalised) maps that layout back and applies conj(zeta^j),
// so inverse(forward(x)) = 512 x.
// The pointwise product never needs natural frequency order, so no reordering pass exists.
//
// Forward passes as geometric DFTs.  With j = t0 + 8 t1 + 64 m and f = k0 + 8 k1 + 64 k2,
//   Z_f = sum_t0 rho3^t0 w8^{t0 k2} sum_t1 rho2^t1 w8^{t1 k1} sum_m psi^m w8^{m k0} x_j
//   psi = zeta^64,  rho2 = zeta^8 w64^{k0},  rho3 = zeta w512^{k0 + 8 k1}
// i.e. every pass is an 8-point DFT of x_e rho^e ("geometric" input twiddles, rho depending on
// the pass and the lane) and there is no separate twiddle multiplication at all.  A geometric
// DFT8 runs as three radix-2 DIT stages of fused butterflies a +- W b with
// W = c (1 + i t), t = tan(arg W) (Goedecker, "Fast radix 2, 3, 4 and 5 kernels for FFT on
// computers with overlapping multiply-add instructions", 1997): 6 FMAs per butterfly, 72 per
// pass, against 56 + 28 for an 8-point DFT plus its seven twiddle products.  The stage
// twiddles are rho^4, rho^2, rho and rho w8 (the (-i) multiples are free relabelings), read as
// (c, t) pairs from LDS (pass 1: compile-time constants).
// Inverse: pass 1 is a plain 8-point DFT over k2, pass 2 the geometric DFT over k1 with
// rho = conj(w64^{t0}), and pass 3 keeps the classic form (twiddles conj(zeta^t w512^{t k0}),
// 8-point DFT over k0, output twist conj(psi^m)), because its conj(zeta^j) twist sits on the
// OUTPUT side, where a twiddle cannot be fused into a butterfly.
//
// Rounding: |computed Wb - Wb| <= (|c| + |s|) u |b| + the table error, i.e. a butterfly's error
// stays within Higham's radix-2 model (Accuracy and Stability, Thm 24.2) that the certified
// bound of DESIGN.md §3 / oracle ora_fft_error_bound uses (mu ~ 2u against gamma doubled).
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
__device__ __forceinline__ void pin(cplx& a) {  // optimisation barrier (kernel_util.hpp pin)
  asm volatile("" : "+v"(a.re), "+v"(a.im));
}
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

// Negate a complex value when `sign` is 1ull << 63 (sign-bit XOR on both parts, no branch).
__device__ __forceinline__ cplx cneg_if(cplx a, uint64_t sign) {
  return {__longlong_as_double((long long)((uint64_t)__double_as_longlong(a.re) ^ sign)),
          __longlong_as_double((long long)((uint64_t)__double_as_longlong(a.im) ^ sign))};
}
__device__ __forceinline__ double dneg_if(double a, uint64_t sign) {
  return __longlong_as_double((long long)((uint64_t)__double_as_longlong(a) ^ sign));
}

// In-register 8-point DFT, natural order in and out: X[k] = sum_m x[m] w8^{+-mk}.  The two
// w8^{1,3} products are fused into the last stage's additions (FMAs with 1/sqrt2): 52 f64
// operations.  IN_XOR4 (sign = 1ull << 63, else 0): inputs given in order m ^ 4 — the DFT of
// the permuted input is (-1)^k X[k], i.e. the terms of the odd outputs are negated (used by the
// wave of a pair that owns the upper frequency half).
template <bool INV, bool IN_XOR4 = false>
__device__ __forceinline__ void dft8(cplx (&v)[8], uint64_t sign = 0) {
  const double r = dneg_if(0.70710678118654752440084436210485, IN_XOR4 ? sign : 0ull);
  cplx a0 = cadd(v[0], v[4]), a4 = csub(v[0], v[4]);
  cplx a1 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
  cplx a2 = cadd(v[2], v[6]), a6 = csub(v[2], v[6]);
  cplx a3 = cadd(v[3], v[7]), a7 = csub(v[3], v[7]);
  a6 = mul_mi<INV>(a6);
  // w8 a5 = r p5, w8^3 a7 = r p7
  cplx p5, p7;
  if constexpr (INV) {
    p5 = {a5.re - a5.im, a5.re + a5.im};
    p7 = {-a7.re - a7.im, a7.re - a7.im};
  } else {
    p5 = {a5.re + a5.im, a5.im - a5.re};
    p7 = {a7.im - a7.re, -a7.re - a7.im};
  }
  const cplx q = cadd(p5, p7), qq = mul_mi<INV>(csub(p5, p7));  // b5 = r q, b7 = r qq
  cplx b0 = cadd(a0, a2), b2 = csub(a0, a2);
  cplx b1 = cadd(a1, a3), b3 = mul_mi<INV>(csub(a1, a3));
  cplx b4 = cadd(a4, a6), b6 = csub(a4, a6);
  if constexpr (IN_XOR4) b4 = cneg_if(b4, sign), b6 = cneg_if(b6, sign);
  v[0] = cadd(b0, b1);
  v[4] = csub(b0, b1);
  v[2] = cadd(b2, b3);
  v[6] = csub(b2, b3);
  v[1] = {__builtin_fma(r, q.re, b4.re), __builtin_fma(r, q.im, b4.im)};
  v[5] = {__builtin_fma(-r, q.re, b4.re), __builtin_fma(-r, q.im, b4.im)};
  v[3] = {__builtin_fma(r, qq.re, b6.re), __builtin_fma(r, qq.im, b6.im)};
  v[7] = {__builtin_fma(-r, qq.re, b6.re), __builtin_fma(-r, qq.im, b6.im)};
}

// Fused radix-2 butterfly (a, b) <- (a + W' b, a - W' b), W = c (1 + i t), W' = W (ROT 0),
// -i W (ROT 1) or +i W (ROT 2): W b = c (u + i v), u = b.re - t b.im, v = b.im + t b.re.
template <int ROT>
__device__ __forceinline__ void gbf(cplx& a, cplx& b, double c, double t) {
  const double u = __builtin_fma(-t, b.im, b.re);
  const double v = __builtin_fma(t, b.re, b.im);
  double pr, pi;
  if constexpr (ROT == 0) pr = u, pi = v;
  else if constexpr (ROT == 1) pr = v, pi = -u;
  else pr = -v, pi = u;
  const cplx y0 = {__builtin_fma(c, pr, a.re), __builtin_fma(c, pi, a.im)};
  const cplx y1 = {__builtin_fma(-c, pr, a.re), __builtin_fma(-c, pi, a.im)};
  a = y0;
  b = y1;
}

// Geometric 8-point DFT: y[k] = sum_e x[e] rho^e w^{ek}, w = exp(-+ i pi / 4) (forward /
// inverse), natural order in and out.  tw[0..3] = (c, t) of rho^4, rho^2, rho, rho w (stored as
// cplx {c, t}).  Stages: e ^ 4 pairs with rho^4; e ^ 2 pairs with rho^2 (k even) or w^2 rho^2
// (k odd); e ^ 1 pairs with rho w^{k mod 4}.  out_sign = 1ull << 63 emits y[k ^ 4] in slot k (the
// sign of the last stage's twiddles; OUT_XOR4 relabeling of the upper-half wave).
// CS4: tw[0] holds (cos, sin) of rho^4 instead of (c, t) and the first stage multiplies in full
// (the inverse pass 2, whose rho^4 = exp(i pi t0 / 8) is exactly i at t0 = 4: no tangent).
template <bool INV, bool CS4 = false>
__device__ __forceinline__ void geo8(cplx (&v)[8], const cplx (&tw)[4], uint64_t out_sign = 0) {
  constexpr int R = INV ? 2 : 1;  // w^2 = -i (forward) or +i (inverse)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if constexpr (CS4) {
      const cplx wb = cmul(v[e + 4], tw[0]);
      v[e + 4] = csub(v[e], wb);
      v[e] = cadd(v[e], wb);
    } else {
      gbf<0>(v[e], v[e + 4], tw[0].re, tw[0].im);
    }
  }
  gbf<0>(v[0], v[2], tw[1].re, tw[1].im);
  gbf<0>(v[1], v[3], tw[1].re, tw[1].im);
  gbf<R>(v[4], v[6], tw[1].re, tw[1].im);
  gbf<R>(v[5], v[7], tw[1].re, tw[1].im);
  const double c2 = dneg_if(tw[2].re, out_sign), c3 = dneg_if(tw[3].re, out_sign);
  gbf<0>(v[0], v[1], c2, tw[2].im);  // y0, y4
  gbf<0>(v[4], v[5], c3, tw[3].im);  // y1, y5
  gbf<R>(v[2], v[3], c2, tw[2].im);  // y2, y6
  gbf<R>(v[6], v[7], c3, tw[3].im);  // y3, y7
  const cplx y1 = v[4], y2 = v[2], y3 = v[6], y4 = v[1], y5 = v[5], y6 = v[3];
  v[1] = y1, v[2] = y2, v[3] = y3, v[4] = y4, v[5] = y5, v[6] = y6;
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

// LDS tables shared by the workgroup (cplx entries):
//   T1[k0 * T1_STRIDE + t] = zeta^t * w512^{t k0}   (8 rows of 64, padded to 72 entries;
//                                                   inverse pass-2 output twiddles, conjugated)
//   GF2[j * 8 + k0]   (c, t) of the forward pass-2 stage twiddles, rho2 = zeta^8 w64^{k0}
//   GF3[j * 64 + lane] (c, t) of the forward pass-3 stage twiddles, rho3 = zeta w512^{k0 + 8 k1}
//   GI2[j * 8 + t0]   (c, t) of the inverse pass-2 stage twiddles, rho = conj(w64^{t0})
//                     (j = 0: (cos, sin) of rho^4, which is i at t0 = 4)
// with j = 0..3 for rho^4, rho^2, rho, rho w.  The [j][index] order keeps every read
// conflict-free (consecutive lanes, or broadcasts of 8 distinct 16-byte entries).  The T1 row
// padding makes the inverse pass-2 read T1[hi * 72 + 8 t1 + lo] conflict-free on the
// ds_read_b128 lane groups (2-way with a 64 stride).
constexpr int T1_STRIDE = 72;
constexpr int FFT512_T1_ENTRIES = 8 * T1_STRIDE;
constexpr int FFT512_TABLE_ENTRIES = FFT512_T1_ENTRIES + 4 * 8 + 4 * 64 + 4 * 8;
struct Fft512Tables {
  const cplx* T1;
  const cplx* GF2;
  const cplx* GF3;
  const cplx* GI2;
};
__device__ __forceinline__ Fft512Tables fft512_tables_at(const cplx* base) {
  return {base, base + FFT512_T1_ENTRIES, base + FFT512_T1_ENTRIES + 32, base + FFT512_T1_ENTRIES + 32 + 256};
}

// (c, t) of exp(i pi a), a in units of pi; c = cos, t = tan (never near pi/2 for the angles it is
// used on: |cos| >= 0.012)
__device__ __forceinline__ cplx geo_ct(double a) {
  double s, c;
  sincospi(a, &s, &c);
  return {c, s / c};
}
// angle (units of pi) of stage twiddle j for base angle a and w8 = exp(wsign i pi / 4)
__device__ __forceinline__ double geo_angle(int j, double a, double wsign) {
  return j == 0 ? 4.0 * a : j == 1 ? 2.0 * a : j == 2 ? a : a + 0.25 * wsign;
}

__device__ __forceinline__ void build_fft512_tables(cplx* base, int tid, int nthreads) {
  cplx* T1 = base;
  cplx* GF2 = base + FFT512_T1_ENTRIES;
  cplx* GF3 = GF2 + 32;
  cplx* GI2 = GF3 + 256;
  for (int e = tid; e < 512; e += nthreads) {
    const int k0 = e >> 6, t = e & 63;
    double s, c;
    // angle / pi = t / 1024 - 2 t k0 / 512, reduced mod 2
    const int num = (t - 4 * ((t * k0) & 511)) & 2047;  // in units of pi / 1024
    sincospi((double)num / 1024.0, &s, &c);
    T1[k0 * T1_STRIDE + t] = {c, s};
  }
  for (int e = tid; e < 4 * 64; e += nthreads) {
    const int j = e >> 6, lane = e & 63, k0 = lane >> 3, k1 = lane & 7;
    GF3[e] = geo_ct(geo_angle(j, 1.0 / 1024.0 - (double)(k0 + 8 * k1) / 256.0, -1.0));
  }
  for (int e = tid; e < 4 * 8; e += nthreads) {
    const int j = e >> 3, x = e & 7;
    GF2[e] = geo_ct(geo_angle(j, 1.0 / 128.0 - (double)x / 32.0, -1.0));
    if (j == 0) {  // (cos, sin) of rho^4 (geo8<true, true>)
      double s, c;
      sincospi((double)x / 8.0, &s, &c);
      GI2[e] = {c, s};
    } else {
      GI2[e] = geo_ct(geo_angle(j, (double)x / 32.0, 1.0));
    }
  }
}

// Forward: v[m] = x[t + 64 m] (real-and-imaginary folded digits, untwisted).
// Stages: P1 (geometric, rho = psi) | hi transpose (registers) | P2 (geometric, rho2) |
//         W2 R2 (LDS transpose) | P3 (geometric, rho3).
__device__ __forceinline__ void fwd_p1(cplx (&v)[8]) {
  // (c, t) of psi^4, psi^2, psi, psi w8 with psi = exp(i pi / 16), w8 = exp(-i pi / 4)
  const cplx tw[4] = {{0x1.6a09e667f3bcdp-1, 1.0},
                      {0x1.d906bcf328d46p-1, 0x1.a827999fcef32p-2},
                      {0x1.f6297cff75cb0p-1, 0x1.975f5e0553158p-3},
                      {0x1.a9b66290ea1a3p-1, -0x1.561b82ab7f990p-1}};
  geo8<false>(v, tw);
}
__device__ __forceinline__ void fwd_p2(cplx (&v)[8], const Fft512Tables& T, int hi) {
  const cplx tw[4] = {T.GF2[hi], T.GF2[8 + hi], T.GF2[16 + hi], T.GF2[24 + hi]};
  geo8<false>(v, tw);
}
__device__ __forceinline__ void fwd_p3_tw(cplx (&tw)[4], const Fft512Tables& T, int lane) {
  tw[0] = T.GF3[lane], tw[1] = T.GF3[64 + lane], tw[2] = T.GF3[128 + lane], tw[3] = T.GF3[192 + lane];
}
__device__ __forceinline__ void fwd_p3(cplx (&v)[8], const Fft512Tables& T, int lane, uint64_t out_xor4) {
  cplx tw[4];
  fwd_p3_tw(tw, T, lane);
  geo8<false>(v, tw, out_xor4);
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

// Forward transform with the pass-2 and pass-3 twiddles supplied (kept in registers by the
// caller: fwd_p2_tw / fwd_p3_tw) and a hook run right before the transform's first LDS write (a
// pair wait in pbs.hip).
__device__ __forceinline__ void fwd_p2_tw(cplx (&tw)[4], const Fft512Tables& T, int hi) {
  tw[0] = T.GF2[hi], tw[1] = T.GF2[8 + hi], tw[2] = T.GF2[16 + hi], tw[3] = T.GF2[24 + hi];
}
template <class BeforeLds>
__device__ __forceinline__ void fft512_fwd_tw(cplx (&v)[8], cplx* xch, int lane, const cplx (&tw2)[4],
                                              const cplx (&tw3)[4], uint64_t out_xor4, BeforeLds before_lds) {
  const int hi = lane >> 3, lo = lane & 7;
  fwd_p1(v);
  xpose_hi(v);  // lane (k0 = hi, t0 = lo), element t1
  geo8<false>(v, tw2);
  before_lds();
  fwd_w2(v, xch, hi, lo);
  wave_lds_fence();
  fwd_r2(v, xch, hi, lo);
  wave_lds_fence();
  geo8<false>(v, tw3, out_xor4);  // out_xor4 = 1 << 63: slots come out in order k2 ^ 4
}

__device__ __forceinline__ void fft512_fwd(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane,
                                           uint64_t out_xor4 = 0) {
  const int hi = lane >> 3, lo = lane & 7;
  fwd_p1(v);
  xpose_hi(v);  // lane (k0 = hi, t0 = lo), element t1
  fwd_p2(v, T, hi);
  cplx tw3[4];  // pass-3 twiddles read ahead of the transpose: their latency hides in its round trip
  fwd_p3_tw(tw3, T, lane);
  fwd_w2(v, xch, hi, lo);
  wave_lds_fence();
  fwd_r2(v, xch, hi, lo);
  wave_lds_fence();
  geo8<false>(v, tw3, out_xor4);  // out_xor4 = 1 << 63: slots come out in order k2 ^ 4
}

// Inverse: v[k2] = Y[k0 + 8 k1 + 64 k2] in lane (k0, k1) -> v[m] = sum_k Y_k w^{-jk} * conj(zeta^j),
// j = t + 64 m in lane t.  Stages: P1 | W1 R1 | P2 | hi transpose | P3 (the kernel interleaves
// them with other work, so each is callable on its own).
__device__ __forceinline__ void inv_p1(cplx (&v)[8], uint64_t in_xor4 = 0) {
  dft8<true, true>(v, in_xor4);  // over k2 -> t0 ; lane (k0 = hi, k1 = lo); in_xor4: inputs in k2 ^ 4 order
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
// inverse pass-2 twiddles: tw[0..3] geometric stages, tw[4..11] the output twiddles
__device__ __forceinline__ void inv_p2_tw(cplx (&tw)[12], const Fft512Tables& T, int hi, int lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) tw[j] = T.GI2[8 * j + lo];
#pragma unroll
  for (int t1 = 0; t1 < 8; ++t1) tw[4 + t1] = T.T1[hi * T1_STRIDE + 8 * t1 + lo];
}
__device__ __forceinline__ void inv_p2_with(cplx (&v)[8], const cplx (&tw)[12]) {
  // geometric over k1 -> t1 with rho = conj(w64^{t0}); lane (k0 = hi, t0 = lo)
  const cplx g[4] = {tw[0], tw[1], tw[2], tw[3]};
  geo8<true, true>(v, g);
#pragma unroll
  for (int t1 = 0; t1 < 8; ++t1) v[t1] = cmulc(v[t1], tw[4 + t1]);
}
__device__ __forceinline__ void inv_p2(cplx (&v)[8], const Fft512Tables& T, int hi, int lo) {
  cplx tw[12];
  inv_p2_tw(tw, T, hi, lo);
  inv_p2_with(v, tw);
}
__device__ __forceinline__ void inv_p3(cplx (&v)[8]) {
  dft8<true>(v);  // over k0 -> m ; lane t holds x[t + 64 m] * zeta^t ... times psi^m still to remove
#pragma unroll
  for (int m = 1; m < 8; ++m) v[m] = cmulc(v[m], psi_pow(m));
}

// Inverse with the pass-2 stage twiddles supplied (registers) and the output twiddles read after
// the LDS transpose (their latency hides behind the pass-2 butterflies).
__device__ __forceinline__ void fft512_inv_tw(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane,
                                              const cplx (&gi2)[4], uint64_t in_xor4) {
  const int hi = lane >> 3, lo = lane & 7;
  inv_p1(v, in_xor4);
  inv_w1(v, xch, hi, lo);
  wave_lds_fence();
  inv_r1(v, xch, hi, lo);
  wave_lds_fence();
  cplx t1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) t1[t] = T.T1[hi * T1_STRIDE + 8 * t + lo];
  geo8<true, true>(v, gi2);
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] = cmulc(v[t], t1[t]);
  xpose_hi(v);
  inv_p3(v);
}
__device__ __forceinline__ void inv_p2_stage_tw(cplx (&tw)[4], const Fft512Tables& T, int lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) tw[j] = T.GI2[8 * j + lo];
}

__device__ __forceinline__ void fft512_inv(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane,
                                           uint64_t in_xor4 = 0) {
  const int hi = lane >> 3, lo = lane & 7;
  inv_p1(v, in_xor4);
  cplx tw[12];  // pass-2 twiddles read ahead of the transpose
  inv_p2_tw(tw, T, hi, lo);
  inv_w1(v, xch, hi, lo);
  wave_lds_fence();
  inv_r1(v, xch, hi, lo);
  wave_lds_fence();
  inv_p2_with(v, tw);
  xpose_hi(v);
  inv_p3(v);
}

// Frequency index held in (lane, slot) after fft512_fwd.
__host__ __device__ constexpr int fft512_freq(int lane, int slot) { return (lane >> 3) + 8 * (lane & 7) + 64 * slot; }

}  // namespace chip
