// bsk.hip — on-device conversion of the standard u64 bootstrapping key into the exact-limb
// Fourier key consumed by pbs.hip.
//
// Reference: cuda_convert_lwe_programmable_bootstrap_key_64 as called by the runtime
// (compiler include/concretelang/Runtime/context.h:86-115); CPU counterpart
// concrete-cpu c_api/bootstrap.rs:241-318 (f64 Fourier conversion).  Here every key
// polynomial g (u64) is split into LIMBS balanced signed limbs, each limb is folded,
// twisted and transformed with a double-double (~106-bit) radix-2 FFT, so the stored f64
// spectrum is correctly rounded to within 1 ulp: the certified error bound of DESIGN.md §3
// charges only u * |G| for the key side.
//
// Input layout : [n][l][k+1 (row)][k+1 (col)][N] u64 (concrete-cpu bootstrap.rs:417-429)
// Output layout: [n][col][limb][row*l + q][k2][lane] complex f64, q = l-1-level_index,
//                frequency of (lane, k2) = fft512_freq(lane, k2), scaled by 2/N.
#include <cmath>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "fft512.hpp"
#include "keycheck.hpp"
#include "pbs.hpp"

namespace chip {

void keep_pool_memory();  // abi.hip: the default pool never releases (see there)

struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd quick_two_sum(double a, double b) {
  double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ dd two_sum(double a, double b) {
  double s = a + b;
  double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd dd_add(dd x, dd y) {
  dd s = two_sum(x.hi, y.hi);
  dd t = two_sum(x.lo, y.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ dd dd_neg(dd x) { return {-x.hi, -x.lo}; }
__device__ __forceinline__ dd dd_mul(dd x, dd y) {
  double p = x.hi * y.hi;
  double e = __builtin_fma(x.hi, y.hi, -p);
  e += x.hi * y.lo + x.lo * y.hi;
  return quick_two_sum(p, e);
}
__device__ __forceinline__ dd dd_from(double a) { return {a, 0.0}; }

struct ddc {
  dd re, im;
};
__device__ __forceinline__ ddc ddc_mul(ddc a, ddc w) {
  return {dd_add(dd_mul(a.re, w.re), dd_neg(dd_mul(a.im, w.im))), dd_add(dd_mul(a.re, w.im), dd_mul(a.im, w.re))};
}

// balanced signed limb `limb` of a 64-bit word (limb widths 64/LIMBS, the first 64 % LIMBS one
// bit wider: 22/21/21 for 3 limbs, 16 x 4 for 4): x = sum_t limb_t 2^{s_t} (mod 2^64)
template <int LIMBS>
__device__ __forceinline__ double limb_value(uint64_t rem, uint32_t limb) {
  int64_t lv = 0;
  for (int t = 0; t <= (int)limb; ++t) {
    int w = 64 / LIMBS + (t < 64 % LIMBS ? 1 : 0);
    uint64_t mask = (1ull << w) - 1ull;
    uint64_t vv = rem & mask;
    int64_t sgn = (vv >= (1ull << (w - 1))) ? (int64_t)vv - (int64_t)(1ull << w) : (int64_t)vv;
    lv = sgn;
    rem = (rem - (uint64_t)sgn) >> w;
  }
  return (double)lv;
}

// In-LDS radix-2 DIT over buf (bit-reversed input, natural output, forward sign)
template <int M>
__device__ __forceinline__ void dd_fft(ddc* buf, const ddc* __restrict__ tw_t) {
  for (int h = 1; h < M; h <<= 1) {
    for (int b = threadIdx.x; b < M / 2; b += blockDim.x) {
      const int grp = b / h, pos = b % h;
      const int i0 = grp * 2 * h + pos, i1 = i0 + h;
      const ddc w = tw_t[pos * (M / (2 * h))];
      const ddc x0 = buf[i0];
      const ddc x1 = ddc_mul(buf[i1], w);
      buf[i0] = {dd_add(x0.re, x1.re), dd_add(x0.im, x1.im)};
      buf[i1] = {dd_add(x0.re, dd_neg(x1.re)), dd_add(x0.im, dd_neg(x1.im))};
    }
    __syncthreads();
  }
}

// dd_fft, then the scatter into the PBS kernels' register layout: element e = (slot, lane) holds
// frequency fft512_freq(lane, slot), scaled 1/M, stored at dst(e).
template <int M, class Dst>
__device__ __forceinline__ void dd_fft_scatter(ddc* buf, const ddc* __restrict__ tw_t, Dst dst,
                                               unsigned long long* smax) {
  dd_fft<M>(buf, tw_t);
  const double scale = 1.0 / (double)M;
  double m2 = 0.0;
  for (int e = threadIdx.x; e < M; e += blockDim.x) {
    const int lane = e & 63, slot = e >> 6;
    const int f = fft512_freq(lane, slot);
    const ddc x = buf[f];
    const cplx y = {(x.re.hi + x.re.lo) * scale, (x.im.hi + x.im.lo) * scale};
    *dst(e) = y;
    m2 = fmax(m2, spec_mag2(y.re, y.im));
  }
  spec_max_commit(smax, m2);
}

// tables: zeta[j] = exp(i pi j / N) for j < N/2 ; tw[t] = exp(-2 pi i t / (N/2)) for t < N/4
template <int N, int K, int L, int LIMBS>
__global__ void __launch_bounds__(256) convert_bsk_kernel(cplx* __restrict__ dest, const uint64_t* __restrict__ src,
                                                         const ddc* __restrict__ zeta_t, const ddc* __restrict__ tw_t,
                                                         uint32_t n, unsigned long long* smax) {
  constexpr int M = N / 2, LOGM = (M == 512 ? 9 : (M == 1024 ? 10 : (M == 256 ? 8 : 11)));
  constexpr int K1 = K + 1;
  __shared__ ddc buf[M];
  // block = (poly, limb); poly index in the standard layout
  const uint64_t blk = blockIdx.x;
  const uint32_t limb = (uint32_t)(blk % LIMBS);
  const uint64_t poly = blk / LIMBS;
  const uint32_t col = (uint32_t)(poly % K1);
  const uint32_t row = (uint32_t)((poly / K1) % K1);
  const uint32_t v = (uint32_t)((poly / (K1 * K1)) % L);
  const uint64_t i = poly / ((uint64_t)K1 * K1 * L);
  const uint64_t* g = src + poly * N;

  for (int j = threadIdx.x; j < M; j += blockDim.x) {
    // z_j = (a + i b) * zeta^j ; store at bit-reversed position for the DIT passes
    ddc z{dd_from(limb_value<LIMBS>(g[j], limb)), dd_from(limb_value<LIMBS>(g[j + M], limb))};
    z = ddc_mul(z, zeta_t[j]);
    const int r = (int)(__builtin_bitreverse32((uint32_t)j) >> (32 - LOGM));
    buf[r] = z;
  }
  __syncthreads();
  // layout [n][limb][co][ro][q][slot][lane] (pbs.hip): slots 0..3 of group (limb, co, ro) hold
  // column co / row ro, slots 4..7 hold column 1 - co / row 1 - ro (K = 1), so each wave of a
  // pair reads "own" and "other" spectra at fixed positions
  static_assert(K1 == 2, "own/other key layout assumes k = 1");
  const uint32_t q = (uint32_t)(L - 1) - v;
  cplx* base = dest + i * (uint64_t)(LIMBS * 4 * L * M);  // per GGSW: limbs x co x ro x levels
  dd_fft_scatter<M>(buf, tw_t, [&](int e) {
    const int slot = e >> 6, lane = e & 63;
    const uint32_t co = slot < 4 ? col : 1u - col, ro = slot < 4 ? row : 1u - row;
    return base + (((uint64_t)(limb * 2 + co) * 2 + ro) * L + q) * M + slot * 64 + lane;
  }, smax);
}

// N = 2048, k = 1, l = 1 (pbs2048.hip).  Block = (i, limb, col, row, parity), in the order of
// the output layout [n][limb][col][row][parity][512]: the parity half p(u) = g[2u + par] of key
// polynomial g (row, col), limb `limb`, as an N = 1024 negacyclic polynomial: folded, twisted,
// transformed exactly like the N = 1024 key.
#if P2_PM
// P2_PM: block = (i, limb, col, q, row); both parity spectra G_e, G_o in double-double, then the key
// at the square roots of each evaluation point, K+-[f] = (G_e[f] +- s_f G_o[f]) / 2 with
// s_f = exp(i pi (1 - 4 f) / 2048) (s_f^2 = alpha_f), correctly rounded from double-double.  Layout
// [n][limb][col][q][row][+-][slot][lane] (level v = l - 1 - q, q in digit order), scaled 1/512 like
// the even/odd key.
template <int LIMBS>
__global__ void __launch_bounds__(256) convert_bsk2048_kernel(cplx* __restrict__ dest, const uint64_t* __restrict__ src,
                                                             const ddc* __restrict__ zeta_t,
                                                             const ddc* __restrict__ tw_t,
                                                             const ddc* __restrict__ sroot_t, uint32_t level,
                                                             unsigned long long* smax) {
  constexpr int M = 512, LOGM = 9;
  __shared__ ddc buf[2][M];
  const uint64_t blk = blockIdx.x;
  const uint32_t row = (uint32_t)(blk & 1);
  const uint32_t q = (uint32_t)((blk >> 1) % level);
  const uint32_t col = (uint32_t)((blk >> 1) / level & 1);
  const uint32_t limb = (uint32_t)(((blk >> 1) / level >> 1) % LIMBS);
  const uint64_t i = ((blk >> 1) / level >> 1) / LIMBS;
  const uint32_t v = level - 1 - q;
  const uint64_t* g = src + ((i * level + v) * 4 + row * 2 + col) * 2048;  // [n][l][row][col][N]
  for (int e = threadIdx.x; e < 2 * M; e += blockDim.x) {
    const int par = e / M, j = e % M;
    ddc z{dd_from(limb_value<LIMBS>(g[2 * j + par], limb)), dd_from(limb_value<LIMBS>(g[2 * (j + M) + par], limb))};
    z = ddc_mul(z, zeta_t[j]);
    const int r = (int)(__builtin_bitreverse32((uint32_t)j) >> (32 - LOGM));
    buf[par][r] = z;
  }
  __syncthreads();
  dd_fft<M>(buf[0], tw_t);
  dd_fft<M>(buf[1], tw_t);
  const double scale = 0.5 / (double)M;
  cplx* base = dest + blk * 2 * M;
  double m2 = 0.0;
  for (int e = threadIdx.x; e < M; e += blockDim.x) {
    const int f = fft512_freq(e & 63, e >> 6);
    const ddc so = ddc_mul(buf[1][f], sroot_t[f]);
    const ddc ge = buf[0][f];
    const ddc kp{dd_add(ge.re, so.re), dd_add(ge.im, so.im)};
    const ddc km{dd_add(ge.re, dd_neg(so.re)), dd_add(ge.im, dd_neg(so.im))};
    const cplx yp = {(kp.re.hi + kp.re.lo) * scale, (kp.im.hi + kp.im.lo) * scale};
    const cplx ym = {(km.re.hi + km.re.lo) * scale, (km.im.hi + km.im.lo) * scale};
    base[e] = yp;
    base[M + e] = ym;
    m2 = fmax(m2, fmax(spec_mag2(yp.re, yp.im), spec_mag2(ym.re, ym.im)));
  }
  spec_max_commit(smax, m2);
}
#else
template <int LIMBS>
__global__ void __launch_bounds__(256) convert_bsk2048_kernel(cplx* __restrict__ dest, const uint64_t* __restrict__ src,
                                                             const ddc* __restrict__ zeta_t,
                                                             const ddc* __restrict__ tw_t, const ddc* __restrict__,
                                                             uint32_t level, unsigned long long* smax) {
  constexpr int M = 512, LOGM = 9;
  __shared__ ddc buf[M];
  const uint64_t blk = blockIdx.x;
  const uint32_t par = (uint32_t)(blk & 1);
  const uint32_t row = (uint32_t)((blk >> 1) & 1);
  const uint32_t q = (uint32_t)((blk >> 2) % level);
  const uint32_t col = (uint32_t)((blk >> 2) / level & 1);
  const uint32_t limb = (uint32_t)(((blk >> 2) / level >> 1) % LIMBS);
  const uint64_t i = ((blk >> 2) / level >> 1) / LIMBS;
  const uint32_t v = level - 1 - q;
  const uint64_t* g = src + ((i * level + v) * 4 + row * 2 + col) * 2048;  // [n][l][row][col][N]
  for (int j = threadIdx.x; j < M; j += blockDim.x) {
    ddc z{dd_from(limb_value<LIMBS>(g[2 * j + par], limb)), dd_from(limb_value<LIMBS>(g[2 * (j + M) + par], limb))};
    z = ddc_mul(z, zeta_t[j]);
    const int r = (int)(__builtin_bitreverse32((uint32_t)j) >> (32 - LOGM));
    buf[r] = z;
  }
  __syncthreads();
  dd_fft_scatter<M>(buf, tw_t, [&](int e) { return dest + blk * M + e; }, smax);
}
#endif

// N = 1024, k = 2 (pbs1024k2.hip; l >= K2_MANY_MIN: level-major, [n][q][limb][col][row][512]).  Block = (i, limb, col, q, row), in the order of the
// output layout [n][limb][col][q][row][512]: limb `limb` of key polynomial (row, col) of level
// v = l - 1 - q (q in digit order), folded, twisted and transformed like the k = 1 key.
__global__ void __launch_bounds__(256) convert_bsk1024k2_kernel(cplx* __restrict__ dest,
                                                               const uint64_t* __restrict__ src,
                                                               const ddc* __restrict__ zeta_t,
                                                               const ddc* __restrict__ tw_t, uint32_t level,
                                                               unsigned long long* smax) {
  constexpr int M = 512, LOGM = 9, N = 1024;
  __shared__ ddc buf[M];
  const uint64_t blk = blockIdx.x;
  const uint32_t row = (uint32_t)(blk % 3);
  uint32_t q, col, limb;
  uint64_t i;
  if (level >= K2_MANY_MIN) {  // level-major: [n][q][limb][col][row]
    col = (uint32_t)((blk / 3) % 3);
    limb = (uint32_t)((blk / 9) % K2_LIMBS);
    q = (uint32_t)((blk / (9 * K2_LIMBS)) % level);
    i = blk / (9 * K2_LIMBS * level);
  } else {
    q = (uint32_t)((blk / 3) % level);
    col = (uint32_t)((blk / (3 * level)) % 3);
    limb = (uint32_t)((blk / (9 * level)) % K2_LIMBS);
    i = blk / (9 * level * K2_LIMBS);
  }
  const uint32_t v = level - 1 - q;
  const uint64_t* g = src + (((i * level + v) * 3 + row) * 3 + col) * N;  // [n][l][row][col][N]
  for (int j = threadIdx.x; j < M; j += blockDim.x) {
    ddc z{dd_from(limb_value<K2_LIMBS>(g[j], limb)), dd_from(limb_value<K2_LIMBS>(g[j + M], limb))};
    z = ddc_mul(z, zeta_t[j]);
    const int r = (int)(__builtin_bitreverse32((uint32_t)j) >> (32 - LOGM));
    buf[r] = z;
  }
  __syncthreads();
  dd_fft_scatter<M>(buf, tw_t, [&](int e) { return dest + blk * M + e; }, smax);
}

// N = 512, k = 3 / N = 256, k = 5, 6, l <= 3 (pbs_small.hip) and N = 512, k = 4, l = 1, 3 .. 5
// (pbs512k4.hip).  Block = (i, limb, cg, q, c2, row) in the order of the output layout
// [n][limb][cg][q][c2][row][N/2] (a key group: one limb, one level, GC = sm_gc(N, K1) output columns
// col = cg GC + c2): limb `limb` of key polynomial (row, col) of level v = l - 1 - q (q in digit
// order), folded, twisted by zeta_2N^j and transformed (M = N / 2 points), scaled 1 / (512 P) with
// P = 1024 / N (the kernels' unnormalised unzip and zip), element e = (slot, lane) at frequency
// fft512_freq(lane, slot).  k = 4, N = 512, l >= K4_MANY_MIN: level-major, [n][q][limb][col][row][N/2].
template <int N, int K1, int LIMBS = SM_LIMBS>
__global__ void __launch_bounds__(256) convert_bsk_small_kernel(cplx* __restrict__ dest,
                                                               const uint64_t* __restrict__ src,
                                                               const ddc* __restrict__ zeta_t,
                                                               const ddc* __restrict__ tw_t, uint32_t level,
                                                               unsigned long long* smax) {
  constexpr int M = N / 2, LOGM = N == 512 ? 8 : 7, P = 1024 / N;
  constexpr int GC = sm_gc(N, K1), NCG = K1 / GC;
  __shared__ ddc buf[M];
  const uint64_t blk = blockIdx.x;
  uint64_t t = blk;
  const uint32_t row = (uint32_t)(t % K1);
  t /= K1;
  uint32_t c2, q, cg, limb;
  uint64_t i;
  if (N == 512 && K1 == 5 && level >= K4_MANY_MIN) {  // level-major: [n][q][limb][col][row] (GC = 1)
    c2 = 0;
    cg = (uint32_t)(t % K1);
    t /= K1;
    limb = (uint32_t)(t % LIMBS);
    t /= LIMBS;
    q = (uint32_t)(t % level);
    i = t / level;
  } else {
    c2 = (uint32_t)(t % GC);
    t /= GC;
    q = (uint32_t)(t % level);
    t /= level;
    cg = (uint32_t)(t % NCG);
    t /= NCG;
    limb = (uint32_t)(t % LIMBS);
    i = t / LIMBS;
  }
  const uint32_t col = cg * GC + c2, v = level - 1 - q;
  const uint64_t* g = src + (((i * level + v) * K1 + row) * K1 + col) * N;  // [n][l][row][col][N]
  for (int j = threadIdx.x; j < M; j += blockDim.x) {
    ddc z{dd_from(limb_value<LIMBS>(g[j], limb)), dd_from(limb_value<LIMBS>(g[j + M], limb))};
    z = ddc_mul(z, zeta_t[j]);
    const int r = (int)(__builtin_bitreverse32((uint32_t)j) >> (32 - LOGM));
    buf[r] = z;
  }
  __syncthreads();
  dd_fft<M>(buf, tw_t);
  const double scale = 1.0 / (512.0 * P);
  double m2 = 0.0;
  for (int e = threadIdx.x; e < M; e += blockDim.x) {
    const ddc x = buf[fft512_freq(e & 63, e >> 6)];
    const cplx y = {(x.re.hi + x.re.lo) * scale, (x.im.hi + x.im.lo) * scale};
    dest[blk * M + e] = y;
    m2 = fmax(m2, spec_mag2(y.re, y.im));
  }
  spec_max_commit(smax, m2);
}

template <int N, int K, int L, int LIMBS>
static int launch_convert(const ConvertArgs& a, const ddc* zeta, const ddc* tw) {
  const uint64_t blocks = (uint64_t)a.n * L * (K + 1) * (K + 1) * LIMBS;
  hipLaunchKernelGGL((convert_bsk_kernel<N, K, L, LIMBS>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                     reinterpret_cast<cplx*>(a.dest), a.src_dev, zeta, tw, a.n, a.smax);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("convert launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

struct dd_host {
  double hi, lo;
};
// dd twiddle tables from long double (64-bit mantissa): hi = rn(x), lo = rn(x - hi)
static void make_tables(uint32_t N, std::vector<ddc>& zeta, std::vector<ddc>& tw) {
  const long double PI = 3.14159265358979323846264338327950288L;
  const uint32_t M = N / 2;
  zeta.resize(M);
  tw.resize(M / 2);
  auto split = [](long double x) -> dd_host {
    double hi = (double)x;
    double lo = (double)(x - (long double)hi);
    return {hi, lo};
  };
  for (uint32_t j = 0; j < M; ++j) {
    long double ang = PI * (long double)j / (long double)N;
    dd_host c = split(cosl(ang)), s = split(sinl(ang));
    zeta[j] = {{c.hi, c.lo}, {s.hi, s.lo}};
  }
  for (uint32_t t = 0; t < M / 2; ++t) {
    long double ang = -2.0L * PI * (long double)t / (long double)M;
    dd_host c = split(cosl(ang)), s = split(sinl(ang));
    tw[t] = {{c.hi, c.lo}, {s.hi, s.lo}};
  }
}
// square roots s_f = exp(i pi (1 - 4 f) / 2048) of the N = 1024 evaluation points, f < 512 (P2_PM)
static void make_sroots(std::vector<ddc>& sr) {
  const long double PI = 3.14159265358979323846264338327950288L;
  sr.resize(512);
  for (uint32_t f = 0; f < 512; ++f) {
    const long double ang = PI * (1.0L - 4.0L * (long double)f) / 2048.0L;
    const long double c = cosl(ang), s = sinl(ang);
    const double ch = (double)c, sh = (double)s;
    sr[f] = {{ch, (double)(c - (long double)ch)}, {sh, (double)(s - (long double)sh)}};
  }
}

int convert_bsk_launch(const ConvertArgs& a) {
  if (key_format(a.k, a.N, a.level).kind == KeyKind::GENERIC) return convert_bsk_generic_launch(a);
  const bool n1024 = a.N == 1024 && a.k == 1 && a.limbs == 3 && a.level >= 1 && a.level <= 3;
  const bool n2048 =
      a.N == 2048 && a.k == 1 && a.limbs == (uint32_t)PBS2_LIMBS && a.level >= 1 && a.level <= PBS2_MAX_LEVEL;
  const bool k2 = a.N == 1024 && a.k == 2 && a.limbs == (uint32_t)K2_LIMBS && a.level >= 1 && a.level <= 64;
  const bool small = pbs_small_shape(a.k, a.N, a.level) && a.limbs == small_limbs(a.k, a.N, a.level);
  if (!n1024 && !n2048 && !k2 && !small) {
    set_error("unsupported BSK conversion parameters: N=%u k=%u level=%u limbs=%u", a.N, a.k, a.level, a.limbs);
    return -2;
  }
  std::vector<ddc> zeta, tw;
  make_tables(small ? a.N : 1024, zeta, tw);  // the others transform N = 1024 negacyclic polynomials
  ddc *dz = nullptr, *dt = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync((void**)&dz, zeta.size() * sizeof(ddc), a.stream));
  CHIP_CHECK(hipMallocAsync((void**)&dt, tw.size() * sizeof(ddc), a.stream));
  CHIP_CHECK(hipMemcpyAsync(dz, zeta.data(), zeta.size() * sizeof(ddc), hipMemcpyHostToDevice, a.stream));
  CHIP_CHECK(hipMemcpyAsync(dt, tw.data(), tw.size() * sizeof(ddc), hipMemcpyHostToDevice, a.stream));
  int rc = 0;
  std::vector<ddc> sr;
  ddc* ds = nullptr;
  if (n2048) {
    make_sroots(sr);
    CHIP_CHECK(hipMallocAsync((void**)&ds, sr.size() * sizeof(ddc), a.stream));
    CHIP_CHECK(hipMemcpyAsync(ds, sr.data(), sr.size() * sizeof(ddc), hipMemcpyHostToDevice, a.stream));
    const uint64_t blocks = (uint64_t)a.n * PBS2_LIMBS * 4 * a.level * (P2_PM ? 1 : 2);
    hipLaunchKernelGGL((convert_bsk2048_kernel<PBS2_LIMBS>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                       reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, ds, a.level, a.smax);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("convert launch failed: %s", hipGetErrorString(e));
      rc = -1;
    }
  } else if (small) {
    const uint64_t blocks = (uint64_t)a.n * a.limbs * (a.k + 1) * (a.k + 1) * a.level;
    if (a.N == 512 && a.k == 3)
      hipLaunchKernelGGL((convert_bsk_small_kernel<512, 4>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                         reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    else if (a.N == 512 && a.limbs == K4_L2_LIMBS)
      hipLaunchKernelGGL((convert_bsk_small_kernel<512, 5, K4_L2_LIMBS>), dim3((uint32_t)blocks), dim3(256), 0,
                         a.stream, reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    else if (a.N == 512)
      hipLaunchKernelGGL((convert_bsk_small_kernel<512, 5>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                         reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    else if (a.k == 5)
      hipLaunchKernelGGL((convert_bsk_small_kernel<256, 6>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                         reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    else
      hipLaunchKernelGGL((convert_bsk_small_kernel<256, 7>), dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                         reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("convert launch failed: %s", hipGetErrorString(e));
      rc = -1;
    }
  } else if (k2) {
    const uint64_t blocks = (uint64_t)a.n * K2_LIMBS * 9 * a.level;
    hipLaunchKernelGGL(convert_bsk1024k2_kernel, dim3((uint32_t)blocks), dim3(256), 0, a.stream,
                       reinterpret_cast<cplx*>(a.dest), a.src_dev, dz, dt, a.level, a.smax);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("convert launch failed: %s", hipGetErrorString(e));
      rc = -1;
    }
  } else switch (a.level) {
    case 1: rc = launch_convert<1024, 1, 1, 3>(a, dz, dt); break;
    case 2: rc = launch_convert<1024, 1, 2, 3>(a, dz, dt); break;
    default: rc = launch_convert<1024, 1, 3, 3>(a, dz, dt); break;
  }
  // the host tables must outlive the async copies: synchronise before they go out of scope
  CHIP_CHECK(hipStreamSynchronize(a.stream));
  CHIP_CHECK(hipFreeAsync(dz, a.stream));
  CHIP_CHECK(hipFreeAsync(dt, a.stream));
  if (ds) CHIP_CHECK(hipFreeAsync(ds, a.stream));
  return rc;
}

}  // namespace chip
