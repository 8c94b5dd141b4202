/*
 * tfhe_oracle.c — CPU restatement of the reference PBS/KS path (TEST INFRASTRUCTURE ONLY).
 * See tfhe_oracle.h for provenance.  Every function cites the reference file:line (or the
 * tfhe 0.10 routine, un-vendored: backends/concrete-cpu/implementation/Cargo.lock:867-870)
 * whose behaviour it restates.
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================================
 * PRNG: splitmix64 + xoshiro256**.  Deterministic synthetic inputs (the reference uses
 * concrete-csprng; bit-compatibility with it is neither possible nor needed: SURVEY §2.2).
 * ====================================================================================== */
static uint64_t splitmix64(uint64_t *x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
void ora_rng_seed(ora_rng *r, uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&x);
    r->has_spare = 0;
    r->spare = 0.0;
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
uint64_t ora_rng_u64(ora_rng *r) {
    uint64_t *s = r->s;
    uint64_t result = rotl(s[1] * 5, 7) * 9;
    uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
}
double ora_rng_gauss(ora_rng *r) {
    if (r->has_spare) {
        r->has_spare = 0;
        return r->spare;
    }
    double u1, u2;
    do {
        u1 = (double)(ora_rng_u64(r) >> 11) * 0x1.0p-53;
    } while (u1 <= 0.0);
    u2 = (double)(ora_rng_u64(r) >> 11) * 0x1.0p-53;
    double rad = sqrt(-2.0 * log(u1));
    r->spare = rad * sin(2.0 * M_PI * u2);
    r->has_spare = 1;
    return rad * cos(2.0 * M_PI * u2);
}
uint64_t ora_gauss_torus(ora_rng *r, double std_torus) {
    double v = ora_rng_gauss(r) * std_torus * 0x1.0p64;
    return (uint64_t)(int64_t)llround(v);
}

/* 128-bit curve (tools/parameter-curves/concrete-security-curves-cpp/include/concrete/curves.gen.h:2;
 * rust security_weights.rs secure_log2_std: max(slope*size + bias, 2 - logQ)). */
double ora_secure_log2_std(uint64_t glwe_dim, uint64_t poly_size) {
    double size = (double)(glwe_dim * poly_size);
    double v = -0.025696778711484593 * size + 2.675931372549016;
    return v > -62.0 ? v : -62.0;
}

/* ======================================================================================
 * sizes (concrete-cpu c_api/secret_key.rs:343-357, bootstrap.rs:417-429, keyswitch.rs:226-236)
 * ====================================================================================== */
size_t ora_lwe_size(size_t n) { return n + 1; }
size_t ora_glwe_size(size_t k, size_t N) { return (k + 1) * N; }
size_t ora_ggsw_size(size_t k, size_t N, size_t l) { return l * (k + 1) * (k + 1) * N; }
size_t ora_bsk_size(size_t n, size_t k, size_t N, size_t l) { return n * ora_ggsw_size(k, N, l); }
size_t ora_ksk_size(size_t n_in, size_t n_out, size_t l) { return n_in * l * (n_out + 1); }

/* ======================================================================================
 * negacyclic ring products over Z_{2^64}[X]/(X^N+1)
 * ====================================================================================== */
/* out += a*b, full (acyclic) product of length 2n-1 accumulated into out[0..2n-2] */
static void poly_mul_school_full(uint64_t *out, const uint64_t *a, const uint64_t *b, size_t n) {
    for (size_t i = 0; i < n; i++) {
        uint64_t ai = a[i];
        if (!ai) continue;
        for (size_t j = 0; j < n; j++) out[i + j] += ai * b[j];
    }
}
/* Karatsuba, exact over the ring Z_{2^64} (wrapping arithmetic is a commutative ring).
 * out[0..2n-2] = a*b (overwritten).  scratch >= 6n words. */
static void kara_full(uint64_t *out, const uint64_t *a, const uint64_t *b, size_t n, uint64_t *scratch) {
    if (n <= 32 || (n & 1)) {
        memset(out, 0, (2 * n - 1) * sizeof(uint64_t));
        poly_mul_school_full(out, a, b, n);
        return;
    }
    size_t h = n / 2;
    uint64_t *sa = scratch, *sb = scratch + h, *mid = scratch + 2 * h, *rest = scratch + 4 * h;
    /* out[0..2h-2] = a0*b0 ; out[2h..4h-2] = a1*b1 */
    kara_full(out, a, b, h, rest);
    kara_full(out + 2 * h, a + h, b + h, h, rest);
    out[2 * h - 1] = 0;
    for (size_t i = 0; i < h; i++) {
        sa[i] = a[i] + a[i + h];
        sb[i] = b[i] + b[i + h];
    }
    kara_full(mid, sa, sb, h, rest);
    for (size_t i = 0; i < 2 * h - 1; i++) mid[i] -= out[i] + out[2 * h + i];
    for (size_t i = 0; i < 2 * h - 1; i++) out[h + i] += mid[i];
}
static void negacyclic_u64_acc(uint64_t *acc, const uint64_t *a, const uint64_t *b, size_t N, int sub) {
    uint64_t *full = (uint64_t *)malloc((2 * N) * sizeof(uint64_t));
    uint64_t *scratch = (uint64_t *)malloc((8 * N + 64) * sizeof(uint64_t));
    kara_full(full, a, b, N, scratch);
    full[2 * N - 1] = 0;
    for (size_t j = 0; j < N; j++) {
        uint64_t v = full[j] - full[j + N]; /* X^N = -1 */
        acc[j] = sub ? acc[j] - v : acc[j] + v;
    }
    free(full);
    free(scratch);
}
void ora_polymul_acc_schoolbook(uint64_t *out, const int64_t *d, const uint64_t *g, size_t N) {
    /* definition: (d*g)_j = sum_{m<=j} d_m g_{j-m} - sum_{m>j} d_m g_{N+j-m} */
    for (size_t m = 0; m < N; m++) {
        uint64_t dm = (uint64_t)d[m];
        if (!dm) continue;
        for (size_t j = 0; j < N; j++) {
            if (j >= m) out[j] += dm * g[j - m];
            else out[j] -= dm * g[N + j - m];
        }
    }
}
void ora_polymul_acc_karatsuba(uint64_t *out, const int64_t *d, const uint64_t *g, size_t N) {
    uint64_t *du = (uint64_t *)malloc(N * sizeof(uint64_t));
    for (size_t i = 0; i < N; i++) du[i] = (uint64_t)d[i];
    negacyclic_u64_acc(out, du, g, N, 0);
    free(du);
}

/* ======================================================================================
 * keys / encryption (tfhe 0.10 encrypt_lwe_ciphertext, encrypt_glwe_ciphertext_assign,
 * encrypt_constant_ggsw_ciphertext; concrete-cpu c_api/secret_key.rs:29-179,
 * bootstrap.rs:18-88)
 * ====================================================================================== */
void ora_binary_key(uint64_t *sk, size_t len, ora_rng *r) {
    for (size_t i = 0; i < len; i++) sk[i] = ora_rng_u64(r) >> 63;
}
void ora_lwe_encrypt(const uint64_t *sk, uint64_t *ct, uint64_t pt, size_t n, double std_torus, ora_rng *r) {
    uint64_t b = pt + ora_gauss_torus(r, std_torus);
    for (size_t i = 0; i < n; i++) {
        ct[i] = ora_rng_u64(r);
        b += ct[i] * sk[i];
    }
    ct[n] = b;
}
/* secret_key.rs:155-179 -> decrypt_lwe_ciphertext: b - <a, s> */
uint64_t ora_lwe_decrypt(const uint64_t *sk, const uint64_t *ct, size_t n) {
    uint64_t acc = ct[n];
    for (size_t i = 0; i < n; i++) acc -= ct[i] * sk[i];
    return acc;
}
void ora_glwe_encrypt_assign(const uint64_t *glwe_sk, uint64_t *ct, size_t k, size_t N, double std_torus,
                             ora_rng *r) {
    uint64_t *body = ct + k * N;
    for (size_t p = 0; p < k; p++)
        for (size_t j = 0; j < N; j++) ct[p * N + j] = ora_rng_u64(r);
    for (size_t j = 0; j < N; j++) body[j] += ora_gauss_torus(r, std_torus);
    for (size_t p = 0; p < k; p++) negacyclic_u64_acc(body, ct + p * N, glwe_sk + p * N, N, 0);
}
void ora_glwe_decrypt(const uint64_t *glwe_sk, const uint64_t *ct, uint64_t *out, size_t k, size_t N) {
    memcpy(out, ct + k * N, N * sizeof(uint64_t));
    for (size_t p = 0; p < k; p++) negacyclic_u64_acc(out, ct + p * N, glwe_sk + p * N, N, 1);
}
/* GGSW(m): level matrix index v (decomposition level j = v+1, stored level 1 first);
 * factor = (-m) * 2^(64 - logB*j); row r<k: body = S_r * factor; last row: body[0] = -factor. */
void ora_ggsw_encrypt(const uint64_t *glwe_sk, uint64_t *ggsw, uint64_t cleartext, size_t k, size_t N,
                      size_t l, size_t logB, double std_torus, ora_rng *r) {
    size_t glwe_sz = (k + 1) * N;
    for (size_t v = 0; v < l; v++) {
        size_t j = v + 1;
        uint64_t factor = (0 - cleartext) * ((uint64_t)1 << (64 - logB * j));
        for (size_t row = 0; row <= k; row++) {
            uint64_t *ct = ggsw + (v * (k + 1) + row) * glwe_sz;
            uint64_t *body = ct + k * N;
            if (row < k) {
                for (size_t t = 0; t < N; t++) body[t] = glwe_sk[row * N + t] * factor;
            } else {
                memset(body, 0, N * sizeof(uint64_t));
                body[0] = 0 - factor;
            }
            ora_glwe_encrypt_assign(glwe_sk, ct, k, N, std_torus, r);
        }
    }
}
void ora_bsk_generate(uint64_t *bsk, const uint64_t *lwe_sk, const uint64_t *glwe_sk, size_t n, size_t k,
                      size_t N, size_t l, size_t logB, double std_torus, uint64_t seed) {
    size_t gs = ora_ggsw_size(k, N, l);
#pragma omp parallel for schedule(dynamic, 1)
    for (long i = 0; i < (long)n; i++) {
        ora_rng r;
        ora_rng_seed(&r, seed ^ (0x5bd1e995ULL * (uint64_t)(i + 1)));
        ora_ggsw_encrypt(glwe_sk, bsk + (size_t)i * gs, lwe_sk[i], k, N, l, logB, std_torus, &r);
    }
}
/* generate_lwe_keyswitch_key: block i stores levels reversed (storage index t <-> level l - t),
 * message = s_in[i] * 2^(64 - logB*level). */
void ora_ksk_generate(uint64_t *ksk, const uint64_t *sk_in, const uint64_t *sk_out, size_t n_in,
                      size_t n_out, size_t l, size_t logB, double std_torus, uint64_t seed) {
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)n_in; i++) {
        ora_rng r;
        ora_rng_seed(&r, seed ^ (0x7feb352dULL * (uint64_t)(i + 1)));
        for (size_t t = 0; t < l; t++) {
            size_t level = l - t;
            uint64_t msg = sk_in[i] * ((uint64_t)1 << (64 - logB * level));
            ora_lwe_encrypt(sk_out, ksk + ((size_t)i * l + t) * (n_out + 1), msg, n_out, std_torus, &r);
        }
    }
}

/* ======================================================================================
 * primitives (tfhe 0.10 commons/math/decomposition, polynomial_algorithms, modulus_switch)
 * ====================================================================================== */
/* SignedDecomposer::init_decomposer_state: round to the top l*logB bits (half up), shifted down */
uint64_t ora_decomp_init_state(uint64_t x, size_t l, size_t logB) {
    size_t nrep = 64 - l * logB;
    if (nrep == 0) return x;
    uint64_t msb = (x >> (nrep - 1)) & 1;
    return (x >> nrep) + msb;
}
/* decompose_one_level: balanced digit with carry ((res-1) | state) & res >> (logB-1) */
uint64_t ora_decomp_one_level(uint64_t *state, size_t logB) {
    uint64_t mask = ((uint64_t)1 << logB) - 1;
    uint64_t res = *state & mask;
    *state >>= logB;
    uint64_t carry = ((res - 1) | *state) & res;
    carry >>= logB - 1;
    *state += carry;
    return res - (carry << logB);
}
void ora_decompose(uint64_t x, size_t l, size_t logB, int64_t *digits) {
    uint64_t st = ora_decomp_init_state(x, l, logB);
    for (size_t q = 0; q < l; q++) digits[q] = (int64_t)ora_decomp_one_level(&st, logB);
}
/* pbs_modulus_switch == simulation.cpp:64-75: round(x * 2N / 2^64) mod 2N (half up) */
size_t ora_modswitch(uint64_t x, size_t N) {
    unsigned log2n2 = 0;
    while (((size_t)1 << log2n2) < 2 * N) log2n2++;
    uint64_t y = x + ((uint64_t)1 << (64 - log2n2 - 1));
    return (size_t)(y >> (64 - log2n2));
}
/* out[j] = coefficient j of in * X^d, d in [0, 2N) */
void ora_monomial_mul(uint64_t *out, const uint64_t *in, size_t d, size_t N) {
    d %= 2 * N;
    for (size_t j = 0; j < N; j++) {
        size_t t = (j + 2 * N - d) % (2 * N); /* source index in the 2N-periodic sign-extended sequence */
        out[j] = t < N ? in[t] : 0 - in[t - N];
    }
}
void ora_monomial_div(uint64_t *out, const uint64_t *in, size_t d, size_t N) {
    ora_monomial_mul(out, in, (2 * N - (d % (2 * N))) % (2 * N), N);
}
/* extract_lwe_sample_from_glwe_ciphertext(.., MonomialDegree(0)) */
void ora_sample_extract(uint64_t *lwe_out, const uint64_t *glwe, size_t k, size_t N) {
    for (size_t r = 0; r < k; r++) {
        const uint64_t *a = glwe + r * N;
        lwe_out[r * N] = a[0];
        for (size_t j = 1; j < N; j++) lwe_out[r * N + j] = 0 - a[N - j];
    }
    lwe_out[k * N] = glwe[k * N];
}

/* ======================================================================================
 * limb-split negacyclic FFT (exact by certified rounding)
 *   z_j = (p_j + i p_{j+M}) * zeta^j, zeta = exp(i pi / N), M = N/2
 *   Z_m = sum_j z_j exp(-2 pi i j m / M)    (natural order here; the GPU uses its own order)
 * ====================================================================================== */
void ora_limb_widths(size_t L, int *w) {
    int base = (int)(64 / L), extra = (int)(64 % L);
    for (size_t i = 0; i < L; i++) w[i] = base + ((int)i < extra ? 1 : 0);
}
void ora_limb_split(uint64_t g, size_t L, int64_t *limbs) {
    int w[16];
    if (L == 1) { /* one 64-bit limb: the signed value (fft64's u64 -> i64 reading) */
        limbs[0] = (int64_t)g;
        return;
    }
    ora_limb_widths(L, w);
    uint64_t rem = g;
    for (size_t i = 0; i < L; i++) {
        uint64_t mask = ((uint64_t)1 << w[i]) - 1;
        uint64_t v = rem & mask;
        int64_t s = (v >= ((uint64_t)1 << (w[i] - 1))) ? (int64_t)v - ((int64_t)1 << w[i]) : (int64_t)v;
        limbs[i] = s;
        rem = (rem - (uint64_t)s) >> w[i];
    }
}

typedef struct { long double re, im; } cld;

/* extended-precision FFT used only for the one-time key transform; tw[t] = exp(-2 pi i t / M) */
static void fft_ld(cld *x, size_t M, const cld *tw) {
    for (size_t i = 1, j = 0; i < M; i++) {
        size_t bit = M >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { cld t = x[i]; x[i] = x[j]; x[j] = t; }
    }
    for (size_t len = 2; len <= M; len <<= 1) {
        size_t stride = M / len;
        for (size_t i = 0; i < M; i += len) {
            for (size_t t = 0; t < len / 2; t++) {
                long double wr = tw[t * stride].re, wi = tw[t * stride].im;
                cld u = x[i + t], v = x[i + t + len / 2];
                cld vw = {v.re * wr - v.im * wi, v.re * wi + v.im * wr};
                x[i + t].re = u.re + vw.re;
                x[i + t].im = u.im + vw.im;
                x[i + t + len / 2].re = u.re - vw.re;
                x[i + t + len / 2].im = u.im - vw.im;
            }
        }
    }
}

/* double-precision runtime FFT plan with correctly rounded twiddles */
typedef struct {
    size_t N, M, logM;
    double *tw_re, *tw_im;     /* per stage twiddles, concatenated */
    double *zeta_re, *zeta_im; /* zeta^j, j < M */
    size_t *rev;
} fft_plan;

static fft_plan *plan_cache[32];

static fft_plan *get_plan(size_t N) {
    size_t lg = 0;
    while (((size_t)1 << lg) < N) lg++;
    fft_plan *p;
#pragma omp critical(ora_plan)
    {
        p = plan_cache[lg];
        if (!p) {
            p = (fft_plan *)calloc(1, sizeof(fft_plan));
            p->N = N;
            p->M = N / 2;
            p->logM = lg - 1;
            size_t M = p->M;
            p->tw_re = (double *)malloc(M * sizeof(double));
            p->tw_im = (double *)malloc(M * sizeof(double));
            /* stage len: twiddles exp(-2 pi i t / len), t < len/2, stored at offset len/2 - 1 */
            for (size_t len = 2; len <= M; len <<= 1)
                for (size_t t = 0; t < len / 2; t++) {
                    long double ang = -2.0L * 3.14159265358979323846264338327950288L * (long double)t / (long double)len;
                    p->tw_re[len / 2 - 1 + t] = (double)cosl(ang);
                    p->tw_im[len / 2 - 1 + t] = (double)sinl(ang);
                }
            p->zeta_re = (double *)malloc(M * sizeof(double));
            p->zeta_im = (double *)malloc(M * sizeof(double));
            for (size_t j = 0; j < M; j++) {
                long double ang = 3.14159265358979323846264338327950288L * (long double)j / (long double)N;
                p->zeta_re[j] = (double)cosl(ang);
                p->zeta_im[j] = (double)sinl(ang);
            }
            p->rev = (size_t *)malloc(M * sizeof(size_t));
            for (size_t i = 0; i < M; i++) {
                size_t r = 0;
                for (size_t b = 0; b < p->logM; b++)
                    if (i & ((size_t)1 << b)) r |= (size_t)1 << (p->logM - 1 - b);
                p->rev[i] = r;
            }
            plan_cache[lg] = p;
        }
    }
    return p;
}

/* in-place radix-2 FFT on split re/im arrays; inverse uses conjugate twiddles, unnormalized */
static void fft_d(const fft_plan *p, double *re, double *im, int inverse) {
    size_t M = p->M;
    for (size_t i = 0; i < M; i++) {
        size_t j = p->rev[i];
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    for (size_t len = 2; len <= M; len <<= 1) {
        size_t h = len / 2;
        const double *wr = p->tw_re + h - 1, *wi = p->tw_im + h - 1;
        for (size_t i = 0; i < M; i += len) {
            for (size_t t = 0; t < h; t++) {
                double cr = wr[t], ci = inverse ? -wi[t] : wi[t];
                double vr = re[i + t + h], vi = im[i + t + h];
                double xr = vr * cr - vi * ci, xi = vr * ci + vi * cr;
                double ur = re[i + t], ui = im[i + t];
                re[i + t] = ur + xr;
                im[i + t] = ui + xi;
                re[i + t + h] = ur - xr;
                im[i + t + h] = ui - xi;
            }
        }
    }
}

size_t ora_fourier_bsk_len(size_t n, size_t k, size_t N, size_t l, size_t L) {
    return n * l * (k + 1) * (k + 1) * L * N; /* M complex = N doubles per (poly, limb) */
}

/* fbsk layout (oracle-private): [i][v][row][col][limb][re(M) | im(M)], scaled by 1/M */
void ora_bsk_to_fourier(double *fbsk, const uint64_t *bsk, size_t n, size_t k, size_t N, size_t l, size_t L) {
    size_t M = N / 2;
    size_t npoly = n * l * (k + 1) * (k + 1);
    const long double PI = 3.14159265358979323846264338327950288L;
    cld *tw = (cld *)malloc(M * sizeof(cld)), *zeta = (cld *)malloc(M * sizeof(cld));
    for (size_t t = 0; t < M; t++) {
        tw[t].re = cosl(-2.0L * PI * (long double)t / (long double)M);
        tw[t].im = sinl(-2.0L * PI * (long double)t / (long double)M);
        zeta[t].re = cosl(PI * (long double)t / (long double)N);
        zeta[t].im = sinl(PI * (long double)t / (long double)N);
    }
#pragma omp parallel
    {
        cld *buf = (cld *)malloc(M * sizeof(cld));
        int64_t *limbs = (int64_t *)malloc(N * L * sizeof(int64_t));
#pragma omp for schedule(static)
        for (long pi = 0; pi < (long)npoly; pi++) {
            const uint64_t *g = bsk + (size_t)pi * N;
            for (size_t j = 0; j < N; j++) ora_limb_split(g[j], L, limbs + j * L);
            for (size_t li = 0; li < L; li++) {
                for (size_t j = 0; j < M; j++) {
                    long double a = (long double)limbs[j * L + li], b = (long double)limbs[(j + M) * L + li];
                    long double zr = zeta[j].re, zi = zeta[j].im;
                    buf[j].re = a * zr - b * zi;
                    buf[j].im = a * zi + b * zr;
                }
                fft_ld(buf, M, tw);
                double *dst = fbsk + ((size_t)pi * L + li) * N;
                for (size_t m = 0; m < M; m++) {
                    dst[m] = (double)(buf[m].re / (long double)M);
                    dst[M + m] = (double)(buf[m].im / (long double)M);
                }
            }
        }
        free(buf);
        free(limbs);
    }
    free(tw);
    free(zeta);
}

/* Certified bound: |err| <= sum_rows ||d||_2 * max|G| * (2*gamma + 2u) + tail,
 * gamma = log2(M) * (u + 4u(sqrt2 + u)) / (1 - ...) (Higham, Accuracy & Stability, Thm 24.2).
 * ||d||_2 <= sqrt(N) * 2^(logB-1) per digit polynomial; (k+1)*l digit polynomials per output.
 * max|G| is measured on this key (stored values are scaled by 1/M: rescale). */
double ora_fft_error_bound(const double *fbsk, size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L) {
    size_t M = N / 2;
    double u = 0x1.0p-53;
    double logM = log2((double)M);
    double eta = u + 4.0 * u / (1.0 - 4.0 * u) * (sqrt(2.0) + u);
    double gamma = logM * eta / (1.0 - logM * eta);
    double maxG = 0.0;
    size_t total = ora_fourier_bsk_len(n, k, N, l, L) / N; /* (poly, limb) blocks */
    for (size_t b = 0; b < total; b++) {
        const double *src = fbsk + b * N;
        for (size_t m = 0; m < M; m++) {
            double a = hypot(src[m], src[M + m]) * (double)M;
            if (a > maxG) maxG = a;
        }
    }
    double dnorm = sqrt((double)N) * ldexp(1.0, (int)logB - 1);
    double rows = (double)((k + 1) * l);
    int w[16];
    ora_limb_widths(L, w);
    /* forward-FFT error of each digit transform, product rounding, inverse-FFT error,
     * key-transform rounding (u * |G|, computed in extended precision), plus the final
     * untwist rounding relative to the largest possible output magnitude.  The radix-8
     * GPU transform is covered by doubling gamma. */
    double max_out = rows * (double)N * ldexp(1.0, (int)logB - 1) * ldexp(1.0, w[0] - 1);
    return rows * dnorm * maxG * (4.0 * gamma + 3.0 * u) * 1.0001 + 4.0 * u * max_out;
}

/* an integer-valued double of any magnitude, reduced mod 2^64 (exact: x - q 2^64 is a multiple of
 * x's ulp and lies in [0, 2^64)) */
static inline uint64_t wrap_u64(double x) {
    double q = floor(ldexp(x, -64));
    double r = x - ldexp(q, 64);
    if (r >= 0x1p63) r -= 0x1p64;
    return (uint64_t)(int64_t)r;
}

/* ======================================================================================
 * external product / CMUX / blind rotate / PBS (tfhe 0.10 fft64 add_external_product_assign,
 * blind_rotate_assign, programmable_bootstrap_lwe_ciphertext_mem_optimized; call site
 * concrete-cpu c_api/bootstrap.rs:405)
 * ====================================================================================== */
void ora_external_product_acc(uint64_t *acc, const uint64_t *ggsw_std, const double *ggsw_fourier,
                              const uint64_t *ct1, size_t k, size_t N, size_t l, size_t logB, size_t L,
                              int mode, double *max_resid) {
    size_t K1 = k + 1;
    /* digits[row][q][j], q = 0 is decomposition level l (least significant) */
    int64_t *digits = (int64_t *)malloc(K1 * l * N * sizeof(int64_t));
    int64_t tmp[64];
    for (size_t row = 0; row < K1; row++)
        for (size_t j = 0; j < N; j++) {
            ora_decompose(ct1[row * N + j], l, logB, tmp);
            for (size_t q = 0; q < l; q++) digits[(row * l + q) * N + j] = tmp[q];
        }
    if (mode == ORA_MODE_SCHOOLBOOK || mode == ORA_MODE_KARATSUBA) {
        /* the K1 l K1 products (row, level, col) are independent: outside a parallel region (one
         * large-N ciphertext, ora_pbs_batch) they run on the OpenMP threads into private buffers, summed
         * per column afterwards in a fixed order (integer adds mod 2^64: the same bits either way) */
        size_t T = K1 * l * K1;
        int inner = 0;
#ifdef _OPENMP
        inner = !omp_in_parallel() && omp_get_max_threads() > 1 && T > 1 && N >= 2048;
#endif
        uint64_t *part = inner ? (uint64_t *)calloc(T * N, sizeof(uint64_t)) : NULL;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) if (inner)
#endif
        for (long t = 0; t < (long)T; t++) {
            size_t row = (size_t)t / (l * K1), q = ((size_t)t / K1) % l, col = (size_t)t % K1;
            size_t v = l - 1 - q; /* GGSW level matrix index of decomposition level l - q */
            const uint64_t *g = ggsw_std + ((v * K1 + row) * K1 + col) * N;
            uint64_t *dst = inner ? part + (size_t)t * N : acc + col * N;
            if (mode == ORA_MODE_SCHOOLBOOK)
                ora_polymul_acc_schoolbook(dst, digits + (row * l + q) * N, g, N);
            else
                ora_polymul_acc_karatsuba(dst, digits + (row * l + q) * N, g, N);
        }
        if (inner) {
            for (size_t t = 0; t < T; t++) {
                uint64_t *dst = acc + (t % K1) * N;
                const uint64_t *src = part + t * N;
                for (size_t j = 0; j < N; j++) dst[j] += src[j];
            }
            free(part);
        }
        free(digits);
        return;
    }
    /* limb FFT path */
    const fft_plan *p = get_plan(N);
    size_t M = N / 2;
    int w[16];
    ora_limb_widths(L, w);
    double *X = (double *)malloc(K1 * l * N * sizeof(double)); /* [row*l+q][re M | im M] */
    double *Y = (double *)malloc(N * sizeof(double));
    for (size_t rq = 0; rq < K1 * l; rq++) {
        double *re = X + rq * N, *im = re + M;
        const int64_t *d = digits + rq * N;
        for (size_t j = 0; j < M; j++) {
            double a = (double)d[j], b = (double)d[j + M];
            re[j] = a * p->zeta_re[j] - b * p->zeta_im[j];
            im[j] = a * p->zeta_im[j] + b * p->zeta_re[j];
        }
        fft_d(p, re, im, 0);
    }
    for (size_t col = 0; col < K1; col++) {
        for (size_t li = 0; li < L; li++) {
            double *yr = Y, *yi = Y + M;
            memset(Y, 0, N * sizeof(double));
            for (size_t row = 0; row < K1; row++)
                for (size_t q = 0; q < l; q++) {
                    size_t v = l - 1 - q;
                    const double *G = ggsw_fourier + ((((v * K1 + row) * K1 + col) * L) + li) * N;
                    const double *xr = X + (row * l + q) * N, *xi = xr + M;
                    for (size_t m = 0; m < M; m++) {
                        yr[m] += xr[m] * G[m] - xi[m] * G[M + m];
                        yi[m] += xr[m] * G[M + m] + xi[m] * G[m];
                    }
                }
            fft_d(p, yr, yi, 1);
            int shift = 0;
            for (size_t t = 0; t < li; t++) shift += w[t];
            for (size_t j = 0; j < M; j++) {
                /* untwist: multiply by conj(zeta^j) */
                double zr = p->zeta_re[j], zi = p->zeta_im[j];
                double cr = yr[j] * zr + yi[j] * zi;
                double ci = yi[j] * zr - yr[j] * zi;
                double rr = nearbyint(cr), ri = nearbyint(ci);
                if (mode == ORA_MODE_FFT64) {
                    /* one 64-bit key limb (concrete-cpu's fft64): the products exceed 2^53, so the
                     * low bits carry f64 rounding noise; the rounded value is reduced mod 2^64 */
                    acc[col * N + j] += wrap_u64(rr);
                    acc[col * N + j + M] += wrap_u64(ri);
                    continue;
                }
                if (max_resid) {
                    double e1 = fabs(cr - rr), e2 = fabs(ci - ri);
                    if (e1 > *max_resid) *max_resid = e1;
                    if (e2 > *max_resid) *max_resid = e2;
                }
                acc[col * N + j] += ((uint64_t)(int64_t)rr) << shift;
                acc[col * N + j + M] += ((uint64_t)(int64_t)ri) << shift;
            }
        }
    }
    free(X);
    free(Y);
    free(digits);
}

void ora_blind_rotate(uint64_t *acc, const uint64_t *lwe_in, const uint64_t *bsk_std, const double *fbsk,
                      size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, int mode, double *max_resid) {
    size_t K1 = k + 1, gsz = (k + 1) * N;
    uint64_t *tmp = (uint64_t *)malloc(gsz * sizeof(uint64_t));
    uint64_t *ct1 = (uint64_t *)malloc(gsz * sizeof(uint64_t));
    /* acc <- acc * X^{-ms(b)} */
    size_t b_t = ora_modswitch(lwe_in[n], N);
    memcpy(tmp, acc, gsz * sizeof(uint64_t));
    for (size_t p = 0; p < K1; p++) ora_monomial_div(acc + p * N, tmp + p * N, b_t, N);
    size_t ggsw_len = ora_ggsw_size(k, N, l);
    size_t fggsw_len = l * K1 * K1 * L * N;
    for (size_t i = 0; i < n; i++) {
        if (lwe_in[i] == 0) continue; /* tfhe: skip on a zero mask element */
        size_t a_t = ora_modswitch(lwe_in[i], N);
        /* ct1 = acc * X^{a_t} - acc */
        for (size_t p = 0; p < K1; p++) {
            ora_monomial_mul(ct1 + p * N, acc + p * N, a_t, N);
            for (size_t j = 0; j < N; j++) ct1[p * N + j] -= acc[p * N + j];
        }
        ora_external_product_acc(acc, bsk_std ? bsk_std + i * ggsw_len : NULL, fbsk ? fbsk + i * fggsw_len : NULL,
                                 ct1, k, N, l, logB, L, mode, max_resid);
    }
    free(tmp);
    free(ct1);
}

void ora_pbs(uint64_t *lwe_out, const uint64_t *lwe_in, const uint64_t *accumulator, const uint64_t *bsk_std,
             const double *fbsk, size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, int mode,
             double *max_resid) {
    size_t gsz = (k + 1) * N;
    uint64_t *acc = (uint64_t *)malloc(gsz * sizeof(uint64_t));
    memcpy(acc, accumulator, gsz * sizeof(uint64_t));
    ora_blind_rotate(acc, lwe_in, bsk_std, fbsk, n, k, N, l, logB, L, mode, max_resid);
    ora_sample_extract(lwe_out, acc, k, N);
    free(acc);
}

void ora_pbs_batch(uint64_t *out, const uint64_t *out_idx, const uint64_t *luts, const uint64_t *lut_idx,
                   const uint64_t *in, const uint64_t *in_idx, const uint64_t *bsk_std, const double *fbsk,
                   size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, size_t num_samples, int mode,
                   int nthreads, double *max_resid) {
    double resid = 0.0;
    int outer = 1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    /* few large ciphertexts: one at a time, each external product's products in parallel instead */
    outer = (long)num_samples * 4 > (long)nthreads || N < 2048;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(max : resid) if (outer)
#endif
    for (long s = 0; s < (long)num_samples; s++) {
        size_t oi = out_idx ? (size_t)out_idx[s] : (size_t)s;
        size_t ii = in_idx ? (size_t)in_idx[s] : (size_t)s;
        size_t li = lut_idx ? (size_t)lut_idx[s] : 0;
        double r = 0.0;
        ora_pbs(out + oi * (k * N + 1), in + ii * (n + 1), luts + li * (k + 1) * N, bsk_std, fbsk, n, k, N, l,
                logB, L, mode, &r);
        if (r > resid) resid = r;
    }
    if (max_resid && resid > *max_resid) *max_resid = resid;
}

/* keyswitch_lwe_ciphertext (call: concrete-cpu c_api/keyswitch.rs:185-223):
 * out = (0,...,0,b) - sum_i sum_t d_{i,t} * KSK[i][t], digits yielded level l first. */
void ora_keyswitch(uint64_t *out, const uint64_t *in, const uint64_t *ksk, size_t l, size_t logB, size_t n_in,
                   size_t n_out) {
    memset(out, 0, (n_out + 1) * sizeof(uint64_t));
    out[n_out] = in[n_in];
    int64_t dig[64];
    for (size_t i = 0; i < n_in; i++) {
        ora_decompose(in[i], l, logB, dig);
        for (size_t t = 0; t < l; t++) {
            uint64_t d = (uint64_t)dig[t];
            if (!d) continue;
            const uint64_t *row = ksk + (i * l + t) * (n_out + 1);
            for (size_t j = 0; j <= n_out; j++) out[j] -= d * row[j];
        }
    }
}
void ora_keyswitch_batch(uint64_t *out, const uint64_t *out_idx, const uint64_t *in, const uint64_t *in_idx,
                         const uint64_t *ksk, size_t l, size_t logB, size_t n_in, size_t n_out,
                         size_t num_samples, int nthreads) {
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (long s = 0; s < (long)num_samples; s++) {
        size_t oi = out_idx ? (size_t)out_idx[s] : (size_t)s;
        size_t ii = in_idx ? (size_t)in_idx[s] : (size_t)s;
        ora_keyswitch(out + oi * (n_out + 1), in + ii * (n_in + 1), ksk, l, logB, n_in, n_out);
    }
}

/* ======================================================================================
 * encoding (compiler lib/Common/Transformers.cpp:364-427, lib/Runtime/wrappers.cpp:388-450,773-783)
 * ====================================================================================== */
uint64_t ora_encode_native(uint64_t m, uint32_t width) { return m << (64 - (width + 1)); }
uint64_t ora_decode_native(uint64_t x, uint32_t precision, int is_signed) {
    uint64_t output = x >> (64 - precision - 2);
    uint64_t carry = output % 2;
    uint64_t mod = ((uint64_t)1) << (precision + 1);
    output = ((output >> 1) + carry) % mod;
    if (is_signed) {
        uint64_t maxPos = ((uint64_t)1) << (precision - 1);
        if (output >= maxPos) output |= UINT64_MAX << precision;
    }
    return output;
}
void ora_encode_expand_lut(uint64_t *out, size_t out_size, const uint64_t *in, size_t in_size,
                           uint32_t out_message_bits, int is_signed) {
    size_t mega = out_size / in_size;
    size_t half = in_size / 2;
#define IDX(i) (is_signed ? ((i) < half ? (i) + half : (i) - half) : (i))
    for (size_t idx = 0; idx < mega / 2; ++idx) out[idx] = in[IDX(0)] << (64 - out_message_bits - 1);
    for (size_t idx = (in_size - 1) * mega + mega / 2; idx < out_size; ++idx)
        out[idx] = 0 - (in[IDX(0)] << (64 - out_message_bits - 1));
    for (size_t li = 1; li < in_size; ++li) {
        uint64_t v = in[IDX(li)] << (64 - out_message_bits - 1);
        size_t start = mega * (li - 1) + mega / 2;
        for (size_t o = start; o < start + mega; ++o) out[o] = v;
    }
#undef IDX
}
void ora_trivial_glwe_from_lut(uint64_t *glwe, const uint64_t *lut, size_t k, size_t N) {
    memset(glwe, 0, k * N * sizeof(uint64_t));
    memcpy(glwe + k * N, lut, N * sizeof(uint64_t));
}
