/*
 * wsmc_math.h — deterministic scalar math shared by the gfx950 kernels and the
 * CPU oracle (oracle/wsmc_oracle.c).
 *
 * Why this exists: the reference (WeightedSampling.jl) draws from Julia's global
 * Xoshiro/ziggurat RNG and calls libm / Distributions.jl (src/default_kernels.jl:12-23,
 * src/resampling.jl:40, src/move_kernels.jl:150,201,209). Neither can be reproduced
 * bit-for-bit on a GPU. The build therefore fixes ONE restatement of every random draw
 * and every transcendental, and compiles the same source for the host (gcc, for the
 * oracle) and for the device (hipcc, for the kernels). With FP contraction disabled
 * (-ffp-contract=off on both sides; explicit fma() only where written) and IEEE
 * correctly-rounded +,-,*,/,sqrt on both sides, every per-particle value is
 * bit-identical between the CPU oracle and the HIP path.
 *
 * Contents
 *   - Philox4x32-10 counter-based RNG (Salmon et al. 2011; Random123 constants)
 *   - uniforms / Box–Muller normals keyed by (seed, op, particle, draw)
 *   - exp / log / log1p / sin / cos restated from the fdlibm algorithms (Sun, 1993)
 *   - Normal / HalfNormal / Uniform / isotropic-MvNormal log-densities
 *     (Distributions.jl semantics used by src/default_kernels.jl:83-102 and
 *      examples/damped_oscillator.jl:24-28)
 *   - the integer (fixed-point) weight map used for order-independent CDFs and ESS
 *   - the stratified / systematic target map and its inverse rank() used by resampling
 *     (restates src/resampling.jl:13-43 on an integer CDF)
 *   - the bound transforms of autoRW/RW (src/move_kernels.jl:37-85)
 *
 * Valid C99 (gcc) and HIP C++ (hipcc). No libm calls.
 */
#ifndef WSMC_MATH_H
#define WSMC_MATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define WSMC_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define WSMC_HD static inline __attribute__((always_inline))
#endif
#if defined(__clang__)
#define WSMC_UNROLL _Pragma("unroll")
#else
#define WSMC_UNROLL _Pragma("GCC unroll 16")
#endif

typedef unsigned __int128 wsmc_u128;

/* WSMC_K(c): a polynomial coefficient. On the device it is held in a scalar register pair, so a
 * Horner step is one v_fma_f64 with an SGPR operand instead of two v_mov_b32 of the literal and a
 * v_fmac_f64 (the value and every rounding are the same; only where the constant lives differs). */
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline __attribute__((always_inline)) double wsmc_sreg(double c) {
    __asm__ volatile("" : "+s"(c));
    return c;
}
#define WSMC_K(c) wsmc_sreg(c)
#else
#define WSMC_K(c) (c)
#endif

/* ------------------------------------------------------------------------- */
/* bit casts                                                                  */
/* ------------------------------------------------------------------------- */
WSMC_HD uint64_t wsmc_d2bits(double x) { union { double d; uint64_t u; } v; v.d = x; return v.u; }
WSMC_HD double wsmc_bits2d(uint64_t u) { union { double d; uint64_t u; } v; v.u = u; return v.d; }

#define WSMC_INF (wsmc_bits2d(0x7ff0000000000000ULL))
#define WSMC_NAN (wsmc_bits2d(0x7ff8000000000000ULL))
#define WSMC_LOG2PI 1.8378770664093453     /* log(2*pi) rounded to double */
#include "wsmc_log_table.h"
#include "wsmc_exp_table.h"
#define WSMC_LOG2   0.69314718055994530942 /* log(2) */
#define WSMC_PI     3.14159265358979311600
#define WSMC_TWO_PI 6.28318530717958623200

WSMC_HD int wsmc_isnan(double x) { return x != x; }
WSMC_HD int wsmc_isfinite(double x) { return (wsmc_d2bits(x) & 0x7ff0000000000000ULL) != 0x7ff0000000000000ULL; }
WSMC_HD double wsmc_fabs(double x) { return wsmc_bits2d(wsmc_d2bits(x) & 0x7fffffffffffffffULL); }

/* 2^k for -1022 <= k <= 1023 */
WSMC_HD double wsmc_pow2i(int k) { return wsmc_bits2d((uint64_t)(k + 1023) << 52); }

/* exact u32 pieces -> one correctly rounded add: identical on gcc and hipcc */
WSMC_HD double wsmc_u64_to_d(uint64_t v) {
    return (double)(uint32_t)(v >> 32) * 4294967296.0 + (double)(uint32_t)v;
}
WSMC_HD double wsmc_u128_to_d(wsmc_u128 v) {
    return wsmc_u64_to_d((uint64_t)(v >> 64)) * 18446744073709551616.0 + wsmc_u64_to_d((uint64_t)v);
}

/* truncating f64 -> u64 for 0 <= x < 2^64 by bit manipulation (no cvt differences) */
WSMC_HD uint64_t wsmc_d_to_u64_trunc(double x) {
    uint64_t b = wsmc_d2bits(x);
    if (b >> 63) return 0;                       /* negative or -0 */
    int e = (int)((b >> 52) & 0x7ff);
    if (e < 1023) return 0;                      /* x < 1 (incl. subnormal, 0) */
    uint64_t m = (b & 0x000fffffffffffffULL) | 0x0010000000000000ULL;
    int sh = e - 1075;                           /* x = m * 2^sh */
    if (sh >= 0) return sh >= 12 ? 0xffffffffffffffffULL : (m << sh);
    return m >> (-sh);
}

/* floor for doubles: IEEE-exact on both compilers (v_floor_f64 / roundsd) */
WSMC_HD double wsmc_floor(double x) { return __builtin_floor(x); }

/* order-preserving u64 encoding of f64 (for atomicMax); NaN canonicalised to +NaN (max) */
WSMC_HD uint64_t wsmc_ord_enc(double x) {
    uint64_t b = wsmc_isnan(x) ? 0x7ff8000000000000ULL : wsmc_d2bits(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
WSMC_HD double wsmc_ord_dec(uint64_t e) {
    return wsmc_bits2d((e >> 63) ? (e & 0x7fffffffffffffffULL) : ~e);
}
#define WSMC_ORD_NEG_INF 0x000fffffffffffffULL   /* wsmc_ord_enc(-inf) */

/* ------------------------------------------------------------------------- */
/* Philox4x32-10                                                              */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t v[4]; } wsmc_u32x4;

WSMC_HD uint32_t wsmc_mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

WSMC_HD wsmc_u32x4 wsmc_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    /* each round's two 32x32 -> 64 products whole (one v_mad_u64_u32 each on the device,
       where separate high and low multiplies took two), rounds unrolled (the key schedule
       becomes scalar adds) */
    WSMC_UNROLL
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    wsmc_u32x4 o; o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
    return o;
}

/*
 * Stream layout (the build's replacement for Julia's global RNG, src/types.jl:24-26):
 *   key     = seed (64 bit)
 *   counter = { particle index lo32, (block << 8) | lane-tag, op lo32, op hi32 }
 * `op` is the context's monotonically increasing stochastic-statement counter, so a
 * fused multi-step runner and the same statements issued one by one draw identical
 * numbers. `block` selects the 128-bit block (2 uniforms / 2 normals) within an op.
 */
WSMC_HD wsmc_u32x4 wsmc_rng_block(uint64_t seed, uint64_t op, uint64_t idx, uint32_t block) {
    return wsmc_philox((uint32_t)idx, (uint32_t)(idx >> 32) ^ (block << 16),
                       (uint32_t)op, (uint32_t)(op >> 32),
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}

/* 53-bit uniform in [0,1) from two words */
WSMC_HD double wsmc_u01(uint32_t hi, uint32_t lo) {
    uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)(int64_t)x * 1.1102230246251565404e-16; /* 2^-53; x < 2^53 exactly representable */
}
/* 53-bit uniform in (0,1] */
WSMC_HD double wsmc_u01_open0(uint32_t hi, uint32_t lo) {
    uint64_t x = ((((uint64_t)hi << 32) | lo) >> 11) + 1;
    return (double)(int64_t)x * 1.1102230246251565404e-16;
}

/* ------------------------------------------------------------------------- */
/* exp and log (table-driven), log1p                                          */
/* ------------------------------------------------------------------------- */
WSMC_HD double wsmc_scalbn_small(double y, int k) {
    /* y in [0.5, 2), returns y * 2^k with a single rounding for normal results */
    if (k > 1023) return y * wsmc_pow2i(1023) * wsmc_pow2i(k - 1023);
    if (k < -1021) return (y * wsmc_pow2i(k + 1000)) * wsmc_pow2i(-1000);
    return y * wsmc_pow2i(k);
}

/* fdlibm's e_exp.c restated: wsmc_exp's path for |x| >= 512 and NaN */
WSMC_HD double wsmc_exp_fd(double x) {
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10,
                 invln2 = 1.44269504088896338700e+00,
                 P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    if (wsmc_isnan(x)) return x;
    if (x > 709.782712893383973096) return WSMC_INF;
    if (x < -745.13321910194110842) return 0.0;
    double ax = wsmc_fabs(x);
    if (ax < 3.725290298461914e-09) return 1.0 + x;  /* |x| < 2^-28 */
    int k; double hi, lo;
    if (ax < 0.34657359027997264) {                     /* |x| < 0.5 ln2 */
        k = 0; hi = x; lo = 0.0;
    } else {
        k = (int)(x * invln2 + (x < 0.0 ? -0.5 : 0.5));
        hi = x - (double)k * ln2hi;
        lo = (double)k * ln2lo;
    }
    double r = hi - lo;
    double z = r * r;
    double c = r - z * (P1 + z * (P2 + z * (P3 + z * (P4 + z * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    if (k == 0) return y;
    return wsmc_scalbn_small(y, k);
}
/* exp(x), table-driven (the approach of Julia's Base.exp and glibc's exp, restated with this
 * file's table: include/wsmc_exp_table.h, generated by tools/gen_exp_table.py). For |x| < 512:
 * n = round(x 128/ln2) = 128 k + j (a shift-add rounding), r = x - n ln2/128 in two parts
 * (|r| <= ln2/256), and exp x = 2^k 2^(j/128) e^r = scale (1 + tail + r + r^2/2 + ... + r^5/120)
 * with scale = 2^k s_j built from the table's bits and tail the table's correction, summed by
 * one fma. No division (fdlibm's form, kept for |x| >= 512 and NaN, divides): about 30
 * instructions where there were 70. Within 0.6 ulp (tests/test_oracle_math.py against
 * decimal). */
WSMC_HD const uint64_t* wsmc_exp_table(void) {
    static const uint64_t t[2 * WSMC_EXP_TABLE_N] = WSMC_EXP_TAB_INIT;
    return t;
}
/* WSMC_TABLES_LDS (a kernel's translation unit defines it; the kernel calls
 * wsmc_tables_to_lds() first): the lookups read LDS copies of the log / exp tables, the same
 * values at LDS latency instead of a vector gather through the caches */
#if defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__)
__shared__ uint64_t wsmc_lds_exp_tab[2 * WSMC_EXP_TABLE_N];
__shared__ double wsmc_lds_log_tab[2 * WSMC_LOG_TABLE_N];
#ifdef WSMC_LDS_TABLE_CHECK
/* the check build: every entry point of a WSMC_TABLES_LDS translation unit must call
 * wsmc_tables_to_lds() before its first log / exp. wsmc_tables_to_lds marks the copies ready; a
 * lookup that finds them unmarked reports the kernel once a block (printf) and reads the constant
 * tables instead, so the mistake shows in the log and not as wrong values. */
__shared__ uint32_t wsmc_lds_tab_ready;
#define WSMC_LDS_TAB_READY 0x7AB1E5u
__device__ inline bool wsmc_lds_tabs_ok(void) {
    if (wsmc_lds_tab_ready == WSMC_LDS_TAB_READY) return true;
    if (threadIdx.x == 0) printf("wsmc: log/exp table lookup before wsmc_tables_to_lds() (block %u)\n", blockIdx.x);
    return false;
}
#endif
#endif
/* the table wsmc_exp reads (as WSMC_LOG_TAB for the log) */
#if defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__) && defined(WSMC_LDS_TABLE_CHECK)
#define WSMC_EXP_TAB (wsmc_lds_tabs_ok() ? wsmc_lds_exp_tab : wsmc_exp_table())
#elif defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__)
#define WSMC_EXP_TAB wsmc_lds_exp_tab
#else
#define WSMC_EXP_TAB wsmc_exp_table()
#endif
WSMC_HD double wsmc_exp_t(double x, const uint64_t* tab) {
    if (!(wsmc_fabs(x) < 512.0)) return wsmc_exp_fd(x);   /* rare: large |x|, infinities, NaN */
    const double shift = 6755399441055744.0;              /* 0x1.8p52: z + shift rounds z to an integer */
    const double kd0 = x * WSMC_EXP_INVLN2N + shift;
    const uint64_t ki = wsmc_d2bits(kd0);
    const double kd = kd0 - shift;
    const double r = (x - kd * WSMC_EXP_LN2HIN) - kd * WSMC_EXP_LN2LON;   /* kd * hi exact */
    const uint32_t j = (uint32_t)ki & (WSMC_EXP_TABLE_N - 1);
    const uint64_t sb = tab[2 * j];
    const double tail = wsmc_bits2d(tab[2 * j + 1]);
    const double scale = wsmc_bits2d(sb + (ki << 45));
    const double r2 = r * r;
    const double p = __builtin_fma(r, WSMC_K(0.16666666666666666), 0.5) +
                     r2 * __builtin_fma(r, WSMC_K(0.008333333333333333), WSMC_K(0.041666666666666664));
    const double tmp = tail + (r + r2 * p);
    return __builtin_fma(scale, tmp, scale);
}
WSMC_HD double wsmc_exp(double x) { return wsmc_exp_t(x, WSMC_EXP_TAB); }

/*
 * exp(x) for the Resample statistics, x = lw - M <= 0 (include/wsmc_math.h wsmc_qparts):
 * Cody-Waite reduction by ln2 and a degree-13 Taylor polynomial in Horner form with
 * explicit fma (IEEE-exact on v_fma_f64 and x86 FMA3), no division or branches on the
 * value path. Returns 0 for x < -80 (exp(-80) < 2^-115, below every fixed point the
 * statistics keep) and NaN for NaN. |error| ~ 2 ulp on [-80, 0].
 */
WSMC_HD double wsmc_expw(double x) {
    /* branch-free (a select at the end): the device evaluates the polynomial for every lane */
    const int ok = x >= -80.0;
    const double xr = x;
    x = ok ? x : -80.0;
    const double kd = wsmc_floor(x * 1.44269504088896338700e+00 + 0.5);
    const double r = (x - kd * 6.93147180369123816490e-01) - kd * 1.90821492927058770002e-10;
    double p = 1.6059043836821613e-10;                 /* 1/13! */
    p = __builtin_fma(p, r, WSMC_K(2.08767569878681e-09));
    p = __builtin_fma(p, r, WSMC_K(2.505210838544172e-08));
    p = __builtin_fma(p, r, WSMC_K(2.755731922398589e-07));
    p = __builtin_fma(p, r, WSMC_K(2.7557319223985893e-06));
    p = __builtin_fma(p, r, WSMC_K(2.48015873015873e-05));
    p = __builtin_fma(p, r, WSMC_K(0.0001984126984126984));
    p = __builtin_fma(p, r, WSMC_K(0.001388888888888889));
    p = __builtin_fma(p, r, WSMC_K(0.008333333333333333));
    p = __builtin_fma(p, r, WSMC_K(0.041666666666666664));
    p = __builtin_fma(p, r, WSMC_K(0.16666666666666666));
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const double y = p * wsmc_pow2i((int)kd);
    return ok ? y : (wsmc_isnan(xr) ? xr : 0.0);
}

/* exp without a division (the damped-oscillator mean, evaluated O(t) times per particle per
 * Move fold): for |x| <= 700 the Cody-Waite reduction and degree-13 Taylor polynomial of
 * wsmc_expw (~2 ulp) scaled by 2^k in the normal range; wsmc_exp elsewhere (and NaN). */
WSMC_HD double wsmc_exp_nd(double x) {
    if (!(x >= -700.0 && x <= 700.0)) return wsmc_exp(x);
    const double kd = wsmc_floor(x * 1.44269504088896338700e+00 + 0.5);
    const double r = (x - kd * 6.93147180369123816490e-01) - kd * 1.90821492927058770002e-10;
    double p = 1.6059043836821613e-10;                 /* 1/13! */
    p = __builtin_fma(p, r, 2.08767569878681e-09);
    p = __builtin_fma(p, r, 2.505210838544172e-08);
    p = __builtin_fma(p, r, 2.755731922398589e-07);
    p = __builtin_fma(p, r, 2.7557319223985893e-06);
    p = __builtin_fma(p, r, 2.48015873015873e-05);
    p = __builtin_fma(p, r, 0.0001984126984126984);
    p = __builtin_fma(p, r, 0.001388888888888889);
    p = __builtin_fma(p, r, 0.008333333333333333);
    p = __builtin_fma(p, r, 0.041666666666666664);
    p = __builtin_fma(p, r, 0.16666666666666666);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return p * wsmc_pow2i((int)kd);
}

/* log(x), table-driven (the approach of Julia's own Base.log and of glibc's log, restated with
 * this file's table: include/wsmc_log_table.h, generated by tools/gen_log_table.py). x = 2^k z
 * with z in [0x1.6p-1, 0x1.6p0); the top 7 bits of z's mantissa above 0x3fe6... select an
 * interval with centre c, invc = 1/c and logc = -log(invc) correctly rounded; then
 *   r = fma(z, invc, -1)             |r| < 2^-7 (one rounding of z/c - 1; exact when c = 1)
 *   log x = k ln2 + logc + log1p(r),  log1p(r) = r + r^2 q(r), q the Taylor series to r^6
 * summed as hi = (k ln2hi + logc) + r plus both sums' rounding errors, k ln2lo and r^2 q. The two
 * intervals around 1 have c = 1 exactly, so log x near 1 is r + r^2 q(r) with r = x - 1 exact:
 * relative accuracy where the result is small. No division (the fdlibm form it replaces
 * divided f / (2 + f)): about 30 instructions where there were 65. Within 0.6 ulp
 * (tests/test_oracle_math.py checks it against decimal logs). Zero, negatives, subnormals,
 * infinities and NaN take one rarely-taken branch. */
WSMC_HD const double* wsmc_log_table(void) {
    static const double t[2 * WSMC_LOG_TABLE_N] = WSMC_LOG_TAB_INIT;
    return t;
}
/* the table wsmc_log reads: the LDS copy in a WSMC_TABLES_LDS translation unit, else the
 * constant one (a kernel may also pass its own LDS copy to wsmc_log_t) */
#if defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__) && defined(WSMC_LDS_TABLE_CHECK)
#define WSMC_LOG_TAB (wsmc_lds_tabs_ok() ? wsmc_lds_log_tab : wsmc_log_table())
#elif defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__)
#define WSMC_LOG_TAB wsmc_lds_log_tab
#else
#define WSMC_LOG_TAB wsmc_log_table()
#endif
#if defined(WSMC_TABLES_LDS) && defined(__HIP_DEVICE_COMPILE__)
/* every thread of the block copies its share of both tables, then one barrier */
__device__ inline void wsmc_tables_to_lds(void) {
    const double* lt = wsmc_log_table();
    const uint64_t* et = wsmc_exp_table();
    for (int k = (int)threadIdx.x; k < 2 * WSMC_LOG_TABLE_N; k += (int)blockDim.x) wsmc_lds_log_tab[k] = lt[k];
    for (int k = (int)threadIdx.x; k < 2 * WSMC_EXP_TABLE_N; k += (int)blockDim.x) wsmc_lds_exp_tab[k] = et[k];
#ifdef WSMC_LDS_TABLE_CHECK
    if (threadIdx.x == 0) wsmc_lds_tab_ready = WSMC_LDS_TAB_READY;
#endif
    __syncthreads();
}
#endif
WSMC_HD double wsmc_log_t(double x, const double* tab) {
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
    uint64_t b = wsmc_d2bits(x);
    if (b - 0x0010000000000000ULL >= 0x7fe0000000000000ULL) {   /* not a positive normal */
        if (wsmc_isnan(x)) return x;
        if (x < 0.0) return WSMC_NAN;
        if (x == 0.0) return -WSMC_INF;
        if (x == WSMC_INF) return x;
        b = wsmc_d2bits(x * 4503599627370496.0) - (52ULL << 52);   /* subnormal: 2^52 x, k - 52 */
    }
    const uint64_t tmp = b - 0x3fe6000000000000ULL;
    const uint32_t i = (uint32_t)(tmp >> 45) & (WSMC_LOG_TABLE_N - 1);
    const int k = (int32_t)(uint32_t)(tmp >> 32) >> 20;   /* (int64_t)tmp >> 52, from the high word */
    const double z = wsmc_bits2d(b - (tmp & (0xfffULL << 52)));
    const double invc = tab[2 * i], logc = tab[2 * i + 1];
    const double r = __builtin_fma(z, invc, -1.0);
    const double kd = (double)k;
    const double kh = kd * ln2hi;   /* exact: ln2hi has 32 trailing zero bits */
    const double w = kh + logc;
    const double we = (kh - w) + logc;   /* w's rounding error (|kh| >= |logc| unless kh = 0) */
    const double hi = w + r;
    const double lo = (kd * ln2lo + we) + ((w - hi) + r);
    double q = -0.125;
    q = __builtin_fma(q, r, WSMC_K(0.14285714285714285));   /* 1/7 */
    q = __builtin_fma(q, r, WSMC_K(-0.16666666666666666));  /* -1/6 */
    q = __builtin_fma(q, r, WSMC_K(0.2));
    q = __builtin_fma(q, r, -0.25);
    q = __builtin_fma(q, r, WSMC_K(0.3333333333333333));    /* 1/3 */
    q = __builtin_fma(q, r, -0.5);
    return hi + __builtin_fma(r * r, q, lo);
}
WSMC_HD double wsmc_log(double x) { return wsmc_log_t(x, WSMC_LOG_TAB); }

/* log1p via the Goldberg correction (accurate to a few ulp; used for log1pexp) */
WSMC_HD double wsmc_log1p(double x) {
    double u = 1.0 + x;
    if (u == 1.0) return x;
    if (u == WSMC_INF) return u;
    return wsmc_log(u) * (x / (u - 1.0));
}

WSMC_HD double wsmc_sqrt(double x) { return __builtin_sqrt(x); }

/* ------------------------------------------------------------------------- */
/* sin / cos (fdlibm k_sin.c / k_cos.c kernels + Cody–Waite reduction)        */
/* ------------------------------------------------------------------------- */
WSMC_HD double wsmc_ksin(double x) {   /* |x| <= pi/4 */
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + (x * z) * (S1 + z * r);
}
WSMC_HD double wsmc_kcos(double x) {   /* |x| <= pi/4 */
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

/* cos(2*pi*u), sin(2*pi*u) for u in [0,1), exact octant reduction */
WSMC_HD void wsmc_sincos2pi(double u, double* s, double* c) {
    const double PIO4 = 7.85398163397448278999e-01;
    double y = u * 8.0;
    int o = (int)y;
    double f = y - (double)o;
    if (o & 1) f = 1.0 - f;
    double t = f * PIO4;
    double st = wsmc_ksin(t), ct = wsmc_kcos(t);
    /* octant o: (cos, sin) = (ct, st), (st, ct), (-st, ct), (-ct, st), (-ct, -st), (-st, -ct),
       (st, -ct), (ct, -st) for o = 0..7 — as selects, no divergent switch */
    const int swap = ((o + 1) & 2) != 0;            /* o = 1, 2, 5, 6 */
    const double a = swap ? st : ct, b = swap ? ct : st;
    *c = ((o + 2) & 4) ? -a : a;                    /* o = 2..5 */
    *s = (o & 4) ? -b : b;                          /* o = 4..7 */
}


/* ---- argument reduction by pi/2 for large |x| (Payne-Hanek) --------------------------------
 * The Cody-Waite three-part reduction below is exact only while fn * p1 is (fn < 2^20), i.e.
 * |x| < 2^19 pi/2. Past that (and up to the largest double) x mod pi/2 comes from the binary
 * expansion of 2/pi: x = M 2^E (M a 53-bit integer), and only the 2/pi bits from E - 1 onward
 * reach x (2/pi) mod 4 (earlier bits give multiples of 4). A 192-bit window W of those bits gives
 * y = M W / 2^190: bits 190-191 the quadrant, bits 62-189 the fraction (128 bits, so a remainder
 * as small as any double's distance to a multiple of pi/2, about 2^-61, keeps 53+ significant
 * bits; the bits past the window move y by < 2^-136). The fraction times pi/2 in double-double
 * is rounded once. Julia's rem_pio2 is exact too, so sin/cos of huge arguments now agree with
 * Base to the kernels' accuracy. */
WSMC_HD uint64_t wsmc_2opi_word(int j) {   /* bits 64j+1 .. 64j+64 of 2/pi (MSB first), j < 20 */
    static const uint64_t t[20] = {
        0xa2f9836e4e441529ULL, 0xfc2757d1f534ddc0ULL, 0xdb6295993c439041ULL, 0xfe5163abdebbc561ULL,
        0xb7246e3a424dd2e0ULL, 0x06492eea09d1921cULL, 0xfe1deb1cb129a73eULL, 0xe88235f52ebb4484ULL,
        0xe99c7026b45f7e41ULL, 0x3991d639835339f4ULL, 0x9c845f8bbdf9283bULL, 0x1ff897ffde05980fULL,
        0xef2f118b5a0a6d1fULL, 0x6d367ecf27cb09b7ULL, 0x4f463f669e5fea2dULL, 0x7527bac7ebe5f17bULL,
        0x3d0739f78a5292eaULL, 0x6bfb5fb11f8d5d08ULL, 0x56033046fc7b6babULL, 0xf0cfbc209af4361dULL};
    return (unsigned)j < 20u ? t[j] : 0;
}
WSMC_HD int wsmc_clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }
/* 64 bits of 2/pi from bit pos on (bits at pos <= 0 are 0: 2/pi < 1) */
WSMC_HD uint64_t wsmc_2opi_bits(int pos) {
    if (pos <= -63) return 0;
    if (pos <= 0) return wsmc_2opi_word(0) >> (1 - pos);
    const int j = (pos - 1) >> 6, sh = (pos - 1) & 63;
    return sh ? (wsmc_2opi_word(j) << sh) | (wsmc_2opi_word(j + 1) >> (64 - sh)) : wsmc_2opi_word(j);
}
/* ax finite, ax >= 2^19 pi/2: r in [-pi/4, pi/4] and the quadrant n with ax = r + n pi/2 (mod 2 pi).
 * Out of line on the device (returned by value, no stack): inlined at every sin / cos it tripled
 * the compile time of the run-time compiled Move blocks whose folds carry oscillator terms. */
typedef struct { double r; int n; } wsmc_rq;
#if defined(__HIPCC__) || defined(__HIP__)
__host__ __device__ inline __attribute__((noinline))
#else
static __attribute__((noinline))
#endif
wsmc_rq wsmc_rem_pio2_large_rq(double ax) {
    int n = 0;
    wsmc_rq o;
    o.r = 0.0;
    {
    const uint64_t b = wsmc_d2bits(ax);
    const int E = (int)((b >> 52) & 0x7ff) - 1075;       /* ax = M 2^E */
    const uint64_t M = (b & 0x000fffffffffffffULL) | 0x0010000000000000ULL;
    /* window W (192 bits) = 2/pi bits E-1 .. E+190: y = M W / 2^190 */
    const int s = E - 1;
    /* P = M W limb by limb, low to high (a rolled loop: one multiply in the code, which keeps the
       inlined path small where sin / cos sit in unrolled folds) */
    uint64_t L0 = 0, L1 = 0, L2 = 0;
    wsmc_u128 acc = 0;
#if defined(__clang__)
#pragma nounroll
#endif
    for (int i = 0; i < 3; ++i) {
        acc += (wsmc_u128)M * wsmc_2opi_bits(s + 128 - 64 * i);
        L0 = L1; L1 = L2; L2 = (uint64_t)acc;
        acc >>= 64;
    }                                              /* bits >= 192 (acc): multiples of 4 in y */
    int q = (int)(L2 >> 62);                                /* bits 190-191 */
    wsmc_u128 G = ((wsmc_u128)(L2 & ((1ULL << 62) - 1)) << 66) | ((wsmc_u128)L1 << 2) | (L0 >> 62);
    int neg = 0;
    if (G >> 127) {                                /* fraction >= 1/2: the next quadrant, r < 0 */
        q = (q + 1) & 3;
        G = (wsmc_u128)0 - G;
        neg = 1;
    }
    n = q;
    if (G == 0) { o.n = n; return o; }
    const uint64_t gh = (uint64_t)(G >> 64), gl = (uint64_t)G;
    const int lz = gh ? wsmc_clz64(gh) : 64 + wsmc_clz64(gl);
    const wsmc_u128 Gn = G << lz;                  /* MSB at bit 127 */
    const uint64_t h53 = (uint64_t)(Gn >> 75), l53 = (uint64_t)(Gn >> 22) & ((1ULL << 53) - 1);
    const double fh = (double)(int64_t)h53 * wsmc_pow2i(-53 - lz);      /* exact */
    const double fl = (double)(int64_t)l53 * wsmc_pow2i(-106 - lz);     /* exact (lz <= 127) */
    const double pio2_hi = 1.5707963267948966, pio2_lo = 6.123233995736766e-17;
    const double rh = fh * pio2_hi;
    const double e = __builtin_fma(fh, pio2_hi, -rh);
    const double rl = e + (fh * pio2_lo + fl * pio2_hi);
    const double r = rh + rl;
    o.r = neg ? -r : r;
    o.n = n;
    return o;
    }
}
WSMC_HD double wsmc_rem_pio2_large(double ax, int* n) {
    const wsmc_rq o = wsmc_rem_pio2_large_rq(ax);
    *n = o.n;
    return o.r;
}
#define WSMC_PIO2_LARGE 823549.0                   /* < 2^19 pi/2: Cody-Waite below, Payne-Hanek above */

/* The oscillator phase's reduction (wsmc_cos_cw, wsmc_sincos), inline and branch-free: the
 * three-part Cody–Waite form below WSMC_PIO2_LARGE (2^19 pi/2 = 8.2e5 rad; the values of every
 * earlier round), and from there to WSMC_PIO2_FMA_MAX (2^43 = 8.8e12 rad) two FMAs against pi/2 =
 * P1 + P2 (double-double): ax - fn P1 is exact in one fma (ax and fn P1 are multiples of 2^-52 and
 * their difference is below 0.79 in magnitude), so r carries one rounding plus fn |pi/2 - P1 - P2|
 * <= 2^-64 of absolute error; fn, rounded from ax 2/pi, is off by at most 2^-10 of a quadrant, so
 * |r| <= pi/4 + 2^-9 stays in the kernels' range. Round 6: the phase past 8.2e5 rad was NaN, so a long time span or a
 * large w gave NaN weights where the reference's cos(w t + p) is finite
 * (examples/damped_oscillator.jl:11); the Payne–Hanek call the general wsmc_cos makes would cost
 * the run-time compiled Move blocks 7 VGPRs (3 -> 2 waves a SIMD). Past 2^43 rad (no physical
 * phase) the value is NaN. */
#define WSMC_PIO2_FMA_MAX 8796093022208.0          /* 2^43 */
WSMC_HD double wsmc_osc_reduce(double ax, int* n) {
    const double invpio2 = 6.36619772367581382433e-01, p1 = 1.57079632673412561417e+00,
                 p2 = 6.07710050630396597660e-11, p3 = 2.02226624879595063154e-21;
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17;     /* pi/2 = P1 + P2 + O(2^-107) */
    const double axr = ax < WSMC_PIO2_FMA_MAX ? ax : 0.0;
    const double fn = (double)(int64_t)(axr * invpio2 + 0.5);
    const double rcw = ((ax - fn * p1) - fn * p2) - fn * p3;
    const double rfm = __builtin_fma(-fn, P2, __builtin_fma(-fn, P1, ax));
    *n = (int)((int64_t)fn & 3);
    return ax < WSMC_PIO2_LARGE ? rcw : ax < WSMC_PIO2_FMA_MAX ? rfm : WSMC_NAN;
}
/* cos(x) for the damped-oscillator phase w t + p (its mean and the rotation anchors, wsmc_sincos) */
WSMC_HD double wsmc_cos_cw(double x) {
    if (!wsmc_isfinite(x)) return WSMC_NAN;
    const double ax = wsmc_fabs(x);
    const int small = ax <= 7.85398163397448278999e-01;
    int nr;
    const double rr = wsmc_osc_reduce(ax, &nr);
    const double r = small ? x : rr;
    const int n = small ? 0 : nr;
    const double kc = wsmc_kcos(r), ks = wsmc_ksin(r);
    const double v = (n & 1) ? ks : kc;
    return ((n + 1) & 2) ? -v : v;
}

/* cos(x) for every finite x (Cody–Waite three-part pi/2 below WSMC_PIO2_LARGE, Payne–Hanek above); NaN/inf -> NaN */
WSMC_HD double wsmc_cos(double x) {
    const double invpio2 = 6.36619772367581382433e-01,
                 p1 = 1.57079632673412561417e+00,   /* first 33 bits of pi/2 */
                 p2 = 6.07710050630396597660e-11,   /* next 33 bits */
                 p3 = 2.02226624879595063154e-21;   /* pi/2 - p1 - p2 */
    if (!wsmc_isfinite(x)) return WSMC_NAN;
    /* branch-free on the value path (a wave's lanes sit in different quadrants): both
       kernel polynomials, then selects; |x| <= pi/4 is quadrant 0 with r = x. The values
       are those of the branchy form (kcos(x) for small |x|, else the quadrant's kernel). */
    const double ax = wsmc_fabs(x);
    const int small = ax <= 7.85398163397448278999e-01;
    const double axr = ax < WSMC_PIO2_LARGE ? ax : 0.0;
    const double fn = (double)(int64_t)(axr * invpio2 + 0.5);
    double rr = ((ax - fn * p1) - fn * p2) - fn * p3;
    int nr = (int)((int64_t)fn & 3);
    if (ax >= WSMC_PIO2_LARGE) rr = wsmc_rem_pio2_large(ax, &nr);
    const double r = small ? x : rr;
    const int n = small ? 0 : nr;
    const double kc = wsmc_kcos(r), ks = wsmc_ksin(r);
    const double v = (n & 1) ? ks : kc;
    return ((n + 1) & 2) ? -v : v;   /* n = 1, 2 negate */
}

/* sin(x), the same reduction and kernels as wsmc_cos: sin(|x|) by quadrant, the sign of x
   restored (ksin is odd bit for bit, so the small case is ksin(x) itself) */
WSMC_HD double wsmc_sin(double x) {
    const double invpio2 = 6.36619772367581382433e-01, p1 = 1.57079632673412561417e+00,
                 p2 = 6.07710050630396597660e-11, p3 = 2.02226624879595063154e-21;
    if (!wsmc_isfinite(x)) return WSMC_NAN;
    const double ax = wsmc_fabs(x);
    const int small = ax <= 7.85398163397448278999e-01;
    const double axr = ax < WSMC_PIO2_LARGE ? ax : 0.0;
    const double fn = (double)(int64_t)(axr * invpio2 + 0.5);
    double rr = ((ax - fn * p1) - fn * p2) - fn * p3;
    int nr = (int)((int64_t)fn & 3);
    if (ax >= WSMC_PIO2_LARGE) rr = wsmc_rem_pio2_large(ax, &nr);
    const double r = small ? ax : rr;
    const int n = small ? 0 : nr;
    const double kc = wsmc_kcos(r), ks = wsmc_ksin(r);
    double v = (n & 1) ? kc : ks;
    v = (n & 2) ? -v : v;            /* n = 2, 3 negate */
    return (wsmc_d2bits(x) >> 63) ? -v : v;
}

/* Base.min / Base.max for Float64 (Julia >= 1.9): the difference's sign picks the operand,
   so min(-0.0, 0.0) = -0.0; a NaN operand gives the (NaN) difference */
WSMC_HD double wsmc_min(double a, double b) {
    const double d = a - b;
    const double m = (wsmc_d2bits(d) >> 63) ? a : b;
    return (wsmc_isnan(a) || wsmc_isnan(b)) ? d : m;
}
WSMC_HD double wsmc_max(double a, double b) {
    const double d = a - b;
    const double m = (wsmc_d2bits(d) >> 63) ? b : a;
    return (wsmc_isnan(a) || wsmc_isnan(b)) ? d : m;
}

/* x^n for an integer n: Base.literal_pow's forms for n in -2..3 (x^2 = x*x, x^3 = x*x*x,
   x^-1 = inv(x), x^-2 = inv(x)^2), else Base.pow_body(::Float64, ::Integer): power by
   squaring carrying each product's rounding error (two_mul by fma), muladd taken as fma */
WSMC_HD double wsmc_powi(double x, int64_t n) {
    if (n == 0) return 1.0;
    if (n == 1) return x;
    if (n == 2) return x * x;
    if (n == 3) return x * x * x;
    if (n == -1) return 1.0 / x;
    if (n == -2) {
        const double r = 1.0 / x;
        return r * r;
    }
    double y = 1.0, xnlo = 0.0, ynlo = 0.0;
    if (n < 0) {
        const double rx = 1.0 / x;
        if (wsmc_isfinite(x)) xnlo = -__builtin_fma(x, rx, -1.0) * rx;
        x = rx;
        n = -n;
    }
    while (n > 1) {
        if (n & 1) {
            const double err = __builtin_fma(y, xnlo, x * ynlo);
            const double h = x * y;
            ynlo = __builtin_fma(x, y, -h) + err;
            y = h;
        }
        const double err = x * 2.0 * xnlo;
        const double h = x * x;
        xnlo = __builtin_fma(x, x, -h) + err;
        x = h;
        n >>= 1;
    }
    const double err = __builtin_fma(y, xnlo, x * ynlo);
    return (wsmc_isfinite(x) && wsmc_isfinite(err)) ? __builtin_fma(x, y, err) : x * y;
}

/* a^b (Base.^(::Float64, ::Float64)): 1 for a == 1, NaN for a NaN b, an integer b as x^n,
   else exp(b log a) — NaN for a < 0 (Julia throws a DomainError); relative error about
   |b log a| 2^-53 beyond the restated exp / log (Julia's double-double log is tighter) */
WSMC_HD double wsmc_pow(double a, double b) {
    /* Base.^(::Float64, ::Float64): |y| clamped to 1.5 2^62 first (past it every power over- or
       underflows, and an even integer keeps a negative base's sign right: (-2.0)^1e19 = Inf), an
       integer y as the integer power, then the domain cases (a negative base is Julia's
       DomainError: NaN here; 0^y and Inf^y by sign), else exp(y log x) */
    if (a == 1.0) return 1.0;
    if (!(wsmc_fabs(b) < 6917529027641081856.0)) {   /* 0x1.8p62 */
        if (wsmc_isnan(b)) return b;
        b = b > 0.0 ? 6917529027641081856.0 : -6917529027641081856.0;
    }
    const int64_t bi = (int64_t)b;
    if (b == (double)bi) return wsmc_powi(a, bi);
    if (a < 0.0) return WSMC_NAN;
    if (a == 0.0) return b > 0.0 ? 0.0 : WSMC_INF;
    if (!wsmc_isfinite(a)) return (b > 0.0 || wsmc_isnan(a)) ? a : 0.0;
    return wsmc_exp(b * wsmc_log(a));
}

/* ------------------------------------------------------------------------- */
/* draws                                                                      */
/* ------------------------------------------------------------------------- */
/* Box–Muller pair from one Philox block: z0 = r cos(2πu2), z1 = r sin(2πu2) */
WSMC_HD void wsmc_normal_pair_t(wsmc_u32x4 w, double* z0, double* z1, const double* logtab) {
    double u1 = wsmc_u01_open0(w.v[0], w.v[1]);
    double u2 = wsmc_u01(w.v[2], w.v[3]);
    double r = wsmc_sqrt(-2.0 * wsmc_log_t(u1, logtab));
    double s, c;
    wsmc_sincos2pi(u2, &s, &c);
    *z0 = r * c; *z1 = r * s;
}
WSMC_HD void wsmc_normal_pair(wsmc_u32x4 w, double* z0, double* z1) { wsmc_normal_pair_t(w, z0, z1, WSMC_LOG_TAB); }
/* k-th standard normal of (op, idx) */
WSMC_HD double wsmc_normal_k(uint64_t seed, uint64_t op, uint64_t idx, uint32_t k) {
    double z0, z1;
    wsmc_normal_pair(wsmc_rng_block(seed, op, idx, k >> 1), &z0, &z1);
    return (k & 1) ? z1 : z0;
}
/* k-th uniform in [0,1) of (op, idx) */
WSMC_HD double wsmc_uniform_k(uint64_t seed, uint64_t op, uint64_t idx, uint32_t k) {
    wsmc_u32x4 w = wsmc_rng_block(seed, op, idx, (k >> 1) | 0x80u);
    return (k & 1) ? wsmc_u01(w.v[2], w.v[3]) : wsmc_u01(w.v[0], w.v[1]);
}
/* 32-bit stratum offset word for resampling slot n (systematic: one word for all slots).
 * A per-Resample key k = murmur3 fmix64(seed ^ op*phi ^ c) (uniform over a launch, so the
 * device evaluates it once on the scalar unit), then a 32-bit integer hash of the slot:
 * x = lo32(n) ^ lo32(k) ^ (hi32(n) * c' ^ hi32(k)), and Wellons' lowbias32 finalizer
 * (xorshift-multiply x2, a bijection on 32 bits). About 8 vector ops with two 32-bit
 * multiplies inside the per-particle rank() of the ancestor fill, where the 64-bit fmix of
 * every slot cost four times that. */
WSMC_HD uint64_t wsmc_strat_key(uint64_t seed, uint64_t op) {
    uint64_t z = seed ^ (op * 0x9E3779B97F4A7C15ULL) ^ 0x5851F42D4C957F2DULL;
    z ^= z >> 33;
    z *= 0xFF51AFD7ED558CCDULL;
    z ^= z >> 33;
    z *= 0xC4CEB9FE1A85EC53ULL;
    z ^= z >> 33;
    return z;
}
WSMC_HD uint32_t wsmc_strat_fin(uint32_t x) {   /* lowbias32 */
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
WSMC_HD uint32_t wsmc_strat_hash(uint64_t key, uint64_t n) {
    /* (lo32(n) ^ lo32(k)) ^ (hi32(n) c' ^ hi32(k)): the device splits the second term off once
       per launch when hi32(n) is constant over the slots (csrc/wsmc_kernels.hip SlotHash) */
    return wsmc_strat_fin((uint32_t)n ^ (uint32_t)key ^ ((uint32_t)(n >> 32) * 0x85EBCA6Bu ^ (uint32_t)(key >> 32)));
}
WSMC_HD uint32_t wsmc_strat_word(uint64_t seed, uint64_t op, uint64_t n) {
    return wsmc_strat_hash(wsmc_strat_key(seed, op), n);
}

/* ------------------------------------------------------------------------- */
/* log-densities (Distributions.jl semantics)                                 */
/* ------------------------------------------------------------------------- */
/* Normal(mu, sigma): -(z^2 + log(2pi))/2 - log(sigma),  z = (x - mu)/sigma
 * evaluated as fma(-h, h, c) with h = (x - mu) rh: per sigma value the pair
 *   c  = -log(2pi)/2 - log(sigma)   (wsmc_normal_c)
 *   rh = (1/sigma) / sqrt(2)        (wsmc_normal_rh)
 * (one log and one reciprocal per sigma value, reused across the terms of a fold that share it:
 * wsmc_scale_memo, or the host's wsmc_scale_pre), then per term a subtraction, a multiply and an
 * fma — -(z^2)/2 = -h^2 within a few ulps of z^2, rounded once into c. Five roundings per term
 * were a Move fold's dominant cost (the oscillator runs of examples/damped_oscillator.jl). */
#define WSMC_SQRT1_2 0.70710678118654752440
WSMC_HD double wsmc_normal_c(double lg) { return (-0.5 * WSMC_LOG2PI) - lg; }
WSMC_HD double wsmc_normal_rh(double rc) { return rc * WSMC_SQRT1_2; }
WSMC_HD double wsmc_normal_lh(double h, double c) { return __builtin_fma(-h, h, c); }
WSMC_HD double wsmc_normal_logpdf(double mu, double sigma, double x) {
    const double h = (x - mu) * wsmc_normal_rh(1.0 / sigma);
    return wsmc_normal_lh(h, wsmc_normal_c(wsmc_log(sigma)));
}
/* Truncated(Normal(0, sigma), 0, Inf) — examples/damped_oscillator.jl:24-28 */
WSMC_HD double wsmc_halfnormal_logpdf(double sigma, double x) {
    if (!(x >= 0.0)) return -WSMC_INF;
    return wsmc_normal_logpdf(0.0, sigma, x) + WSMC_LOG2;
}
/* Uniform(a, b) on the closed support [a, b] */
WSMC_HD double wsmc_uniform_logpdf(double a, double b, double x) {
    if (!(x >= a && x <= b)) return -WSMC_INF;
    return -wsmc_log(b - a);
}
/* the damped-oscillator mean, examples/damped_oscillator.jl:11 */
WSMC_HD double wsmc_oscillator(double t, double A, double om, double ga, double ph) {
    return A * wsmc_exp_nd(-ga * t) * wsmc_cos_cw(om * t + ph);
}
/* sin and cos with wsmc_cos_cw's reduction and kernels (the oscillator's phase): *c is wsmc_cos_cw(x)
   bit for bit (wsmc_cos(x) below WSMC_PIO2_LARGE, within an ulp of it up to 2^43 rad) */
WSMC_HD void wsmc_sincos(double x, double* s, double* c) {
    if (!wsmc_isfinite(x)) {
        *s = WSMC_NAN;
        *c = WSMC_NAN;
        return;
    }
    const double ax = wsmc_fabs(x);
    const int small = ax <= 7.85398163397448278999e-01;
    int nr;
    const double rr = wsmc_osc_reduce(ax, &nr);
    const double r = small ? x : rr;
    const int n = small ? 0 : nr;
    const double kc = wsmc_kcos(r), ks = wsmc_ksin(r);
    const double vc = (n & 1) ? ks : kc;
    *c = ((n + 1) & 2) ? -vc : vc;              /* cos(r + n pi/2): kc, -ks, -kc, ks */
    const double vs = (n & 1) ? kc : ks;
    const double sa = (n & 2) ? -vs : vs;       /* sin(r + n pi/2): ks, kc, -ks, -kc */
    *s = (!small && x < 0.0) ? -sa : sa;        /* reduced from |x|: sin is odd */
}
/* The oscillator mean by rotation (a restatement within floating-point
 * tolerance of examples/damped_oscillator.jl:11): the phasor z(t) = A e^{-g t} e^{i(w t + p)}
 * at an anchor t_a (Re z(t_a) is wsmc_oscillator(t_a, ...) bit for bit), advanced m times by
 * R = e^{(-g + i w) d}: Re z(t_a + m d) at one complex multiply per step instead of an exp and
 * a cos per term. The Observe terms of a regularly spaced run carry (t_a, d, m) (wsmc_osc_link). */
WSMC_HD void wsmc_osc_anchor(double ta, double A, double om, double ga, double ph, double* zr, double* zi) {
    double s, c;
    wsmc_sincos(om * ta + ph, &s, &c);
    const double ae = A * wsmc_exp_nd(-ga * ta);
    *zr = ae * c;
    *zi = ae * s;
}
WSMC_HD void wsmc_osc_step(double d, double om, double ga, double* rr, double* ri) {
    double s, c;
    wsmc_sincos(om * d, &s, &c);
    const double e = wsmc_exp_nd(-ga * d);
    *rr = e * c;
    *ri = e * s;
}
WSMC_HD void wsmc_osc_rotate(double* zr, double* zi, double rr, double ri) {
    const double a = *zr, b = *zi;
    *zr = __builtin_fma(a, rr, -(b * ri));
    *zi = __builtin_fma(a, ri, b * rr);
}
WSMC_HD double wsmc_osc_rolled(double ta, double d, int m, double A, double om, double ga, double ph) {
    double zr, zi;
    wsmc_osc_anchor(ta, A, om, ga, ph, &zr, &zi);
    if (m > 0) {
        double rr, ri;
        wsmc_osc_step(d, om, ga, &rr, &ri);
        for (int j = 0; j < m; ++j) wsmc_osc_rotate(&zr, &zi, rr, ri);
    }
    return zr;
}

/* ------------------------------------------------------------------------- */
/* bound transforms of RW/autoRW (src/move_kernels.jl:37-85)                  */
/* ------------------------------------------------------------------------- */
WSMC_HD double wsmc_to_unc_t(double x, double lo, double hi, const double* logtab) {
    int flo = wsmc_isfinite(lo), fhi = wsmc_isfinite(hi);
    if (flo && fhi) return wsmc_log_t(x - lo, logtab) - wsmc_log_t(hi - x, logtab);
    if (flo) return wsmc_log_t(x - lo, logtab);
    if (fhi) return wsmc_log_t(hi - x, logtab);
    return x;
}
WSMC_HD double wsmc_to_unc(double x, double lo, double hi) { return wsmc_to_unc_t(x, lo, hi, WSMC_LOG_TAB); }
WSMC_HD double wsmc_from_unc(double z, double lo, double hi) {
    int flo = wsmc_isfinite(lo), fhi = wsmc_isfinite(hi);
    if (flo && fhi) return lo + (hi - lo) / (1.0 + wsmc_exp(-z));
    if (flo) return lo + wsmc_exp(z);
    if (fhi) return hi - wsmc_exp(z);
    return z;
}
WSMC_HD double wsmc_log1pexp(double z) {
    return z > 0.0 ? z + wsmc_log1p(wsmc_exp(-z)) : wsmc_log1p(wsmc_exp(z));
}
/* log|dx/dz| of wsmc_from_unc; lgw = wsmc_log(hi - lo) (a bounded interval: callers with
 * constant bounds evaluate it once). log1pexp(z) and log1pexp(-z) are z+ + P and (-z)+ + P
 * with the one P = log1p(exp(-|z|)) (z > 0: z + log1p(exp(-z)) and log1p(exp(-z)); z <= 0,
 * -0.0 and NaN included: log1p(exp(z)) and (-z) + log1p(exp(z)) or, at 0, log1p(exp(0))):
 * wsmc_log1pexp's values with one exp and one log1p instead of two each. */
WSMC_HD double wsmc_log_abs_jac_pre(double z, double lo, double hi, double lgw) {
    int flo = wsmc_isfinite(lo), fhi = wsmc_isfinite(hi);
    if (flo && fhi) {
        const double P = wsmc_log1p(wsmc_exp(z > 0.0 ? -z : z));
        const double a = z > 0.0 ? z + P : P;            /* wsmc_log1pexp(z)  */
        const double b = -z > 0.0 ? -z + P : P;          /* wsmc_log1pexp(-z) */
        return lgw - a - b;
    }
    if (flo || fhi) return z;
    return 0.0;
}
WSMC_HD double wsmc_log_abs_jac(double z, double lo, double hi) {
    const int both = wsmc_isfinite(lo) && wsmc_isfinite(hi);
    return wsmc_log_abs_jac_pre(z, lo, hi, both ? wsmc_log(hi - lo) : 0.0);
}
/* One proposal step of a target under bounds (src/move_kernels.jl:154-172): from the current
 * value x and the unconstrained increment dz, the proposal xn = from_unc(to_unc(x) + dz)
 * (returned) and *dj = log|dx/dz|(zn) - log|dx/dz|(zo), the Jacobian part of the log proposal
 * ratio. flo / fhi: the bounds' finiteness (wsmc_isfinite, or known at compile time). With
 * both bounds finite the step shares its transcendentals, a restatement within rounding of the
 * term-by-term transforms above:
 *   la = log(x - lo), lb = log(hi - x), zo = la - lb                      (to_unc, the same bits)
 *   log|dx/dz|(zo) = log((x - lo)(hi - x)/(hi - lo)) = (la + lb) - lgw    (no exp, no log1p)
 *   e = exp(-|zn|), P = log1p(e): log|dx/dz|(zn) = (lgw - |zn|) - 2P   (= lgw - log1pexp(zn)
 *                                                                         - log1pexp(-zn))
 *   xn = lo + w/(1 + e) for zn >= 0, lo + (w e)/(1 + e) below (w = hi - lo; 1/(1 + exp(-zn)))
 * — three logs, one exp and two divisions where the transforms took four logs, three exps and
 * three divisions. One finite bound: zo = log(x - lo) or log(hi - x), xn = lo + exp(zn) or
 * hi - exp(zn), *dj = zn - zo; none: xn = x + dz, *dj = 0. */
WSMC_HD double wsmc_bounded_step(double x, double dz, double lo, double hi, double lgw, int flo, int fhi,
                                 double* dj) {
    if (flo && fhi) {
        const double la = wsmc_log(x - lo), lb = wsmc_log(hi - x);
        const double zn = (la - lb) + dz;
        const double az = wsmc_fabs(zn);
        const double e = wsmc_exp(-az);
        const double u = 1.0 + e;
        const double w = hi - lo;
        *dj = ((lgw - az) - 2.0 * wsmc_log1p(e)) - ((la + lb) - lgw);
        return lo + (zn >= 0.0 ? w / u : (w * e) / u);
    }
    if (flo || fhi) {
        const double zo = flo ? wsmc_log(x - lo) : wsmc_log(hi - x);
        const double zn = zo + dz;
        *dj = zn - zo;
        return flo ? lo + wsmc_exp(zn) : hi - wsmc_exp(zn);
    }
    *dj = 0.0;
    return x + dz;
}

/* ------------------------------------------------------------------------- */
/* integer weights, ESS, and the stratified/systematic target map            */
/* ------------------------------------------------------------------------- */
/*
 * exp_norm/ess_perc/icdf (src/resampling.jl:13-77) on an integer CDF:
 *   q_i = floor(expw(lw_i - M) * 2^K),  K = min(63 - ceil(log2 N), 43)   =>  Q = sum q_i <= 2^63
 * (expw: the division-free exp above)
 * Integer sums are associative, so the CDF, Q, the ESS sums and the ancestors are
 * identical for any reduction order, grid shape or shard count.
 */
WSMC_HD int wsmc_qbits(uint64_t n) {
    /* min(63 - ceil(log2 n), 43): Q = sum q_i <= n 2^K <= 2^63, and a 1024-particle tile's
       sums of q, q2 (<= 2^(K+10) <= 2^53) and wf, wf2 (< 2^52) are exact in f64, so a device
       accumulates all four per-particle integers in f64 and converts once per tile. The cap
       binds below n = 2^20 (C2's 1M particles already have K = 43). */
    const int k = n <= 1 ? 63 : 63 - (64 - __builtin_clzll(n - 1));
    return k < 43 ? k : 43;
}
/*
 * The reference point of the integer weights (round 6): R = ceil(M) for a finite max M (M
 * itself when it is +-inf or NaN). Every q, wf, q2, wf2 is taken against R, not M: e_i =
 * expw(lw_i - R) <= 1, the largest e lies in (1/e, 1], so the fixed point keeps all but
 * log2(e) = 1.44 bits of its resolution. R is a function of M alone, so the statement path
 * and the oracle need nothing else; but a kernel that knows an upper bound U >= M before M
 * itself (the fused 2D-SSM propagate: U = the previous step's max or log-mean + the
 * observation density's maximum) computes every q against ceil(U) in the same pass as the
 * weights, and ceil(U) == ceil(M) except when M and U straddle an integer — checked after
 * the fact, with the exact statistics recomputed then.
 */
WSMC_HD double wsmc_qref(double M) { return (M - M == 0.0) ? __builtin_ceil(M) : M; }

WSMC_HD uint64_t wsmc_qweight(double lw, double M, int K) {
    /* M: the reference point (wsmc_qref of the max) */
    double e = wsmc_expw(lw - M);
    if (!(e > 0.0)) return 0;            /* -inf weights, NaN */
    return wsmc_d_to_u64_trunc(e * wsmc_pow2i(K));
}

/*
 * The exact per-particle integers behind the Resample statistics (e = exp(lw - M), e2 = e*e
 * rounded once in f64):
 *   q   = floor(e * 2^K)                 CDF weight (above)
 *   wf  = floor(frac(e * 2^K) * 2^42)    so that  sum floor(e * 2^(K+42)) = Q * 2^42 + sum wf:
 *                                        sum_i e_i to 2^-(K+42) per particle (logsumexp,
 *                                        evidence, log-mean)
 *   q2  = floor(e2 * 2^K)                the same two-part fixed point of e^2:
 *   wf2 = floor(frac(e2 * 2^K) * 2^42)   sum floor(e2 * 2^(K+42)) = Q2 * 2^42 + sum wf2
 * ESS% = (sum e)^2 / (N sum e^2) (src/resampling.jl:51-54 on w = e / sum e) is then taken
 * from the two 85-bit sums: both are exact integers, so every reduction order, grid and shard
 * layout gives the same bits, and each sum carries at most N 2^-(K+42) <= 2^-42 of
 * truncation against a max term of 1 — the ESS matches the reference's f64 value to ~1e-15
 * relative, heavy tails included. wf, wf2 < 2^42 and a 1024-particle tile sum stays below
 * 2^53, so a device sums them in f64 exactly; q, q2 <= 2^K and their totals are u64
 * (Q2 <= Q <= 2^63, since e2 <= e).
 */
typedef struct { uint64_t q, wf, q2, wf2; } wsmc_qparts;
/* M: the reference point (wsmc_qref of the max) */
WSMC_HD wsmc_qparts wsmc_qparts_of(double lw, double M, int K) {
    wsmc_qparts p = {0, 0, 0, 0};
    double e = wsmc_expw(lw - M);
    if (!(e > 0.0)) return p;
    const double sK = wsmc_pow2i(K);
    double s = e * sK;
    double qd = wsmc_floor(s);
    p.q = wsmc_d_to_u64_trunc(qd);
    p.wf = wsmc_d_to_u64_trunc(wsmc_floor((s - qd) * 4398046511104.0));   /* 2^42 */
    double s2 = (e * e) * sK;
    double q2d = wsmc_floor(s2);
    p.q2 = wsmc_d_to_u64_trunc(q2d);
    p.wf2 = wsmc_d_to_u64_trunc(wsmc_floor((s2 - q2d) * 4398046511104.0));
    return p;
}

/*
 * Targets: slot n (0-based) has A_n = n*2^32 + R_n (stratified: R_n = strat word of n;
 * systematic: R_n = R_0), and x_n = floor(A_n * Q / (N * 2^32)) in [0, Q).  This is
 * us[n] = (n-1)/N + rand()/N of src/resampling.jl:40 with the uniform on a 2^-32 grid,
 * scaled to the integer CDF. ancestor(n) = smallest m with C_m > x_n, where C_m is the
 * inclusive prefix of q — the `while s < us[n]` merge of src/resampling.jl:18-24.
 */
WSMC_HD uint64_t wsmc_target(uint64_t n, uint32_t R, uint64_t Q, uint64_t N) {
    wsmc_u128 A = ((wsmc_u128)n << 32) | R;
    wsmc_u128 num = A * (wsmc_u128)Q;
    wsmc_u128 den = (wsmc_u128)N << 32;
    return (uint64_t)(num / den);
}

/* #{ n : x_n < c }  (monotone in c); scheme 0 = stratified, 1 = systematic.
 * ratio = N/Q as a double (any estimate works: the result is corrected exactly). */
/* x * y exactly, for y < 2^32 (two 32x32->64 products; cheap on the device) */
WSMC_HD wsmc_u128 wsmc_mul64x32(uint64_t x, uint32_t y) {
    return ((wsmc_u128)((x >> 32) * (uint64_t)y) << 32) + (wsmc_u128)((x & 0xffffffffULL) * (uint64_t)y);
}
WSMC_HD uint64_t wsmc_rank_r(uint64_t c, uint64_t Q, uint64_t N, double ratio, int scheme,
                             uint64_t seed, uint64_t op, uint64_t slot_base) {
    if (c == 0) return 0;
    if (c >= Q) return N;
    /* N < 2^32 (a shard): every product below is 64 x 32 bits */
    const wsmc_u128 cN = wsmc_mul64x32(c, (uint32_t)N);
    /* n* = floor(c*N/Q) and rem = c*N - n*·Q in [0, Q): float estimate, exact correction
       (the estimate only seeds the correction, so its rounding never shows in the result) */
    uint64_t ns = wsmc_d_to_u64_trunc(wsmc_u64_to_d(c) * ratio);
    if (ns > N) ns = N;
    wsmc_u128 p = wsmc_mul64x32(Q, (uint32_t)ns);
    while (p > cN) { --ns; p -= Q; }
    while (cN - p >= Q) { ++ns; p += Q; }
    if (ns >= N) return N;
    const uint64_t rem = (uint64_t)(cN - p);
    const uint32_t R = wsmc_strat_word(seed, op, scheme == 1 ? slot_base : slot_base + ns);
    /* x_{n*} < c  <=>  (n*·2^32 + R)·Q < c·N·2^32  <=>  R·Q < rem·2^32 */
    return ns + (wsmc_mul64x32(Q, R) < ((wsmc_u128)rem << 32) ? 1u : 0u);
}
WSMC_HD uint64_t wsmc_rank(uint64_t c, uint64_t Q, uint64_t N, int scheme,
                           uint64_t seed, uint64_t op, uint64_t slot_base) {
    return wsmc_rank_r(c, Q, N, wsmc_u64_to_d(N) / wsmc_u64_to_d(Q), scheme, seed, op, slot_base);
}

/*
 * Multinomial resampling (north-star addition; the reference has stratified only), drawn
 * as sorted uniforms from normalised exponential spacings (the order statistics of N iid
 * uniforms: U_(n) = P_n / P_N, P_n = E_0 + ... + E_n, N + 1 exponentials). The offspring
 * counts are Multinomial(N, q/Q); the ancestors come out sorted, so the column gather and
 * the history trace-back stay coalesced.
 * Exact in integers: E_k = floor(-log(u_k) * 2^24) + 1 >= 1 (u_k in (0, 1], a 53-bit word of
 * (seed, op, slot k); the terminal E_N has its own stream), so every P_n < 2^62 for
 * N < 2^31 and P_n < P_N for n < N. Slot n's ancestor is the smallest m with
 * C_m > floor(Q P_n / P_N), i.e. Q * P_n < C_m * P_N (u128 products, no division).
 */
WSMC_HD uint64_t wsmc_multi_word(uint64_t seed, uint64_t op, uint64_t n) {
    uint64_t z = seed ^ (op * 0x9E3779B97F4A7C15ULL) ^ (n * 0xD1B54A32D192ED03ULL) ^ 0x2545F4914F6CDD1DULL;
    z ^= z >> 33;
    z *= 0xFF51AFD7ED558CCDULL;
    z ^= z >> 33;
    z *= 0xC4CEB9FE1A85EC53ULL;
    z ^= z >> 33;
    return z;
}
WSMC_HD uint64_t wsmc_multi_expo(uint64_t word) {
    const double u = wsmc_u64_to_d((word >> 11) + 1) * 1.1102230246251565e-16;   /* (0, 1], 2^-53 grid */
    return wsmc_d_to_u64_trunc(wsmc_floor(-wsmc_log(u) * 16777216.0)) + 1;       /* 2^24 fixed point */
}
/* E_k of slot k (k < n) and the terminal E_n of a shard of n slots starting at slot_base */
WSMC_HD uint64_t wsmc_multi_e(uint64_t seed, uint64_t op, uint64_t slot_base, uint64_t k, uint64_t n) {
    return k < n ? wsmc_multi_expo(wsmc_multi_word(seed, op, slot_base + k))
                 : wsmc_multi_expo(wsmc_multi_word(seed, ~op, slot_base));
}
/* floor(U Q / 2^64) in [0, Q): one independent draw on the integer CDF */
WSMC_HD uint64_t wsmc_multi_target(uint64_t U, uint64_t Q) {
    return (uint64_t)(((wsmc_u128)U * (wsmc_u128)Q) >> 64);
}
/* C_m > floor(Q P / PN)  <=>  Q P < C_m PN */
WSMC_HD int wsmc_multi_above(uint64_t Cm, uint64_t Q, uint64_t P, uint64_t PN) {
    return (wsmc_u128)Q * (wsmc_u128)P < (wsmc_u128)Cm * (wsmc_u128)PN;
}

/*
 * sample(state, n; replace) (src/utils.jl:92-118) on the integer weights q:
 *  replace = true:  draw j is the smallest m with C_m > floor(U_j Q / 2^64), U_j a 64-bit
 *                   word of (seed, op, j) — independent draws, in draw order;
 *  replace = false: Efraimidis–Spirakis keys log(u_i) / q_i (u_i in (0, 1], a 53-bit word of
 *                   (seed, op, i); -inf for q_i = 0), the n largest, ties to the lower index.
 */
WSMC_HD double wsmc_es_key(uint64_t seed, uint64_t op, uint64_t i, uint64_t q) {
    if (q == 0) return -WSMC_INF;
    const double u = wsmc_u64_to_d((wsmc_multi_word(seed, op, i) >> 11) + 1) * 1.1102230246251565e-16;
    return wsmc_log(u) / wsmc_u64_to_d(q);
}

/*
 * describe()'s weighted median and sparkline histogram (src/utils.jl:94-141, :233-240), on
 * the integer weights q (exact sums, any order):
 *  median = StatsBase.quantile(v, Weights(w), 0.5): zero weights dropped, pairs sorted by
 *    (value, weight), h = (W - w1)/2 + w1 with w1 the first pair's weight; the first k with
 *    S_k > h (in integers: 2 S_k > Q + q1); vkold + (h - S_{k-1}) / w_k * (vk - vkold);
 *    no such k -> the largest value.
 *  histogram: 8 bins on edges range(lo, hi, length = 9) (Julia's twice-precision range:
 *    lo + k (hi - lo) / 8 rounded once, restated in double-double), bin =
 *    clamp(searchsortedlast(edges, v), 1, 8); levels clamp(ceil(8 c_b / max c), 1, 8).
 */
WSMC_HD double wsmc_linspace_edge(double lo, double hi, int k, int n) {
    if (k == 0) return lo;
    if (k == n) return hi;
    /* hi - lo = d + e exactly (TwoSum) */
    const double d = hi - lo;
    const double bb = d - hi;
    const double e = (hi - (d - bb)) + (-lo - bb);
    /* k (d + e) / n: k d exactly as p + pe (fma), then / n (n a power of two: exact) */
    const double p = (double)k * d;
    const double pe = __builtin_fma((double)k, d, -p);
    const double inv = 1.0 / (double)n;
    const double s_hi = p * inv, s_lo = (pe + (double)k * e) * inv;
    /* lo + s_hi + s_lo, rounded once (TwoSum of lo + s_hi, then the tails) */
    const double t = lo + s_hi;
    const double tb = t - lo;
    const double te = (lo - (t - tb)) + (s_hi - tb);
    return t + (te + s_lo);
}
WSMC_HD int wsmc_hist_bin(double v, const double* edges, int nbins) {
    int c = 0;                                   /* searchsortedlast: #edges <= v */
    for (int k = 0; k <= nbins; ++k) c += edges[k] <= v;
    return c < 1 ? 0 : (c > nbins ? nbins - 1 : c - 1);   /* 0-based, clamped */
}
WSMC_HD int wsmc_spark_level(uint64_t c, uint64_t maxc) {
    if (maxc == 0) return 1;
    const wsmc_u128 num = (wsmc_u128)c * 8u + (maxc - 1);
    int l = (int)(num / maxc);
    return l < 1 ? 1 : (l > 8 ? 8 : l);
}
/* the median's last step: vkold + (h - Skold) / (Sk - Skold) * (vk - vkold), with
 * h - Skold = (Q + q1 - 2 Skold) / 2 */
WSMC_HD double wsmc_median_interp(double vkold, double vk, uint64_t Q, uint64_t q1, uint64_t Skold, uint64_t wk) {
    const wsmc_u128 num = (wsmc_u128)Q + q1 - 2 * (wsmc_u128)Skold;
    const double f = wsmc_u128_to_d(num) / (2.0 * wsmc_u64_to_d(wk));
    return vkold + f * (vk - vkold);
}

/* 4x4-max Cholesky of a symmetric matrix (row-major a[d*d]) -> lower L; 0 if not PD */
WSMC_HD int wsmc_cholesky(const double* a, double* L, int d) {
    for (int i = 0; i < d * d; ++i) L[i] = 0.0;
    for (int j = 0; j < d; ++j) {
        double s = a[j * d + j];
        for (int k = 0; k < j; ++k) s -= L[j * d + k] * L[j * d + k];
        if (!(s > 0.0)) return 0;
        double ljj = wsmc_sqrt(s);
        L[j * d + j] = ljj;
        for (int i = j + 1; i < d; ++i) {
            double t = a[i * d + j];
            for (int k = 0; k < j; ++k) t -= L[i * d + k] * L[j * d + k];
            L[i * d + j] = t / ljj;
        }
    }
    return 1;
}

/*
 * autoRW's proposal factor from one pass over the particles (src/move_kernels.jl:144-151;
 * StatsBase's cov(Z, ProbabilityWeights(w)) with corrected = false, i.e. the weighted
 * covariance Σ w_i (z_i - z̄)(z_i - z̄)ᵀ / Σ w_i). With e_i = exp(w_i - M) and the values taken
 * relative to a pivot p (one particle's values, so the shift is of the order of the spread
 * and the subtraction below loses nothing measurable), the canonical totals are
 *   tot[0] = Σ e_i,  tot[1 + k] = Σ e_i d_ik,  tot[1 + d + v] = Σ (e_i d_ia) d_ib (a <= b),
 * d_ik = z_ik - p_k, and the covariance is S_ab = tot2_ab / T0 - (tot1_a / T0)(tot1_b / T0)
 * (shift-invariant). Then zero entries -> min_step, times 2.38/sqrt(d), Cholesky.
 * S (the scaled covariance) and L are row-major d x d; returns 0 if not positive definite.
 */
WSMC_HD int wsmc_autorw_factor(const double* tot, int d, double min_step, double* S, double* L) {
    const double T0 = tot[0];
    double m[4];
    for (int k = 0; k < d; ++k) m[k] = tot[1 + k] / T0;
    int v = 0;
    for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b) {
            const double c = tot[1 + d + v] / T0 - m[a] * m[b];
            S[a * d + b] = c;
            S[b * d + a] = c;
            ++v;
        }
    const double lam = 2.38 / wsmc_sqrt((double)d);
    for (int k = 0; k < d * d; ++k) {
        if (S[k] == 0.0) S[k] = min_step;          /* Σ[Σ .== 0] .= min_step */
        S[k] = lam * S[k];
    }
    return wsmc_cholesky(S, L, d);
}

/*
 * Per-shard weight statistics and the global Resample decision
 * (src/transformers.jl:479-489). G = 1 is the single-GPU case; G > 1 combines shard
 * records in rank order (island resampling). Shared by oracle and kernels.
 */
typedef struct {
    double M;          /* shard max log-weight (NaN if any NaN); the sums are against wsmc_qref(M) */
    uint64_t Q;        /* sum q_i */
    uint64_t Q2;       /* sum q2_i */
    wsmc_u128 Wf2;     /* sum wf2_i (sum floor(e_i^2 2^(K+42)) = Q2 2^42 + Wf2) */
    wsmc_u128 Wf;      /* sum wf_i  (sum floor(e_i 2^(K+42)) = Q 2^42 + Wf) */
    uint64_t n;        /* shard size */
} wsmc_shard_stats;

/* sum exp(lw_i - R) of one shard (R = wsmc_qref(M)), from its fixed point sum floor(e 2^(K+42)) */
WSMC_HD double wsmc_shard_expsum(const wsmc_shard_stats* s) {
    int K = wsmc_qbits(s->n);
    wsmc_u128 W = ((wsmc_u128)s->Q << 42) + s->Wf;
    return wsmc_u128_to_d(W) * wsmc_pow2i(-(K + 42));
}
/* sum exp(lw_i - R)^2 of one shard, from its fixed point Q2 2^42 + Wf2 */
WSMC_HD double wsmc_shard_expsum2(const wsmc_shard_stats* s) {
    int K = wsmc_qbits(s->n);
    wsmc_u128 W = ((wsmc_u128)s->Q2 << 42) + s->Wf2;
    return wsmc_u128_to_d(W) * wsmc_pow2i(-(K + 42));
}
/* A flat shard: every particle's fixed point floor(e 2^(K+42)) equals the max particle's, i.e.
 * sum = n * (the max's), since no term exceeds the max's. Its weights are equal (to within the
 * resolution of expw), so its ESS is exactly 1 and its log-mean is M itself, as with e = 1 exactly
 * (the reference point R = ceil(M) makes the common e < 1, and the f64 ratio of the two sums
 * would otherwise round either way of 1). */
WSMC_HD int wsmc_shard_flat(const wsmc_shard_stats* s) {
    if (!(s->M - s->M == 0.0) || s->n == 0) return 0;
    const wsmc_qparts p = wsmc_qparts_of(s->M, wsmc_qref(s->M), wsmc_qbits(s->n));
    const wsmc_u128 a = ((wsmc_u128)p.q << 42) + p.wf;
    return ((wsmc_u128)s->Q << 42) + s->Wf == (wsmc_u128)s->n * a;
}
/* every shard flat at one common max: the population's weights are all equal */
WSMC_HD int wsmc_all_flat(const wsmc_shard_stats* st, int G) {
    for (int g = 0; g < G; ++g)
        if (!wsmc_shard_flat(&st[g]) || st[g].M != st[0].M) return 0;
    return G > 0;
}
/* ess_perc = 1 / (N sum w^2), w = exp_norm(weights) (src/resampling.jl:51-54), i.e.
 * (sum e)^2 / (N sum e^2), over every shard's fixed-point sums rescaled by exp(R_g - R) (rank
 * order; R_g - R is an integer). All-equal weights give exactly 1. */
WSMC_HD double wsmc_global_ess(const wsmc_shard_stats* st, int G) {
    if (wsmc_all_flat(st, G)) return 1.0;
    double R = -WSMC_INF;
    uint64_t N = 0;
    int nan = 0;
    for (int g = 0; g < G; ++g) {
        const double Rg = wsmc_qref(st[g].M);
        if (wsmc_isnan(Rg)) nan = 1;
        else if (Rg > R) R = Rg;
        N += st[g].n;
    }
    if (nan) R = WSMC_NAN;
    double s1 = 0.0, s2 = 0.0;
    for (int g = 0; g < G; ++g) {
        double f = wsmc_exp(wsmc_qref(st[g].M) - R);
        s1 = s1 + wsmc_shard_expsum(&st[g]) * f;
        s2 = s2 + wsmc_shard_expsum2(&st[g]) * (f * f);
    }
    return (s1 * s1) / (wsmc_u64_to_d(N) * s2);
}
/* logsumexp(shard weights) - log(n): the value every weight is reset to (src/transformers.jl:486-489);
 * a flat shard's sum is n exactly against M */
WSMC_HD double wsmc_shard_mean(const wsmc_shard_stats* s) {
    const double ln = wsmc_log(wsmc_u64_to_d(s->n));
    if (wsmc_shard_flat(s)) return (s->M + ln) - ln;
    return (wsmc_qref(s->M) + wsmc_log(wsmc_shard_expsum(s))) - ln;
}
/* logsumexp(all weights) - log(N)  (src/utils.jl:21) */
WSMC_HD double wsmc_global_log_evidence(const wsmc_shard_stats* st, int G) {
    uint64_t N = 0;
    for (int g = 0; g < G; ++g) N += st[g].n;
    const double lN = wsmc_log(wsmc_u64_to_d(N));
    if (wsmc_all_flat(st, G)) return (st[0].M + lN) - lN;
    double R = -WSMC_INF;
    for (int g = 0; g < G; ++g) {
        const double Rg = wsmc_qref(st[g].M);
        if (Rg > R || wsmc_isnan(Rg)) R = Rg;
    }
    double S = 0.0;
    for (int g = 0; g < G; ++g) S = S + wsmc_shard_expsum(&st[g]) * wsmc_exp(wsmc_qref(st[g].M) - R);
    return (R + wsmc_log(S)) - lN;
}

#endif /* WSMC_MATH_H */
