// stage.cpp — host side of the sampler paths -> HBM staging.
//
// The reference concatenates every path's f64 observations (npg_cg.py:87-89) and
// the policy casts them to f32 on every forward (gaussian_mlp.py:103).  Staging
// does that cast once, on the host thread pool, straight into a pinned slab, and
// takes each column's range in the same pass: the split rows' column scales then
// need no device pass over the batch (mjrl_obs_colscale_range), and the pack of a
// chunk never waits for a whole-batch reduction on the device.
//
// Host-only C++ (g++), built into its own library lib/libmjrl_stage.so (the pool
// controller and the staging threads never load the HIP library) and linked into
// libmjrl_amd.so too, which exports the whole C ABI.  Two code paths, chosen at
// run time (no -m flag ties the library to one CPU):
//   AVX-512 (Zen 4/5, Xeon): per block of rows (32 KB of f32), strip by strip of
//     192 columns, each 16-column chunk is converted (two masked 8 x f64 loads ->
//     one 16 x f32 vector), folded into the strip's column range held in
//     registers across the block's rows (min / max, NaN skipped: vminps returns
//     its second operand when either is NaN) and written to an L1/L2-resident
//     block buffer; the block, which is contiguous in the slab, then leaves with
//     non-temporal 64-byte stores.  Round 4's scalar-typed loop did cached stores:
//     every written line was first read from DRAM (read-for-ownership) and the
//     slab displaced the source from the caches, so the conversion, not the PCIe
//     copy, set the end-to-end time.
//   portable: the same one-pass loop, auto-vectorised for the build's baseline ISA.
#include <cmath>
#include <cstdint>
#include <cstring>

#include <immintrin.h>

#include "../../include/mjrl_amd.h"

namespace {

template <typename S>
__attribute__((always_inline)) inline int portable_body(const S* __restrict__ src, int64_t rows, int32_t n,
                                                        float* __restrict__ dst, float* __restrict__ cmin,
                                                        float* __restrict__ cmax) {
    const int64_t ne = rows * (int64_t)n;
    if (!cmin) {
        for (int64_t i = 0; i < ne; ++i) dst[i] = (float)src[i];
        return MJRL_OK;
    }
    for (int64_t r = 0; r < rows; ++r) {
        const S* __restrict__ s = src + r * n;
        float* __restrict__ d = dst + r * n;
        for (int32_t k = 0; k < n; ++k) {
            const float v = (float)s[k];
            d[k] = v;
            const float lo = cmin[k], hi = cmax[k];
            cmin[k] = v < lo ? v : lo;   // a NaN compares false: skipped
            cmax[k] = v > hi ? v : hi;
        }
    }
    return MJRL_OK;
}

// the loop auto-vectorised for the build's baseline ISA (SSE2), and again for AVX2
// hosts without AVX-512 (Zen 2 / 3), chosen at run time like the AVX-512 path
template <typename S>
int stage_portable(const S* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    return portable_body(src, rows, n, dst, cmin, cmax);
}
template <typename S>
__attribute__((target("avx2,fma"))) int stage_portable_avx2(const S* src, int64_t rows, int32_t n, float* dst,
                                                            float* cmin, float* cmax) {
    return portable_body(src, rows, n, dst, cmin, cmax);
}

bool have_avx2() {
    static const int ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    return ok;
}

// LinearBaseline extras of the f64 pass (baselines/linear_baseline.py:10-18, 46-49):
// pred[r] = [clip(x_r, +-10), a, a^2, a^3, 1] . coeffs (a = r / 1000, the row's index in
// its path) in fp64 from the sampler's own values, and a flag raised when a value
// is not a float32 (its f32 image then differs from what the reference reads).
struct Extras {
    const double* coeffs;   // n + 4, or null (no prediction)
    double* pred;           // rows, or null
    int32_t* inexact;       // set to 1 on the first value with (double)(float)x != x, or null
};

inline double clip10(double x) {   // np.clip(x, -10, 10): NaN stays NaN
    return x < -10.0 ? -10.0 : (x > 10.0 ? 10.0 : x);
}

inline double time_terms(int64_t r, const double* c, int32_t n) {
    const double a = (double)r / 1000.0;   // np.arange(l) / 1000.0
    return a * c[n] + (a * a) * c[n + 1] + std::pow(a, 3.0) * c[n + 2] + c[n + 3];
}

// One row s (n values, index t in its path): its prediction when c is given (else
// 0), and whether any value is not a float32.  Every staging entry point computes
// a row's prediction through the row function of the CPU's path (row_extras), so
// the block pass, the per-row pass of the streaming sink and the tests agree bit
// for bit.
inline double row_extras_portable(const double* __restrict__ s, int64_t t, int32_t n, const double* c, bool& bad) {
    double acc = 0.0;
    for (int32_t k = 0; k < n; ++k) {
        const double v = s[k];
        bad |= !((double)(float)v == v);
        if (c) acc += clip10(v) * c[k];
    }
    return c ? acc + time_terms(t, c, n) : 0.0;
}

int extras_portable(const double* __restrict__ src, int64_t rows, int32_t n, const Extras& x) {
    bool bad = false;
    for (int64_t r = 0; r < rows; ++r) {
        const double p = row_extras_portable(src + r * n, r, n, x.coeffs, bad);
        if (x.pred) x.pred[r] = p;
    }
    if (bad && x.inexact) *x.inexact = 1;
    return MJRL_OK;
}

#define MJRL_AVX512 __attribute__((target("avx512f,avx512vl,avx512dq,avx512bw")))

MJRL_AVX512 inline __m512 load16(const double* p, __mmask16 m) {
    const __m256 lo = _mm512_cvtpd_ps(_mm512_maskz_loadu_pd((__mmask8)(m & 0xff), p));
    const __m256 hi = _mm512_cvtpd_ps(_mm512_maskz_loadu_pd((__mmask8)(m >> 8), p + 8));
    return _mm512_insertf32x8(_mm512_castps256_ps512(lo), hi, 1);
}
MJRL_AVX512 inline __m512 load16(const float* p, __mmask16 m) { return _mm512_maskz_loadu_ps(m, p); }

// `count` floats from an L1/L2-resident buffer to dst with non-temporal stores
// (64-byte aligned body; head and tail with masked ordinary stores)
MJRL_AVX512 inline void stream_out(float* dst, const float* buf, int64_t count) {
    int64_t i = 0;
    const int64_t mis = (int64_t)(reinterpret_cast<uintptr_t>(dst) & 63) / 4;
    if (reinterpret_cast<uintptr_t>(dst) & 3) {   // not even float aligned: ordinary stores throughout
        std::memcpy(dst, buf, count * sizeof(float));
        return;
    }
    if (mis) {
        const int64_t h = 16 - mis < count ? 16 - mis : count;
        const __mmask16 m = (__mmask16)((1u << h) - 1);
        _mm512_mask_storeu_ps(dst, m, _mm512_maskz_loadu_ps(m, buf));
        i = h;
    }
    for (; i + 16 <= count; i += 16) _mm512_stream_ps(dst + i, _mm512_loadu_ps(buf + i));
    if (i < count) {
        const __mmask16 m = (__mmask16)((1u << (count - i)) - 1);
        _mm512_mask_storeu_ps(dst + i, m, _mm512_maskz_loadu_ps(m, buf + i));
    }
}

// One column strip [c0, c0 + 16 NCH) of rows r0 .. r1 - 1: converted into the block
// buffer, the strip's range kept in 2 NCH registers across the rows
template <typename S, bool RANGE, int NCH>
MJRL_AVX512 inline void strip(const S* __restrict__ src, int64_t r0, int64_t r1, int32_t n, int c0, int nc,
                              __mmask16 tail, float* __restrict__ buf, float* __restrict__ cmin,
                              float* __restrict__ cmax) {
    __m512 lo[NCH], hi[NCH];
    __mmask16 mk[NCH];
#pragma GCC unroll 16
    for (int j = 0; j < NCH; ++j) {
        const int c = c0 / 16 + j;
        mk[j] = c < nc ? (c + 1 < nc ? (__mmask16)0xffff : tail) : (__mmask16)0;
        if (RANGE) {
            lo[j] = _mm512_maskz_loadu_ps(mk[j], cmin + 16 * c);
            hi[j] = _mm512_maskz_loadu_ps(mk[j], cmax + 16 * c);
        }
    }
    for (int64_t r = r0; r < r1; ++r) {
        const S* s = src + r * n + c0;
        float* b = buf + (r - r0) * n + c0;
#pragma GCC unroll 16
        for (int j = 0; j < NCH; ++j) {
            const __m512 v = load16(s + 16 * j, mk[j]);
            _mm512_mask_storeu_ps(b + 16 * j, mk[j], v);
            if (RANGE) {
                // vminps / vmaxps return the SECOND operand when either is NaN:
                // (v, range) keeps the range for a NaN value, and for a -0.0 / 0.0 tie
                lo[j] = _mm512_min_ps(v, lo[j]);
                hi[j] = _mm512_max_ps(v, hi[j]);
            }
        }
    }
    if (RANGE) {
#pragma GCC unroll 16
        for (int j = 0; j < NCH; ++j) {
            const int c = c0 / 16 + j;
            _mm512_mask_storeu_ps(cmin + 16 * c, mk[j], lo[j]);
            _mm512_mask_storeu_ps(cmax + 16 * c, mk[j], hi[j]);
        }
    }
}

// The extras of rows r0 .. r1 - 1, right after the strips converted them: the
// block's source (rb rows, ~64 KB) is still in the core's L2, so this second look
// at it costs no DRAM traffic.  8 doubles per step: the float round trip compared
// with the value (NEQ_UQ: a NaN counts as inexact), clip as max(-10, x) then
// min(10, .) with x the SECOND operand of each (vmaxpd / vminpd return it when
// either is NaN: NaN stays NaN, as np.clip), fused multiply-add with the coefficients.
MJRL_AVX512 double row_extras_avx512(const double* __restrict__ s, int64_t t, int32_t n, const double* c,
                                     __mmask8& bad) {
    const __m512d lo = _mm512_set1_pd(-10.0), hi = _mm512_set1_pd(10.0);
    __m512d acc = _mm512_setzero_pd();
    for (int32_t k = 0; k < n; k += 8) {
        const __mmask8 m = n - k >= 8 ? (__mmask8)0xff : (__mmask8)((1u << (n - k)) - 1);
        const __m512d v = _mm512_maskz_loadu_pd(m, s + k);
        bad |= _mm512_cmp_pd_mask(_mm512_cvtps_pd(_mm512_cvtpd_ps(v)), v, _CMP_NEQ_UQ);
        if (c) acc = _mm512_fmadd_pd(_mm512_min_pd(hi, _mm512_max_pd(lo, v)), _mm512_maskz_loadu_pd(m, c + k), acc);
    }
    return c ? _mm512_reduce_add_pd(acc) + time_terms(t, c, n) : 0.0;
}

MJRL_AVX512 void extras_avx512(const double* __restrict__ src, int64_t r0, int64_t r1, int32_t n, const Extras& x) {
    __mmask8 bad = 0;
    for (int64_t r = r0; r < r1; ++r) {
        const double p = row_extras_avx512(src + r * n, r, n, x.coeffs, bad);
        if (x.pred) x.pred[r] = p;
    }
    if (bad && x.inexact) *x.inexact = 1;
}

template <typename S, bool RANGE>
MJRL_AVX512 int stage_avx512(const S* __restrict__ src, int64_t rows, int32_t n, float* __restrict__ dst,
                             float* __restrict__ cmin, float* __restrict__ cmax, const Extras* xt = nullptr) {
    constexpr int BUF = 8192;   // floats of the block buffer (32 KB: stays in L1 / L2)
    constexpr int NCH = 12;     // 16-column chunks per strip: 24 range registers of the 32
    alignas(64) float buf[BUF + 16];
    const int64_t rb = n <= BUF ? BUF / n : 0;
    if (rb == 0) {
        if constexpr (sizeof(S) == 8)
            if (xt) extras_portable(src, rows, n, *xt);
        return stage_portable(src, rows, n, dst, cmin, cmax);
    }
    const int nc = (n + 15) / 16;
    const __mmask16 tail = (__mmask16)(n % 16 ? (1u << (n % 16)) - 1 : 0xffff);
    for (int64_t r0 = 0; r0 < rows; r0 += rb) {
        const int64_t r1 = r0 + rb < rows ? r0 + rb : rows;
        // the next block's source lines requested now (one contiguous run of rb
        // rows), so the strips below find them in L2: the strips' short strided
        // pieces (rb rows x 192 columns) are not a stream the hardware prefetcher
        // follows
        if (r1 < rows) {
            const char* p = reinterpret_cast<const char*>(src + r1 * n);
            const int64_t nb = ((r1 + rb < rows ? r1 + rb : rows) - r1) * n * (int64_t)sizeof(S);
            for (int64_t o = 0; o < nb; o += 64) _mm_prefetch(p + o, _MM_HINT_T1);
        }
        // strip by strip over the block: the block's source (rb rows) stays in the
        // core's caches between strips, the ranges in registers within one
        for (int c0 = 0; c0 < n; c0 += 16 * NCH) strip<S, RANGE, NCH>(src, r0, r1, n, c0, nc, tail, buf, cmin, cmax);
        if constexpr (sizeof(S) == 8)
            if (xt) extras_avx512(src, r0, r1, n, *xt);
        stream_out(dst + r0 * n, buf, (r1 - r0) * n);
    }
    _mm_sfence();   // the streamed lines are globally visible before the caller's H2D copy
    return MJRL_OK;
}

bool have_avx512() {
    static const int ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                          __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("avx512bw");
    return ok;
}

template <typename S>
int stage_rows(const S* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax,
               const Extras* xt = nullptr) {
    if (rows < 0 || n <= 0 || (rows > 0 && (!src || !dst))) return MJRL_EINVAL;
    if ((cmin == nullptr) != (cmax == nullptr)) return MJRL_EINVAL;
    if (rows == 0) return MJRL_OK;
    if (have_avx512())
        return cmin ? stage_avx512<S, true>(src, rows, n, dst, cmin, cmax, xt)
                    : stage_avx512<S, false>(src, rows, n, dst, cmin, cmax, xt);
    if constexpr (sizeof(S) == 8)
        if (xt) extras_portable(src, rows, n, *xt);
    return have_avx2() ? stage_portable_avx2(src, rows, n, dst, cmin, cmax) : stage_portable(src, rows, n, dst, cmin, cmax);
}

// lo = float(x - double(float(x))): with hi = float(x), hi + lo carries x to 2^-48
// relative (x - hi is exact in f64; its float rounding keeps 24 of its <= 29 bits).
// A value past the float range (hi = +-inf) gets lo = 0, so hi + lo stays the
// infinity the clip at +-10 maps to the same feature; NaN stays NaN.
int stage_lo_rows(const double* __restrict__ src, int64_t rows, int32_t n, float* __restrict__ dst) {
    if (rows < 0 || n <= 0 || (rows > 0 && (!src || !dst))) return MJRL_EINVAL;
    const int64_t ne = rows * (int64_t)n;
    for (int64_t i = 0; i < ne; ++i) {
        const double v = src[i];
        const float h = (float)v;
        dst[i] = std::isinf(h) ? 0.0f : (float)(v - (double)h);
    }
    return MJRL_OK;
}

}  // namespace

extern "C" {

int mjrl_host_stage_f64(const double* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    return stage_rows(src, rows, n, dst, cmin, cmax);
}

int mjrl_host_stage_f32(const float* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    return stage_rows(src, rows, n, dst, cmin, cmax);
}

// `count` row-major arrays (srcs[i]: rows[i] x n) converted one after another into
// dst, one call per chunk of paths instead of one per path (a path of the action
// slot is 17 x 1000 values: per-call overhead, not bandwidth, set its time).
int mjrl_host_stage_paths_f64(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n, float* dst,
                              float* cmin, float* cmax) {
    if (count < 0 || (count > 0 && (!srcs || !rows))) return MJRL_EINVAL;
    for (int32_t i = 0; i < count; ++i) {
        const int rc = stage_rows(srcs[i], rows[i], n, dst, cmin, cmax);
        if (rc != MJRL_OK) return rc;
        dst += rows[i] * (int64_t)n;
    }
    return MJRL_OK;
}

// mjrl_host_stage_paths_f64 with the LinearBaseline extras: the first npred arrays
// (the RL paths of the chunk; demonstration paths follow them) get their fp64
// predictions written one after another into pred when coeffs is given, and
// *inexact is set to 1 when any value of the chunk is not a float32.
int mjrl_host_stage_paths_f64x(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n, float* dst,
                               float* cmin, float* cmax, const double* coeffs, double* pred, int32_t npred,
                               int32_t* inexact) {
    if (count < 0 || (count > 0 && (!srcs || !rows))) return MJRL_EINVAL;
    if ((coeffs == nullptr) != (pred == nullptr) || npred < 0) return MJRL_EINVAL;
    for (int32_t i = 0; i < count; ++i) {
        const Extras xt{i < npred ? coeffs : nullptr, i < npred ? pred : nullptr, inexact};
        const int rc = stage_rows(srcs[i], rows[i], n, dst, cmin, cmax, &xt);
        if (rc != MJRL_OK) return rc;
        dst += rows[i] * (int64_t)n;
        if (i < npred && pred) pred += rows[i];
    }
    return MJRL_OK;
}

// The low halves of `count` f64 arrays (stage_lo_rows), one after another into dst:
// with the f32 rows of the pass above, the device LinearBaseline fit reads every
// observation to 2^-48 (mjrl_linear_baseline_gram_f32x2).
int mjrl_host_stage_lo_paths_f64(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n,
                                 float* dst) {
    if (count < 0 || (count > 0 && (!srcs || !rows))) return MJRL_EINVAL;
    for (int32_t i = 0; i < count; ++i) {
        const int rc = stage_lo_rows(srcs[i], rows[i], n, dst);
        if (rc != MJRL_OK) return rc;
        dst += rows[i] * (int64_t)n;
    }
    return MJRL_OK;
}

// Rows that are not contiguous in their destination (the streaming sink of the
// vectorised sampler: one row per environment per step, each to its trajectory's
// pinned slab): row i of src goes to dst_rows[i] as f32, folded into the column
// ranges, with its prediction at path index tidx[i] (when coeffs is given) and
// the exactness flag, through the same per-row arithmetic as the block pass.
int mjrl_host_stage_rows_f64x(const double* src, int64_t rows, int32_t n, float* const* dst_rows, float* cmin,
                              float* cmax, const double* coeffs, const int64_t* tidx, double* pred,
                              int32_t* inexact) {
    if (rows < 0 || n <= 0 || (rows > 0 && (!src || !dst_rows))) return MJRL_EINVAL;
    if ((cmin == nullptr) != (cmax == nullptr) || (coeffs == nullptr) != (pred == nullptr)) return MJRL_EINVAL;
    if (coeffs && !tidx) return MJRL_EINVAL;
    const bool vec = have_avx512();
    bool bad = false;
    __mmask8 badv = 0;
    for (int64_t i = 0; i < rows; ++i) {
        const double* s = src + i * n;
        float* d = dst_rows[i];
        if (!d) return MJRL_EINVAL;
        for (int32_t k = 0; k < n; ++k) {
            const float v = (float)s[k];
            d[k] = v;
            if (cmin) {
                const float lo = cmin[k], hi = cmax[k];
                cmin[k] = v < lo ? v : lo;   // a NaN compares false: skipped (as the block pass)
                cmax[k] = v > hi ? v : hi;
            }
        }
        const int64_t t = tidx ? tidx[i] : 0;
        const double p = vec ? row_extras_avx512(s, t, n, coeffs, badv) : row_extras_portable(s, t, n, coeffs, bad);
        if (pred) pred[i] = p;
    }
    if ((bad || badv) && inexact) *inexact = 1;
    return MJRL_OK;
}

// The extras alone through the portable loop, whatever the CPU (tests compare the paths).
int mjrl_host_extras_portable(const double* src, int64_t rows, int32_t n, const double* coeffs, double* pred,
                              int32_t* inexact) {
    if (rows < 0 || n <= 0 || (rows > 0 && !src) || (coeffs == nullptr) != (pred == nullptr)) return MJRL_EINVAL;
    return extras_portable(src, rows, n, Extras{coeffs, pred, inexact});
}

// The portable loop, callable whatever the CPU (tests compare the two paths).
int mjrl_host_stage_f64_portable(const double* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    if (rows < 0 || n <= 0 || (rows > 0 && (!src || !dst))) return MJRL_EINVAL;
    if ((cmin == nullptr) != (cmax == nullptr)) return MJRL_EINVAL;
    return stage_portable(src, rows, n, dst, cmin, cmax);
}

int mjrl_host_stage_avx512(void) { return have_avx512() ? 1 : 0; }

// The 1-D slots of a chunk (rewards, advantages, host predictions): np.concatenate
// over a chunk's 125 reward arrays held the GIL across its per-array work, so the
// staging threads ran those chunks one at a time (3.9 ms for the 8 MB of a 1M-row
// batch, profiles/r05d/stage_probe4.txt); a native call releases it.
int mjrl_host_gather(const void* const* srcs, const int64_t* nbytes, int32_t count, void* dst) {
    if (count < 0 || (count > 0 && (!srcs || !nbytes || !dst))) return MJRL_EINVAL;
    char* d = static_cast<char*>(dst);
    for (int32_t i = 0; i < count; ++i) {
        if (nbytes[i] < 0 || (nbytes[i] > 0 && !srcs[i])) return MJRL_EINVAL;
        if (nbytes[i]) std::memcpy(d, srcs[i], (size_t)nbytes[i]);
        d += nbytes[i];
    }
    return MJRL_OK;
}

}  // extern "C"
