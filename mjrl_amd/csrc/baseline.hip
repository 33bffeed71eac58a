// baseline.hip — LinearBaseline.fit and QuadraticBaseline.fit on the device (SURVEY.md
// §8f row f1).
//
// Reference: mjrl/baselines/linear_baseline.py:10-44.  fit() builds the feature
// matrix F = [clip(obs, +-10), a, a^2, a^3, 1] (a = index within the path / 1000)
// and solves (F^T F + reg I) c = F^T y by lstsq, retrying with 10x reg on NaN.
// The T x k products are the whole cost (Humanoid 1M: k = 380, 2 T k^2 = 289
// GFLOP fp64); the k x k solve stays on the host, exactly as the reference runs it.
//
// Observations staged as f32 rows can come with their low halves (an f32 pair,
// hi + lo = the sampler's f64 value to 2^-48): the features are then formed from
// both, so the fit is the reference's on observations that are not float32s.
//
// k_gram computes the Gram matrix of the augmented rows [f_t, y_t] (k+1 = n+5
// columns: F^T F, F^T y and y^T y in one pass) with v_mfma_f64_16x16x4_f64:
//   - output 64 x 64 tiles of the upper triangle; workgroup = 4 waves, each wave
//     a 32 x 32 quarter (2 x 2 MFMA tiles, 16 f64 accumulators per lane);
//   - split-K over row slices (fixed slice count), slabs reduced in slice order
//     by k_gram_reduce (deterministic, no atomics);
//   - features are built on the fly from obs (HBM read once per XCD: the pair
//     tiles of one row slice are mapped to the same XCD so they share its L2);
//   - 32-row chunks double-buffered through LDS, the next chunk's loads in
//     registers while the current one is multiplied.
//
// QuadraticBaseline (quadratic_baseline.py:10-65) runs the same Gram with its own
// features, o = clip(obs, +-10) / 10: [o, o_i o_j (i <= j, row-major), 1, a, a^2,
// a^3, a^4] (n + n(n+1)/2 + 5 columns, n <= 64): o is formed once per value by
// k_quad_obs (the f64 division off the Gram's loaders), each loader thread decodes
// its eight columns of each panel once per launch (QCol) and forms them per row.
#include <math.h>

#include "common.h"

using namespace mjrl;

namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));

constexpr int GT = 64;          // output tile
constexpr int GRC = 32;         // rows per chunk
constexpr int GLD = GT + 16;    // LDS row stride (doubles): rows 1 apart land 32 banks apart
constexpr int GSLICES = 24;     // row slices (multiple of 8: one XCD per slice group)
constexpr int GTHREADS = 256;

// a_t = (t - path start) / 1000 for every row (np.arange(l) / 1000.0); one wave per path
__global__ void __launch_bounds__(256) k_path_time(const int64_t* __restrict__ off, int64_t P,
                                                   double* __restrict__ al) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < P; p += nw) {
        const int64_t b = off[p], e = off[p + 1];
        for (int64_t t = b + lane; t < e; t += 64) al[t] = (double)(t - b) / 1000.0;
    }
}

// observation k of row `row` in fp64: the staged value, or hi + lo for an f32 pair
// (the low halves of mjrl_host_stage_lo_paths_f64; lo is null otherwise)
template <typename TO>
__device__ __forceinline__ double obs_at(const TO* __restrict__ obs, const float* __restrict__ lo, int64_t i) {
    return lo ? (double)obs[i] + (double)lo[i] : (double)obs[i];
}

// feature g of row `row` (linear_baseline.py:10-18), the return as feature n + 4, zero pad
template <typename TO>
__device__ __forceinline__ double feat(const TO* __restrict__ obs, const float* __restrict__ lo,
                                       const double* __restrict__ y, const double* __restrict__ al, int64_t row,
                                       int g, int n) {
    if (g < n) {
        const double o = obs_at(obs, lo, row * n + g);
        return o < -10.0 ? -10.0 : (o > 10.0 ? 10.0 : o);
    }
    const double a = al[row];
    switch (g - n) {
        case 0: return a;
        case 1: return a * a;
        case 2: return pow(a, 3.0);
        case 3: return 1.0;
        case 4: return y[row];
        default: return 0.0;
    }
}

// QuadraticBaseline column g (quadratic_baseline.py:10-37) as (kind, i, j); the
// augmented Gram appends the return as column n + nq + 5
// (kind, i, j) packed in one int (kind << 16 | i << 8 | j; n <= 64): the loader's
// sixteen decoded columns stay in sixteen registers
enum QKind { Q_LIN, Q_QUAD, Q_ONE, Q_A1, Q_A2, Q_A3, Q_A4, Q_Y, Q_ZERO };
typedef int QCol;
__device__ __forceinline__ QCol qpack(int kind, int i, int j) { return kind << 16 | i << 8 | j; }
__device__ __forceinline__ QCol qcol(int g, int n) {
    const int nq = n * (n + 1) / 2;
    if (g < n) return qpack(Q_LIN, g, 0);
    if (g < n + nq) {
        int r = g - n, i = 0;
        while (r >= n - i) {   // row i of the upper triangle holds n - i products
            r -= n - i;
            ++i;
        }
        return qpack(Q_QUAD, i, i + r);
    }
    const int t = g - n - nq;
    return qpack(t <= 5 ? Q_ONE + t : Q_ZERO, 0, 0);
}

// o = clip(obs, +-10) / 10 (quadratic_baseline.py:12)
template <typename TO>
__device__ __forceinline__ double qobs(const TO* __restrict__ obs, const float* __restrict__ lo, int64_t i) {
    const double o = obs_at(obs, lo, i);
    return (o < -10.0 ? -10.0 : (o > 10.0 ? 10.0 : o)) / 10.0;
}

template <typename TO>
__global__ void __launch_bounds__(256) k_quad_obs(const TO* __restrict__ obs, const float* __restrict__ lo, int64_t N,
                                                  double* __restrict__ o) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) o[i] = qobs(obs, lo, i);
}

// the row's time features (quadratic_baseline.py:31-35): al ** 1 (numpy: the value
// itself), al ** 2 (numpy: square), al ** 3 and al ** 4 (C pow), once per row
struct QTime {
    double a1, a2, a3, a4;
};
__device__ __forceinline__ QTime qtime(const double* __restrict__ al, int64_t row) {
    const double a = al[row];
    return {a, a * a, pow(a, 3.0), pow(a, 4.0)};
}

// column c of row `row` from o = clip(obs, +-10) / 10 formed beforehand (k_quad_obs:
// the f64 divisions once per value, not once per product)
__device__ __forceinline__ double qfeat(const double* __restrict__ o, const double* __restrict__ y,
                                        const QTime& tm, int64_t row, QCol c, int n) {
    const int ci = (c >> 8) & 0xff, cj = c & 0xff;
    switch (c >> 16) {
        case Q_LIN: return o[row * n + ci];
        case Q_QUAD: return o[row * n + ci] * o[row * n + cj];
        case Q_ONE: return 1.0;
        case Q_A1: return tm.a1;
        case Q_A2: return tm.a2;
        case Q_A3: return tm.a3;
        case Q_A4: return tm.a4;
        case Q_Y: return y[row];
        default: return 0.0;
    }
}

template <typename TO>
struct GramArgs {
    const TO* obs;
    const float* lo;   // low halves of an f32 pair, or null
    const double* y;
    const double* al;
    int64_t T;
    int n, ntile, npair;
    double* slab;   // [GSLICES][npair][GT][GT]
};

template <typename TO, bool QUAD>
__global__ void __launch_bounds__(GTHREADS, 2) k_gram(GramArgs<TO> a) {
    __shared__ __attribute__((aligned(16))) double PI[2][GRC][GLD];
    __shared__ __attribute__((aligned(16))) double PJ[2][GRC][GLD];
    // block -> (slice, pair): the npair blocks of a slice sit on one XCD (b % 8)
    const int b = blockIdx.x, xcd = b & 7, loc = b >> 3;
    const int slice = (loc / a.npair) * 8 + xcd, pair = loc % a.npair;
    if (slice >= GSLICES) return;
    int ti = 0, rem = pair;
    while (rem >= a.ntile - ti) {
        rem -= a.ntile - ti;
        ++ti;
    }
    const int tj = ti + rem;
    const int64_t per = (a.T + GSLICES - 1) / GSLICES;
    const int64_t r0 = (int64_t)slice * per, r1 = r0 + per < a.T ? r0 + per : a.T;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    // loader: thread -> (row tid / 8, columns 8 (tid % 8) .. +8) of both panels
    const int lr = tid >> 3, lc = (tid & 7) * 8;
    double vi[8], vj[8];
    QCol ci[8], cj[8];   // QUAD: this thread's columns, decoded once
    if (QUAD) {
        const int nf = a.n + a.n * (a.n + 1) / 2 + 5;   // the return's column
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int gi = ti * GT + lc + u, gj = tj * GT + lc + u;
            ci[u] = gi == nf ? qpack(Q_Y, 0, 0) : (gi > nf ? qpack(Q_ZERO, 0, 0) : qcol(gi, a.n));
            cj[u] = gj == nf ? qpack(Q_Y, 0, 0) : (gj > nf ? qpack(Q_ZERO, 0, 0) : qcol(gj, a.n));
        }
    }
    auto gload = [&](int64_t c0) {
        const int64_t row = c0 + lr;
        const bool in = row < r1;
        if (QUAD) {
            const QTime tm = qtime(a.al, in ? row : r0);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                vi[u] = in ? qfeat((const double*)a.obs, a.y, tm, row, ci[u], a.n) : 0.0;
                vj[u] = in ? qfeat((const double*)a.obs, a.y, tm, row, cj[u], a.n) : 0.0;
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            vi[u] = in ? feat(a.obs, a.lo, a.y, a.al, row, ti * GT + lc + u, a.n) : 0.0;
            vj[u] = in ? feat(a.obs, a.lo, a.y, a.al, row, tj * GT + lc + u, a.n) : 0.0;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            PI[buf][lr][lc + u] = vi[u];
            PJ[buf][lr][lc + u] = vj[u];
        }
    };

    doublex4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};

    const int r16 = lane & 15, q = lane >> 4;
    int buf = 0;
    if (r0 < r1) {
        gload(r0);
        lstore(0);
    }
    __syncthreads();
    for (int64_t c0 = r0; c0 < r1; c0 += GRC) {
        const bool more = c0 + GRC < r1;
        if (more) gload(c0 + GRC);
#pragma unroll
        for (int k = 0; k < GRC; k += 4) {
            double av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i] = PI[buf][k + q][wr * 32 + i * 16 + r16];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = PJ[buf][k + q][wc * 32 + j * 16 + r16];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    double* out = a.slab + ((int64_t)slice * a.npair + pair) * GT * GT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = wr * 32 + i * 16 + q + 4 * r;   // f64 C/D map: row = (l>>4) + 4 reg
                const int col = wc * 32 + j * 16 + r16;
                out[row * GT + col] = acc[i][j][r];
            }
}

// out[K][K] (K = n + 5) = sum over slices (in order) of the slab tiles, mirrored
__global__ void __launch_bounds__(256) k_gram_reduce(const double* __restrict__ slab, int ntile, int npair, int K,
                                                     double* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)npair * GT * GT) return;
    const int pair = (int)(e / (GT * GT)), rc = (int)(e % (GT * GT));
    int ti = 0, rem = pair;
    while (rem >= ntile - ti) {
        rem -= ntile - ti;
        ++ti;
    }
    const int tj = ti + rem;
    const int gi = ti * GT + rc / GT, gj = tj * GT + rc % GT;
    if (gi >= K || gj >= K || (ti == tj && gj < gi)) return;
    double s = 0.0;
    for (int sl = 0; sl < GSLICES; ++sl) s += slab[((int64_t)sl * npair + pair) * GT * GT + rc];
    out[(int64_t)gi * K + gj] = s;
    out[(int64_t)gj * K + gi] = s;
}

// r_t = y_t - [clip(o_t), a, a^2, a^3, 1] . c  (fit(return_errors=True)'s residuals)
template <typename TO>
__global__ void __launch_bounds__(256) k_linear_residual(const TO* __restrict__ obs, const float* __restrict__ lo,
                                                         const double* __restrict__ y,
                                                         const double* __restrict__ al, int64_t T, int n,
                                                         const double* __restrict__ coef, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < T; row += nw) {
        double acc = 0.0;
        for (int j = lane; j < n; j += 64) {
            double o = obs_at(obs, lo, row * n + j);
            o = o < -10.0 ? -10.0 : (o > 10.0 ? 10.0 : o);
            acc += o * coef[j];
        }
        acc = wave_sum(acc);
        if (lane == 0) {
            const double t = al[row];
            acc += t * coef[n] + (t * t) * coef[n + 1] + pow(t, 3.0) * coef[n + 2] + coef[n + 3];
            out[row] = y[row] - acc;
        }
    }
}

// r_t = y_t - F_t . c with QuadraticBaseline's features (fit(return_errors=True))
__global__ void __launch_bounds__(256) k_quadratic_residual(const double* __restrict__ o, const double* __restrict__ y,
                                                            const double* __restrict__ al, int64_t T, int n,
                                                            const double* __restrict__ coef, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int nf = n + n * (n + 1) / 2 + 5;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < T; row += nw) {
        double acc = 0.0;
        const QTime tm = qtime(al, row);
        for (int g = lane; g < nf; g += 64) acc += qfeat(o, y, tm, row, qcol(g, n), n) * coef[g];
        acc = wave_sum(acc);
        if (lane == 0) out[row] = y[row] - acc;
    }
}

inline int err(hipError_t e) { return e == hipSuccess ? MJRL_OK : (int)e; }

inline int grid_for(int64_t work, int per_block, int cap) {
    int64_t g = (work + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

constexpr int QMAX_N = 64;   // QuadraticBaseline: n + n(n+1)/2 + 6 <= 2,150 Gram columns

inline void gram_dims(int n, int& K, int& ntile, int& npair, bool quad = false) {
    K = quad ? n + n * (n + 1) / 2 + 6 : n + 5;
    ntile = (K + GT - 1) / GT;
    npair = ntile * (ntile + 1) / 2;
}

}  // namespace

extern "C" {

int mjrl_linear_baseline_gram_scratch(int32_t n, int64_t T, int64_t* doubles) {
    if (n <= 0 || T < 0 || !doubles) return MJRL_EINVAL;
    int K, ntile, npair;
    gram_dims(n, K, ntile, npair);
    *doubles = (int64_t)GSLICES * npair * GT * GT + T;
    return MJRL_OK;
}

extern "C++" {
template <typename TO, bool QUAD = false>
static int linear_baseline_gram(const TO* obs, const float* lo, const double* returns, int64_t T, int32_t n,
                                const int64_t* path_off, int64_t P, double* scratch, double* out, void* stream) {
    if (n <= 0 || T < 0 || P < 0 || !out || !scratch || (T > 0 && (!obs || !returns || !path_off)) ||
        (QUAD && n > QMAX_N))
        return MJRL_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    int K, ntile, npair;
    gram_dims(n, K, ntile, npair, QUAD);
    double* slab = scratch;
    double* al = scratch + (int64_t)GSLICES * npair * GT * GT;
    if (P > 0) {
        const int64_t g = (P + 3) / 4;
        hipLaunchKernelGGL(k_path_time, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, st, path_off, P, al);
    }
    const int groups = (GSLICES + 7) / 8;   // slices per XCD
    if (QUAD) {
        // o = clip(obs) / 10 once per value (scratch behind the path times), then the
        // Gram over the features formed from it
        double* o = al + T;
        const int64_t N = T * (int64_t)n;
        if (N > 0)
            hipLaunchKernelGGL(k_quad_obs<TO>, dim3((unsigned)grid_for(N, 256, 8192)), dim3(256), 0, st, obs, lo, N, o);
        GramArgs<double> ga{o, nullptr, returns, al, T, n, ntile, npair, slab};
        hipLaunchKernelGGL((k_gram<double, true>), dim3(8 * groups * npair), dim3(GTHREADS), 0, st, ga);
    } else {
        GramArgs<TO> ga{obs, lo, returns, al, T, n, ntile, npair, slab};
        hipLaunchKernelGGL((k_gram<TO, false>), dim3(8 * groups * npair), dim3(GTHREADS), 0, st, ga);
    }
    const int64_t ne = (int64_t)npair * GT * GT;
    hipLaunchKernelGGL(k_gram_reduce, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, slab, ntile, npair, K,
                       out);
    return err(hipGetLastError());
}
}  // extern "C++"

extern "C++" {
template <typename TO, bool QUAD = false>
static int linear_baseline_residual(const TO* obs, const float* lo, const double* returns, int64_t T, int32_t n,
                                    const int64_t* path_off, int64_t P, const double* coeffs, double* scratch,
                                    double* out, void* stream) {
    if (n <= 0 || T < 0 || P < 0 || (T > 0 && (!obs || !returns || !path_off || !coeffs || !scratch || !out)) ||
        (QUAD && n > QMAX_N))
        return MJRL_EINVAL;
    if (T == 0) return MJRL_OK;
    hipStream_t st = (hipStream_t)stream;
    int K, ntile, npair;
    gram_dims(n, K, ntile, npair, QUAD);
    double* al = scratch + (int64_t)GSLICES * npair * GT * GT;
    if (P > 0) {
        const int64_t g = (P + 3) / 4;
        hipLaunchKernelGGL(k_path_time, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, st, path_off, P, al);
    }
    const int64_t g = (T + 3) / 4;
    if (QUAD) {
        double* o = al + T;
        const int64_t N = T * (int64_t)n;
        hipLaunchKernelGGL(k_quad_obs<TO>, dim3((unsigned)grid_for(N, 256, 8192)), dim3(256), 0, st, obs, lo, N, o);
        hipLaunchKernelGGL(k_quadratic_residual, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, st, o, returns,
                           al, T, n, coeffs, out);
    } else
        hipLaunchKernelGGL(k_linear_residual<TO>, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, st, obs,
                           lo, returns, al, T, n, coeffs, out);
    return err(hipGetLastError());
}
}  // extern "C++"

int mjrl_linear_baseline_gram(const double* obs, const double* returns, int64_t T, int32_t n,
                              const int64_t* path_off, int64_t P, double* scratch, double* out, void* stream) {
    return linear_baseline_gram(obs, (const float*)nullptr, returns, T, n, path_off, P, scratch, out, stream);
}

int mjrl_linear_baseline_gram_f32(const float* obs, const double* returns, int64_t T, int32_t n,
                                  const int64_t* path_off, int64_t P, double* scratch, double* out, void* stream) {
    return linear_baseline_gram(obs, (const float*)nullptr, returns, T, n, path_off, P, scratch, out, stream);
}

int mjrl_linear_baseline_residual(const double* obs, const double* returns, int64_t T, int32_t n,
                                  const int64_t* path_off, int64_t P, const double* coeffs, double* scratch,
                                  double* out, void* stream) {
    return linear_baseline_residual(obs, (const float*)nullptr, returns, T, n, path_off, P, coeffs, scratch, out,
                                    stream);
}

int mjrl_linear_baseline_residual_f32(const float* obs, const double* returns, int64_t T, int32_t n,
                                      const int64_t* path_off, int64_t P, const double* coeffs, double* scratch,
                                      double* out, void* stream) {
    return linear_baseline_residual(obs, (const float*)nullptr, returns, T, n, path_off, P, coeffs, scratch, out,
                                    stream);
}

int mjrl_linear_baseline_gram_f32x2(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                    int32_t n, const int64_t* path_off, int64_t P, double* scratch, double* out,
                                    void* stream) {
    if (T > 0 && !obs_lo) return MJRL_EINVAL;
    return linear_baseline_gram(obs, obs_lo, returns, T, n, path_off, P, scratch, out, stream);
}

int mjrl_linear_baseline_residual_f32x2(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                        int32_t n, const int64_t* path_off, int64_t P, const double* coeffs,
                                        double* scratch, double* out, void* stream) {
    if (T > 0 && !obs_lo) return MJRL_EINVAL;
    return linear_baseline_residual(obs, obs_lo, returns, T, n, path_off, P, coeffs, scratch, out, stream);
}

int mjrl_quadratic_baseline_gram_scratch(int32_t n, int64_t T, int64_t* doubles) {
    if (n <= 0 || n > QMAX_N || T < 0 || !doubles) return MJRL_EINVAL;
    int K, ntile, npair;
    gram_dims(n, K, ntile, npair, true);
    *doubles = (int64_t)GSLICES * npair * GT * GT + T + T * (int64_t)n;   // slabs, path times, o
    return MJRL_OK;
}

int mjrl_quadratic_baseline_gram(const double* obs, const double* returns, int64_t T, int32_t n,
                                 const int64_t* path_off, int64_t P, double* scratch, double* out, void* stream) {
    return linear_baseline_gram<double, true>(obs, nullptr, returns, T, n, path_off, P, scratch, out, stream);
}

int mjrl_quadratic_baseline_gram_f32(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                     int32_t n, const int64_t* path_off, int64_t P, double* scratch, double* out,
                                     void* stream) {
    return linear_baseline_gram<float, true>(obs, obs_lo, returns, T, n, path_off, P, scratch, out, stream);
}

int mjrl_quadratic_baseline_residual(const double* obs, const double* returns, int64_t T, int32_t n,
                                     const int64_t* path_off, int64_t P, const double* coeffs, double* scratch,
                                     double* out, void* stream) {
    return linear_baseline_residual<double, true>(obs, nullptr, returns, T, n, path_off, P, coeffs, scratch, out,
                                                  stream);
}

int mjrl_quadratic_baseline_residual_f32(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                         int32_t n, const int64_t* path_off, int64_t P, const double* coeffs,
                                         double* scratch, double* out, void* stream) {
    return linear_baseline_residual<float, true>(obs, obs_lo, returns, T, n, path_off, P, coeffs, scratch, out,
                                                 stream);
}

}  // extern "C"
