// batch.hip — batch assembly, returns / GAE scan, moments and whitening.
//
// HBM-bound fp64 / byte work: coalesced grid-stride loops, no MFMA.
// Reference: mjrl/utils/process_samples.py:3-44, mjrl/algos/npg_cg.py:86-105,
// mjrl/algos/dapg.py:62-74, mjrl/policies/gaussian_mlp.py:103,177.
#include "common.h"

using namespace mjrl;

namespace {

constexpr int MOM_BLOCKS = 256;
constexpr int MOM_THREADS = 256;

// obs f64 (or f32: staged by the host) [T][n] -> xhat f32 [T][np]; act -> f32.
// One thread per 4 output columns so the xhat stores are 16 B per lane.
template <typename TO>
__global__ void __launch_bounds__(256) k_pack_batch(const TO* __restrict__ obs, const TO* __restrict__ act,
                                                    int64_t T, int n, int m, int np,
                                                    const float* __restrict__ in_shift,
                                                    const float* __restrict__ in_scale, float* __restrict__ xhat,
                                                    float* __restrict__ act32) {
    const int64_t nq = (int64_t)T * (np / 4);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += stride) {
        const int64_t row = i / (np / 4);
        const int c0 = (int)(i - row * (np / 4)) * 4;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = c0 + u;
            float x;
            if (c < n) {
                x = (float)obs[row * n + c];                  // torch .float(): round to nearest
                if (in_shift) x = (x - in_shift[c]) / (in_scale[c] + 1e-8f);   // MuNet.forward:177
            } else {
                x = (c == n) ? 1.0f : 0.0f;                   // bias column, zero pad
            }
            v[u] = x;
        }
        *reinterpret_cast<float4*>(xhat + row * np + c0) = make_float4(v[0], v[1], v[2], v[3]);
    }
    const int64_t na = (int64_t)T * m;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) act32[i] = (float)act[i];
}

// Column maxima of xhat over the batch (the input of the split rows' column
// scales, common.h col_scale): cm[k] = max_t |xhat[t][k]| as f32 bits (atomicMax on
// the bits of non-negative floats: order-independent, so deterministic), cm[n] =
// 1 (the bias column).  Thread (rsub, j) of a workgroup owns the V-wide column
// group j (n / V <= NT groups: np <= 512) of rows rsub, rsub + RPP, ... of the
// workgroup's row stride, CR rows per batch with every load issued before the
// first max: rows past T are clamped to row T - 1 (a max is idempotent), so the
// batch has no branches between its loads.  Maxima go through LDS (ds_max_u32),
// then one global atomicMax per column per workgroup.
template <typename TO, int V, int NT>
__global__ void __launch_bounds__(NT) k_colmax(const TO* __restrict__ obs, int64_t T, int n,
                                                const float* __restrict__ in_shift,
                                                const float* __restrict__ in_scale, unsigned* __restrict__ cm) {
    constexpr int CR = 8;
    __shared__ unsigned smax[512];
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += NT) smax[i] = 0u;
    __syncthreads();
    const int nv = n / V;                       // V divides n (host)
    const int rpp = NT / nv;                    // rows per pass
    const int rsub = tid / nv, j = tid % nv;
    if (rsub < rpp) {
        float mx[V], sh[V], den[V];
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const int c = j * V + e;
            mx[e] = 0.f;
            sh[e] = in_shift ? in_shift[c] : 0.f;
            den[e] = in_shift ? in_scale[c] + 1e-8f : 1.f;
        }
        const int64_t rstride = (int64_t)gridDim.x * rpp;
        for (int64_t row0 = (int64_t)blockIdx.x * rpp + rsub; row0 < T; row0 += CR * rstride) {
            float x[CR][V];
#pragma unroll
            for (int i = 0; i < CR; ++i) {
                const int64_t row = min(row0 + i * rstride, T - 1);
                const TO* src = obs + row * n + V * j;
                if constexpr (V == 4 && sizeof(TO) == 4) {
                    const float4 q = *reinterpret_cast<const float4*>(src);
                    x[i][0] = q.x; x[i][1] = q.y; x[i][2] = q.z; x[i][3] = q.w;
                } else {
#pragma unroll
                    for (int e = 0; e < V; ++e) x[i][e] = (float)src[e];   // torch .float()
                }
            }
#pragma unroll
            for (int i = 0; i < CR; ++i)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    float v = x[i][e];
                    if (in_shift) v = (v - sh[e]) / den[e];   // MuNet.forward:177, as the pack
                    mx[e] = fmaxf(mx[e], fabsf(v));
                }
        }
#pragma unroll
        for (int e = 0; e < V; ++e) atomicMax(&smax[j * V + e], __float_as_uint(mx[e]));
    }
    __syncthreads();
    for (int c = tid; c < n; c += NT)
        if (smax[c]) atomicMax(&cm[c], smax[c]);
    if (blockIdx.x == 0 && tid == 0) atomicMax(&cm[n], __float_as_uint(1.0f));
}

// obs f64 [T][n] -> split-f16 rows (mjrl_rows.xs / xu): one wave per row, lane l
// owns columns l, l + 64, ... (np <= 512), so every load (8 B per lane) and every
// hi / lo store (2 B per lane) is one contiguous wave-wide segment.  Each column is
// divided by its power-of-two scale xc[k] (col_scale, common.h), then the row's
// max |xhat / xc| (> 0: the bias column) gives xu = 2^(E-15) with the row's
// max |y| in [2^14, 2^15), y = xhat / (xc xu); then hi = f16(y), lo = f16(y - hi).
// Every scaling is by a power of two, so y * xc * xu is the f32 xhat of
// k_pack_batch exactly, and the pair (hi, lo) carries it to the bound of common.h.
constexpr int PS_MAXP = 4;   // column pairs per lane (np <= 512)
template <typename TO>
__global__ void __launch_bounds__(256) k_pack_split(const TO* __restrict__ obs, const TO* __restrict__ act,
                                                    int64_t T, int n, int m, int np,
                                                    const float* __restrict__ in_shift,
                                                    const float* __restrict__ in_scale,
                                                    const float* __restrict__ xc, _Float16* __restrict__ xs,
                                                    float* __restrict__ xu, float* __restrict__ act32) {
    // lane l owns the column pairs (2l + 128j, 2l + 128j + 1): 16-byte loads of the f64
    // row when n is even (8-byte otherwise), 4-byte hi / lo stores
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int npair = (np + 127) / 128;
    float icx[PS_MAXP][2];   // 1 / xc of the lane's columns (exact: powers of two)
#pragma unroll
    for (int j = 0; j < PS_MAXP; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int ce = 2 * lane + 128 * j + e;
            icx[j][e] = ce < np ? 1.f / xc[ce] : 1.f;
        }
    const bool even = (n & 1) == 0 && (reinterpret_cast<uintptr_t>(obs) & (2 * sizeof(TO) - 1)) == 0;   // pair loads
    for (int64_t row = wid; row < T; row += nw) {
        const TO* src = obs + row * n;
        float v[PS_MAXP][2];
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < PS_MAXP; ++j) {
            const int c = 2 * lane + 128 * j;
            TO d0 = 0, d1 = 0;
            if (j < npair) {
                if (even && c + 1 < n) {
                    if constexpr (sizeof(TO) == 8) {
                        const double2 d = *reinterpret_cast<const double2*>(src + c);
                        d0 = d.x;
                        d1 = d.y;
                    } else {
                        const float2 d = *reinterpret_cast<const float2*>(src + c);
                        d0 = d.x;
                        d1 = d.y;
                    }
                } else {
                    if (c < n) d0 = src[c];
                    if (c + 1 < n) d1 = src[c + 1];
                }
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int ce = c + e;
                float x = 0.f;
                if (j < npair) {
                    if (ce < n) {
                        x = (float)(e ? d1 : d0);                    // torch .float(): round to nearest
                        if (in_shift) x = (x - in_shift[ce]) / (in_scale[ce] + 1e-8f);   // MuNet.forward:177
                    } else if (ce == n) {
                        x = 1.0f;                                    // bias column (zero padding after)
                    }
                }
                v[j][e] = x * icx[j][e];
                mx = fmaxf(mx, fabsf(v[j][e]));
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float inv;
        const float s = pow2_scale(mx, inv);
        _Float16* dst = xs + row * (2 * (int64_t)np);
#pragma unroll
        for (int j = 0; j < PS_MAXP; ++j) {
            const int c = 2 * lane + 128 * j;
            if (j < npair && c < np) {
                typedef _Float16 half2v __attribute__((ext_vector_type(2)));
                half2v h, l;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const float y = v[j][e] * s;
                    h[e] = (_Float16)y;
                    l[e] = (_Float16)(y - (float)h[e]);
                }
                *reinterpret_cast<half2v*>(dst + c) = h;
                *reinterpret_cast<half2v*>(dst + np + c) = l;
            }
        }
        if (lane == 0) xu[row] = inv;
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t na = (int64_t)T * m;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) act32[i] = (float)act[i];
}

// The same for f32 observations with n % 4 == 0 (the default staging of
// train_step): lane l owns the column quads 4l + 256j, so each row is read with
// 16-byte loads and written with 8-byte hi / lo stores, and the lane's
// normalisation constants are loaded once per launch.  Same values as
// k_pack_split (the same f32 operations per element).
constexpr int PQ_MAXQ = 2;   // column quads per lane (np <= 512)
__global__ void __launch_bounds__(256) k_pack_split_q(const float* __restrict__ obs, const float* __restrict__ act,
                                                      int64_t T, int n, int m, int np,
                                                      const float* __restrict__ in_shift,
                                                      const float* __restrict__ in_scale,
                                                      const float* __restrict__ xc, _Float16* __restrict__ xs,
                                                      float* __restrict__ xu, float* __restrict__ act32) {
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int nq = (np + 255) / 256;
    float sh[PQ_MAXQ][4], den[PQ_MAXQ][4], icx[PQ_MAXQ][4];
#pragma unroll
    for (int j = 0; j < PQ_MAXQ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int ce = 4 * lane + 256 * j + e;
            sh[j][e] = in_shift && ce < n ? in_shift[ce] : 0.f;
            den[j][e] = in_shift && ce < n ? in_scale[ce] + 1e-8f : 1.f;
            icx[j][e] = ce < np ? 1.f / xc[ce] : 1.f;   // exact: powers of two
        }
    for (int64_t row = wid; row < T; row += nw) {
        const float* src = obs + row * n;
        float v[PQ_MAXQ][4];
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < PQ_MAXQ; ++j) {
            const int c = 4 * lane + 256 * j;
            float d[4] = {0.f, 0.f, 0.f, 0.f};
            if (j < nq) {
                if (c + 3 < n) {
                    const float4 q = *reinterpret_cast<const float4*>(src + c);
                    d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (c + e < n) d[e] = src[c + e];
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ce = c + e;
                float x = 0.f;
                if (j < nq) {
                    if (ce < n) {
                        x = d[e];
                        if (in_shift) x = (x - sh[j][e]) / den[j][e];   // MuNet.forward:177
                    } else if (ce == n) {
                        x = 1.0f;                                    // bias column (zero padding after)
                    }
                }
                v[j][e] = x * icx[j][e];
                mx = fmaxf(mx, fabsf(v[j][e]));
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float inv;
        const float sc = pow2_scale(mx, inv);
        _Float16* dst = xs + row * (2 * (int64_t)np);
#pragma unroll
        for (int j = 0; j < PQ_MAXQ; ++j) {
            const int c = 4 * lane + 256 * j;
            if (j < nq && c < np) {
                half4 h, l;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float y = v[j][e] * sc;
                    h[e] = (_Float16)y;
                    l[e] = (_Float16)(y - (float)h[e]);
                }
                *reinterpret_cast<half4*>(dst + c) = h;
                *reinterpret_cast<half4*>(dst + np + c) = l;
            }
        }
        if (lane == 0) xu[row] = inv;
    }
    if (act32 != act) {
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        const int64_t na = (int64_t)T * m;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) act32[i] = act[i];
    }
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One wave per path.  The path's rewards and baselines come into LDS with
// coalesced loads, in windows of GW steps; lane 0 runs the serial fp64 chains out
// of LDS (separate multiply and add, __dmul_rn / __dadd_rn cannot be contracted:
// bit-identical to discount_sum), writing returns / advantages back in place; the
// wave then stores the window with coalesced writes.  Paths longer than a window
// are walked window by window (forward for the path-return sum, backward for the
// recurrences), carrying the chain state across windows.
constexpr int GW = 1024;           // steps per LDS window

// LDS written by some lanes of a wave and read by others: order the accesses
// (waitcnt + compiler barrier) without a workgroup barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int GAE_WAVES = 2;       // waves (paths in flight) per workgroup (3 x 8 KB windows each)
// serial steps per batch of LDS reads: 8 / 16 / 32 measured 47.8 / 45.1 / 44.3 us for
// 125 paths of 1000 steps (profiles/r05x/gae.txt): the chain is the dependent fp64
// multiply -> add (~44 ns a step), not the LDS reads
#ifndef MJRL_GAE_GU
#define MJRL_GAE_GU 32
#endif
constexpr int GU = MJRL_GAE_GU;

__global__ void __launch_bounds__(64 * GAE_WAVES) k_gae(const double* __restrict__ rew,
                                                        const double* __restrict__ base,
                                                        const int64_t* __restrict__ off,
                                                        const uint8_t* __restrict__ term, int64_t P, double gamma,
                                                        double gl, int use_gae, double* __restrict__ ret,
                                                        double* __restrict__ adv, double* __restrict__ path_ret) {
    __shared__ double sr[GAE_WAVES][GW];
    __shared__ double sb[GAE_WAVES][GW];
    __shared__ double stt[GAE_WAVES][GW];
    __shared__ double sjunk[GAE_WAVES][GW];   // the stores of chains whose outputs are not kept
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* R = sr[w];
    double* B = sb[w];
    double* TD = stt[w];
    for (int64_t p = (int64_t)blockIdx.x * GAE_WAVES + w; p < P; p += (int64_t)gridDim.x * GAE_WAVES) {
        const int64_t b = off[p], e = off[p + 1];
        if (e - b <= GW) {
            // One window: the three serial chains — the path-return sum (forward),
            // the returns and the advantages (backward) — run side by side on lanes 0,
            // 1 and 2 of ONE instruction stream, acc = x + c * acc with (x, c) =
            // (reward, 1), (reward, gamma), (td, gamma * lambda): c = 1 makes the
            // product exact, so lane 0 is Python's front-to-back sum bit for bit, and
            // lanes 1 / 2 are discount_sum's recurrences (process_samples.py:37-44).
            // The td terms are formed by the whole wave first.
            const int cnt = (int)(e - b);
            {
                double x[GW / 64], y[GW / 64];
#pragma unroll
                for (int k = 0; k < GW / 64; ++k) {
                    const bool in = lane + 64 * k < cnt;
                    x[k] = in ? rew[b + lane + 64 * k] : 0.0;
                    y[k] = in ? base[b + lane + 64 * k] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < GW / 64; ++k)
                    if (lane + 64 * k < cnt) {
                        R[lane + 64 * k] = x[k];
                        B[lane + 64 * k] = y[k];
                    }
            }
            wave_sync();
            // GAE td = r + gamma * b1[t+1] - b[t] with b1 = append(b, 0 if terminated
            // else b[-1]) (process_samples.py:23-27); plain advantages keep b here
            const double blast = cnt > 0 ? (term[p] ? 0.0 : B[cnt - 1]) : 0.0;
            for (int i = lane; i < cnt; i += 64) {
                const double bb = B[i];
                if (use_gae) {
                    const double bn = i + 1 < cnt ? B[i + 1] : blast;
                    TD[i] = __dsub_rn(__dadd_rn(R[i], __dmul_rn(gamma, bn)), bb);
                } else {
                    TD[i] = bb;
                }
            }
            wave_sync();
            if (lane < 3) {
                const bool fwd = lane == 0;
                const double c = lane == 0 ? 1.0 : (lane == 1 ? gamma : gl);
                const double* src = lane == 2 ? TD : R;
                // returns over B (free now), advantages in place; the path-return sum's
                // (and plain advantages') chain stores into a junk window, so every step's
                // store is unconditional (an exec-masked store per step cost a branch
                // with its exec save / restore on the serial chain)
                const bool put = lane == 1 || (lane == 2 && use_gae);
                double* dst = lane == 1 ? B : (put ? TD : sjunk[w]);
                double acc = 0.0;
                int j = 0;
                // software-pipelined: the LDS reads of batch j + GU are issued (in program
                // order, before this batch's stores: legal even in place) ahead of batch
                // j's serial steps, so only the dependent fp64 multiply-add chain is on
                // the critical path, not a ~50-cycle LDS round trip per batch
                const int nfull = cnt / GU * GU;
                double xv[GU];
                if (nfull > 0) {
#pragma unroll
                    for (int u = 0; u < GU; ++u) xv[u] = src[fwd ? u : cnt - 1 - u];
                }
                for (; j < nfull; j += GU) {
                    double xn[GU];
                    const int jn = j + GU < nfull ? j + GU : j;   // clamped: the last batch re-reads itself
#pragma unroll
                    for (int u = 0; u < GU; ++u) xn[u] = src[fwd ? jn + u : cnt - 1 - jn - u];
#pragma unroll
                    for (int u = 0; u < GU; ++u) {
                        acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                        dst[cnt - 1 - j - u] = acc;
                    }
#pragma unroll
                    for (int u = 0; u < GU; ++u) xv[u] = xn[u];
                }
                for (; j < cnt; ++j) {
                    const int idx = fwd ? j : cnt - 1 - j;
                    acc = __dadd_rn(src[idx], __dmul_rn(c, acc));
                    dst[idx] = acc;
                }
                if (lane == 0) path_ret[p] = acc;
            }
            wave_sync();
            for (int i = lane; i < cnt; i += 64) {
                const double rr = B[i];
                ret[b + i] = rr;
                adv[b + i] = use_gae ? TD[i] : __dsub_rn(rr, TD[i]);   // plain: ret - baseline
            }
            wave_sync();
            continue;
        }
        // sum(p["rewards"]) — Python's builtin sum, front to back (npg_cg.py:97)
        double s = 0.0;
        for (int64_t w0 = b; w0 < e; w0 += GW) {
            const int cnt = e - w0 < GW ? (int)(e - w0) : GW;
            {
                double x[GW / 64];   // all of the lane's loads in flight at once
#pragma unroll
                for (int k = 0; k < GW / 64; ++k) x[k] = lane + 64 * k < cnt ? rew[w0 + lane + 64 * k] : 0.0;
#pragma unroll
                for (int k = 0; k < GW / 64; ++k)
                    if (lane + 64 * k < cnt) R[lane + 64 * k] = x[k];
            }
            wave_sync();
            if (lane == 0) {
                int i = 0;
                for (; i + GU <= cnt; i += GU) {
                    double x[GU];
#pragma unroll
                    for (int u = 0; u < GU; ++u) x[u] = R[i + u];
#pragma unroll
                    for (int u = 0; u < GU; ++u) s = __dadd_rn(s, x[u]);
                }
                for (; i < cnt; ++i) s = __dadd_rn(s, R[i]);
            }
            wave_sync();
        }
        if (lane == 0) path_ret[p] = s;
        if (e <= b) continue;
        // returns: discount_sum(rewards, gamma) (process_samples.py:3-5, 37-44)
        // GAE (process_samples.py:21-29): b1 = append(b, 0 if terminated else b[-1]),
        // td = r + gamma*b1[1:] - b1[:-1], adv = discount_sum(td, gamma*lambda);
        // plain advantages (process_samples.py:10-13): ret - baseline.
        double acc_r = 0.0, acc_a = 0.0;
        double bnext = term[p] ? 0.0 : base[e - 1];
        for (int64_t w1 = e; w1 > b; w1 -= GW) {
            const int64_t w0 = w1 - GW > b ? w1 - GW : b;
            const int cnt = (int)(w1 - w0);
            {
                // a one-window path still has its rewards in R from the sum above
                const bool reload = e - b > GW;
                double x[GW / 64], y[GW / 64];
#pragma unroll
                for (int k = 0; k < GW / 64; ++k) {
                    const bool in = lane + 64 * k < cnt;
                    x[k] = in && reload ? rew[w0 + lane + 64 * k] : 0.0;
                    y[k] = in ? base[w0 + lane + 64 * k] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < GW / 64; ++k)
                    if (lane + 64 * k < cnt) {
                        if (reload) R[lane + 64 * k] = x[k];
                        B[lane + 64 * k] = y[k];
                    }
            }
            wave_sync();
            if (lane == 0) {
                int i = cnt;
                for (; i >= GU; i -= GU) {   // steps i-1 .. i-GU
                    double r[GU], bb[GU];
#pragma unroll
                    for (int u = 0; u < GU; ++u) {
                        r[u] = R[i - 1 - u];
                        bb[u] = B[i - 1 - u];
                    }
#pragma unroll
                    for (int u = 0; u < GU; ++u) {
                        acc_r = __dadd_rn(r[u], __dmul_rn(gamma, acc_r));
                        R[i - 1 - u] = acc_r;
                        if (use_gae) {
                            const double td = __dsub_rn(__dadd_rn(r[u], __dmul_rn(gamma, bnext)), bb[u]);
                            acc_a = __dadd_rn(td, __dmul_rn(gl, acc_a));
                            B[i - 1 - u] = acc_a;
                            bnext = bb[u];
                        } else {
                            B[i - 1 - u] = __dsub_rn(acc_r, bb[u]);
                        }
                    }
                }
                for (; i > 0; --i) {
                    const double r = R[i - 1], bb = B[i - 1];
                    acc_r = __dadd_rn(r, __dmul_rn(gamma, acc_r));
                    R[i - 1] = acc_r;
                    if (use_gae) {
                        const double td = __dsub_rn(__dadd_rn(r, __dmul_rn(gamma, bnext)), bb);
                        acc_a = __dadd_rn(td, __dmul_rn(gl, acc_a));
                        B[i - 1] = acc_a;
                        bnext = bb;
                    } else {
                        B[i - 1] = __dsub_rn(acc_r, bb);
                    }
                }
            }
            wave_sync();
            for (int i = lane; i < cnt; i += 64) {
                ret[w0 + i] = R[i];
                adv[w0 + i] = B[i];
            }
            wave_sync();
        }
    }
}

// Lanes = paths (round 6): the serial recurrences of LP_PATHS paths run side by side
// in ONE instruction stream each, one wave per chain, each lane one path — wave 0
// the returns (discount_sum(rewards, gamma)), wave 1 the advantages (discount_sum(td,
// gamma lambda), idle without GAE), wave 2 the path-return sum (front to back; on a
// mover wave instead it measured slower, profiles/r06e/rejected/).  A
// dependent fp64 multiply -> add costs ~11 cycles of issue per step for the whole
// wave, however many lanes are on (profiles/r06b/gae_latency.txt), so LP_PATHS paths
// advance for the price one did — as long as the chain wave does little else: a
// store of its outputs costs it ~10 cycles a step to HBM and ~13 to LDS, an LDS read
// ~2 (profiles/r06c/gae_latency.txt, the "lanes" rows).  So the chain waves only read
// and keep one checkpoint per LP_GB-step segment (the accumulator entering it, one
// LDS write per segment), and the four mover waves (3..6) recompute every segment
// from its checkpoint — the same __dmul_rn / __dadd_rn in the same order, so the
// same values bit for bit — one segment per lane, 256 segments side by side, and
// store them (each lane a 128-byte run).  The steps come through three LDS buffers in
// windows of LP_W steps per path (backward windows aligned at each path's end,
// forward windows at its start): while the chains consume window i, the movers
// recompute and store window i - 1, put window i + 1 (td formed on the way) and issue
// window i + 2's loads.  One barrier per window.  Bit-identical to k_gae.
typedef double lp_d2 __attribute__((ext_vector_type(2), aligned(8)));   // 16-byte store, 8-byte aligned
constexpr int LP_PATHS = 8;               // paths per workgroup (lanes 0..7 of each chain wave)
#ifndef MJRL_GAE_W
#define MJRL_GAE_W 256
#endif
constexpr int LP_W = MJRL_GAE_W;          // steps per window
constexpr int LP_LD = LP_W + 1;           // LDS row stride (doubles): chain lanes conflict-free
constexpr int LP_GB = 16;                 // steps per segment (chain register batch, recompute task)
constexpr int LP_NS = LP_W / LP_GB;       // segments per window row
constexpr int LP_CH = 3;                  // chain waves 0..2
constexpr int LP_MVW = 4;                 // mover waves 3..6
constexpr int LP_T = 64 * (LP_CH + LP_MVW);
constexpr int LP_MV = 64 * LP_MVW;
constexpr int LP_TPP = LP_MV / LP_PATHS;  // mover threads a path: runs of LP_TPP consecutive steps a load
constexpr int LP_PER = LP_W / LP_TPP;     // window elements per mover thread per array
constexpr int LP_BUF = LP_PATHS * LP_LD;  // one array of one buffer (doubles)
constexpr int LP_NB = 3;                  // LDS buffers
static_assert(LP_W % LP_TPP == 0 && LP_W % LP_GB == 0, "window split");
static_assert(2 * LP_PATHS * LP_NS <= LP_MV, "one recompute segment per mover thread");

// A chain wave's pass over one window row (its lane's path), batch k + 2's LDS reads
// issued before batch k's steps (the compiler barrier keeps them from all being
// hoisted to the top).  Forward: the path-return sum front to back, Python's
// sum(p["rewards"]) (npg_cg.py:97; x + 1.0 * acc is x + acc exactly, k_gae's form;
// steps past the path's end hold 0.0).  Backward: acc = x + c * acc over the whole
// window with no step mask (a partial window, the path's first steps, holds its valid
// steps at the top, which the chain meets first; what it computes below them is never
// stored and the path's chain ends there), writing the accumulator entering each
// segment to ck[k * LP_PATHS] (segment k = batch k: u in [W - (k + 1) GB, W - k GB)).
template <bool FWD>
__device__ __forceinline__ double lp_chain(const double* __restrict__ row, double acc, double c,
                                           double* __restrict__ ck) {
    double X[3][LP_GB];
    auto at = [](int k) { return FWD ? k * LP_GB : LP_W - (k + 1) * LP_GB; };
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
        for (int g = 0; g < LP_GB; ++g) X[k][g] = row[at(k) + g];
    }
#pragma unroll
    for (int k = 0; k < LP_NS; ++k) {
        if (k + 2 < LP_NS) {
#pragma unroll
            for (int g = 0; g < LP_GB; ++g) X[(k + 2) % 3][g] = row[at(k + 2) + g];
        }
        asm volatile("" ::: "memory");
#ifndef MJRL_GAE_ABL_NOFWD
        if (FWD) {
#pragma unroll
            for (int g = 0; g < LP_GB; ++g) acc = __dadd_rn(X[k % 3][g], acc);
        }
#endif
        if (!FWD) {
            ck[k * LP_PATHS] = acc;
#pragma unroll
            for (int g = LP_GB - 1; g >= 0; --g) acc = __dadd_rn(X[k % 3][g], __dmul_rn(c, acc));
        }
    }
    return acc;
}

__global__ void __launch_bounds__(LP_T) k_gae_lp(const double* __restrict__ rew, const double* __restrict__ base,
                                                 const int64_t* __restrict__ off, const uint8_t* __restrict__ term,
                                                 int64_t P, double gamma, double gl, int use_gae,
                                                 double* __restrict__ ret, double* __restrict__ adv,
                                                 double* __restrict__ path_ret) {
    // buffer q of array A at A + q * LP_BUF: RB backward rewards, TD td (no GAE: the
    // baseline), RF forward rewards; CK[chain][window parity][segment][path]
    __shared__ double RB[LP_NB * LP_BUF], TD[LP_NB * LP_BUF], RF[LP_NB * LP_BUF];
    __shared__ double CK[2][2][LP_NS][LP_PATHS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar branches
    const int64_t p0 = (int64_t)blockIdx.x * LP_PATHS;
    const int np = (int)(P - p0 < LP_PATHS ? P - p0 : LP_PATHS);
    // the window count from the workgroup's path bounds (uniform addresses: scalar
    // loads); chain lanes and movers read their own path's bounds with vector loads
    int64_t hmax = 0;
#pragma unroll
    for (int i = 0; i < LP_PATHS; ++i) {
        if (i < np) {
            const int64_t l = off[p0 + i + 1] - off[p0 + i];
            hmax = l > hmax ? l : hmax;
        }
    }
    const int nwin = (int)((hmax + LP_W - 1) / LP_W);
    if (w < LP_CH) {
        // ---- a chain wave: LDS reads, one checkpoint write a segment ----
        const bool chain = lane < np && (w != 1 || use_gae);
        const double c = w == 0 ? gamma : gl;
        const double* const cw = (w == 0 ? RB : (w == 1 ? TD : RF)) + lane * LP_LD;
        double acc = 0.0;
        __syncthreads();   // window 0 put
        for (int i = 0; i < nwin; ++i) {
#ifdef MJRL_GAE_ABL_NOCHAIN
            if (i >= 0) {   // timing ablation: the chains skipped, barriers kept
                __syncthreads();
                continue;
            }
#endif
            if (chain) {
                const double* const row = cw + (i % LP_NB) * LP_BUF;
                if (w == 2)
                    acc = lp_chain<true>(row, acc, c, nullptr);
                else
                    acc = lp_chain<false>(row, acc, c, &CK[w][i & 1][0][lane]);
            }
            __syncthreads();
        }
        if (w == 2 && lane < np) path_ret[p0 + lane] = acc;
        return;
    }
    // ---- a mover: every global load, the recompute, every output store ----
    const int m = (w - LP_CH) * 64 + lane;
    const int mp = m / LP_TPP, mu = m % LP_TPP;
    const bool okp = mp < np;
    const int64_t db = okp ? off[p0 + mp] : 0, de = okp ? off[p0 + mp + 1] : 0, plen = de - db;
    // b1's last entry: 0 if terminated else b[-1] (process_samples.py:24-27)
    const double pbl = de > db ? (term[p0 + mp] ? 0.0 : base[de - 1]) : 0.0;
    // an empty path (or a thread past the last path) reads index 0: valid whenever a
    // window exists, and never used (nothing is stored for its steps)
    const int64_t pb = de > db ? db : 0, pe = de > db ? de : 1;
    double xr[LP_PER], xb[LP_PER], xn[LP_PER], xf[LP_PER];
    auto load = [&](int j) {
        // backward window: step t = e - (j + 1) W + u; forward window: t = b + j W + u;
        // loads from clamped indices, unconditional (no exec-masked loads in the stream)
#pragma unroll
        for (int k = 0; k < LP_PER; ++k) {
            const int u = mu + LP_TPP * k;
            int64_t tb = pe - (int64_t)(j + 1) * LP_W + u, tf = pb + (int64_t)j * LP_W + u;
            tb = tb < pb ? pb : tb;
            tf = tf < pe ? tf : pe - 1;
            const int64_t tn = tb + 1 < pe ? tb + 1 : pe - 1;
            xr[k] = rew[tb];
            xb[k] = base[tb];
            xn[k] = base[tn];
            xf[k] = rew[tf];
        }
    };
    auto put = [&](int j) {
        const int q = (j % LP_NB) * LP_BUF + mp * LP_LD;
#pragma unroll
        for (int k = 0; k < LP_PER; ++k) {
            const int u = mu + LP_TPP * k;
            const int64_t tb = pe - (int64_t)(j + 1) * LP_W + u;
            const double bn = tb + 1 < pe ? xn[k] : pbl;   // b1[t + 1] (process_samples.py:24-27)
            RB[q + u] = xr[k];
            // GAE td = r + gamma * b1[t+1] - b1[t] (process_samples.py:28); plain: b
            TD[q + u] = use_gae ? __dsub_rn(__dadd_rn(xr[k], __dmul_rn(gamma, bn)), xb[k]) : xb[k];
            // past the path's end: 0.0, which the forward sum adds exactly (acc is never -0.0)
            RF[q + u] = (int64_t)j * LP_W + u < plen ? xf[k] : 0.0;
        }
    };
    // recompute task: chain rc (0 returns from RB, 1 advantages from TD), path rp,
    // segment rs (u in [rs GB, (rs + 1) GB) = the chain's batch k = NS - 1 - rs)
    const int rc = m / (LP_PATHS * LP_NS), rp = (m / LP_NS) % LP_PATHS, rs = m % LP_NS;
    const bool rok = rp < np && (rc == 0 || use_gae) && rc < 2;
    const int64_t rb = rok ? off[p0 + rp] : 0, re = rok ? off[p0 + rp + 1] : 0;
    const double rcoef = rc == 0 ? gamma : gl;
    double* const rout = rc == 0 ? ret : adv;
    auto recompute = [&](int j) {
        if (!rok) return;
        const int q = (j % LP_NB) * LP_BUF + rp * LP_LD + rs * LP_GB;
        const double* const row = (rc == 0 ? RB : TD) + q;
        double x[LP_GB], bb[LP_GB];
#pragma unroll
        for (int g = 0; g < LP_GB; ++g) {
            x[g] = row[g];
            if (!use_gae) bb[g] = TD[q + g];   // plain: the baseline, for ret - b
        }
        double acc = CK[rc][j & 1][LP_NS - 1 - rs][rp];
#pragma unroll
        for (int g = LP_GB - 1; g >= 0; --g) {
            acc = __dadd_rn(x[g], __dmul_rn(rcoef, acc));
            x[g] = acc;
        }
        // step t = e - (j + 1) W + rs GB + g, stored when t >= b
        const int64_t t0 = re - (int64_t)(j + 1) * LP_W + rs * LP_GB;
        double* const o = rout + t0;
        double* const o2 = adv + t0;
        if (t0 >= rb) {
#pragma unroll
            for (int g = 0; g < LP_GB; g += 2) {
                *(lp_d2*)(o + g) = lp_d2{x[g], x[g + 1]};
                if (!use_gae)   // plain advantages: ret - b (process_samples.py:31-32)
                    *(lp_d2*)(o2 + g) = lp_d2{__dsub_rn(x[g], bb[g]), __dsub_rn(x[g + 1], bb[g + 1])};
            }
        } else if (t0 + LP_GB > rb) {   // the segment holding the path's first step
#pragma unroll
            for (int g = 0; g < LP_GB; ++g) {
                if (t0 + g >= rb) {
                    o[g] = x[g];
                    if (!use_gae) o2[g] = __dsub_rn(x[g], bb[g]);
                }
            }
        }
    };
    if (nwin > 0) {
        load(0);
        put(0);
    }
    if (nwin > 1) load(1);
    __syncthreads();   // window 0 put
    for (int i = 0; i < nwin; ++i) {
        // the chains run window i (buffer i % 3); buffer (i - 1) % 3 holds window i - 1,
        // whose checkpoints are CK[.][(i - 1) & 1]; put(i + 1) fills the third buffer
        if (i >= 1) recompute(i - 1);
#ifndef MJRL_GAE_ABL_NOLOAD
        if (i + 1 < nwin) put(i + 1);
        if (i + 2 < nwin) load(i + 2);
#endif
        __syncthreads();
    }
    if (nwin > 0) recompute(nwin - 1);
}

// Moments pass 1: per-block partials of sum(x-c), sum((x-c)^2), min, max.
template <typename T>
__global__ void __launch_bounds__(MOM_THREADS) k_moments_part(const T* __restrict__ x, int64_t N,
                                                              const double* __restrict__ cstat,
                                                              double* __restrict__ part) {
    __shared__ double red[MOM_THREADS / 64];
    const double c = cstat ? cstat[0] / cstat[2] : 0.0;
    double s1 = 0.0, s2 = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        const double v = (double)x[i];
        const double dv = v - c;
        s1 += dv;
        s2 += dv * dv;
        mn = fmin(mn, v);
        mx = fmax(mx, v);
    }
    const double t1 = block_sum<MOM_THREADS>(s1, red);
    const double t2 = block_sum<MOM_THREADS>(s2, red);
    // min / max through the same LDS words (order irrelevant for min/max)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, o, 64));
        mx = fmax(mx, __shfl_xor(mx, o, 64));
    }
    __shared__ double mm[2][MOM_THREADS / 64];
    if ((threadIdx.x & 63) == 0) {
        mm[0][threadIdx.x >> 6] = mn;
        mm[1][threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < MOM_THREADS / 64; ++i) {
            mn = fmin(mn, mm[0][i]);
            mx = fmax(mx, mm[1][i]);
        }
        part[blockIdx.x * 4 + 0] = t1;
        part[blockIdx.x * 4 + 1] = t2;
        part[blockIdx.x * 4 + 2] = fmin(mm[0][0], mn);
        part[blockIdx.x * 4 + 3] = fmax(mm[1][0], mx);
    }
}

// Moments pass 2: one wave folds the block partials — lane l takes blocks
// l, l+64, ... in order, then a fixed shuffle tree (deterministic).
__global__ void __launch_bounds__(64) k_moments_final(const double* __restrict__ part, int nb, int64_t N,
                                                      double* __restrict__ out) {
    const int lane = threadIdx.x;
    double s1 = 0.0, s2 = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    for (int b = lane; b < nb; b += 64) {
        s1 += part[b * 4 + 0];
        s2 += part[b * 4 + 1];
        mn = fmin(mn, part[b * 4 + 2]);
        mx = fmax(mx, part[b * 4 + 3]);
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, o, 64));
        mx = fmax(mx, __shfl_xor(mx, o, 64));
    }
    if (lane == 0) {
        out[0] = s1;
        out[1] = s2;
        out[2] = (double)N;
        out[3] = mn;
        out[4] = mx;
        out[5] = -mn;   // so one MAX all-reduce over out[4..5] gives the global extrema
    }
}

// ---------------------------------------------------------------------------
// One-launch statistics: the per-block partials of k_moments_part, then the LAST
// workgroup folds them in block order (common.h last_wg_fold, no grid barrier).
// Layout of rpart (MJRL_MOM_SCRATCH doubles): 4 partials per block, then the
// ticket word at MOM2_TICKET.
// ---------------------------------------------------------------------------
constexpr int MOM2_MAXB = 512;
// workgroups of one moments / whitening pass: one per 4096 elements, 16..256.
// Each takes a ticket on one counter (the last folds) and those atomics
// serialise, while too few workgroups leave each thread a long dependent load
// chain: 256 of them at 1M rows 15.6 us, 64 24 us; at 125k rows 64 beat 123
// (9.4 vs 9.6 us, whitening 7.7 vs 8.5)
__host__ __device__ inline int mom2_grid(int64_t n) {
    const int64_t g = n / 4096;
    return (int)(g < 16 ? 16 : (g > 256 ? 256 : g));
}
constexpr int MOM2_TICKET = 4 * MOM2_MAXB;

// block partial (s1, s2, min, max) of x[i0 + k * stride_blocks...] for one array
template <typename T>
__device__ __forceinline__ void mom_block(const T* __restrict__ x, int64_t N, double c, int blk, int nblk,
                                          double* red, double (&o)[4]) {
    double s1 = 0.0, s2 = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    const int64_t stride = (int64_t)nblk * blockDim.x;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < N; i += stride) {
        const double v = (double)x[i];
        const double dv = v - c;
        s1 += dv;
        s2 += dv * dv;
        mn = fmin(mn, v);
        mx = fmax(mx, v);
    }
    o[0] = block_sum<MOM_THREADS>(s1, red);
    o[1] = block_sum<MOM_THREADS>(s2, red);
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, k, 64));
        mx = fmax(mx, __shfl_xor(mx, k, 64));
    }
    __shared__ double mm[2][MOM_THREADS / 64];
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        mm[0][threadIdx.x >> 6] = mn;
        mm[1][threadIdx.x >> 6] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MOM_THREADS / 64; ++i) {
        mn = fmin(mn, mm[0][i]);
        mx = fmax(mx, mm[1][i]);
    }
    o[2] = mn;
    o[3] = mx;
}

// the last workgroup (wave 0) folds blocks [b0, b1) of the partials into out[6]
__device__ __forceinline__ void mom_fold(const double* part, int b0, int b1, int64_t N, double* out) {
    const int lane = threadIdx.x & 63;
    double s1 = 0.0, s2 = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    for (int b = b0 + lane; b < b1; b += 64) {
        s1 += __hip_atomic_load(part + 4 * b + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s2 += __hip_atomic_load(part + 4 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mn = fmin(mn, __hip_atomic_load(part + 4 * b + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        mx = fmax(mx, __hip_atomic_load(part + 4 * b + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, o, 64));
        mx = fmax(mx, __shfl_xor(mx, o, 64));
    }
    if (lane == 0) {
        out[0] = s1;
        out[1] = s2;
        out[2] = (double)N;
        out[3] = mn;
        out[4] = mx;
        out[5] = -mn;
    }
}

// publish this block's partial, take a ticket; true in the last block (wave 0)
__device__ __forceinline__ bool mom_publish(double* part, const double (&o)[4], int nb) {
    __shared__ unsigned tk;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) part[4 * blockIdx.x + k] = o[k];
        __threadfence();
        tk = atomicAdd(reinterpret_cast<unsigned*>(part + MOM2_TICKET), 1u);
    }
    __syncthreads();
    if (tk != (unsigned)(nb - 1)) return false;
    __threadfence();
    return threadIdx.x < 64;
}

// two arrays in one launch: blocks [0, nb1) take x1, [nb1, nb1 + nb2) take x2;
// centres c1 / c2 are moments outputs (mean = c[0] / c[2]) or null (0)
__global__ void __launch_bounds__(MOM_THREADS) k_moments2(const double* __restrict__ x1, int64_t N1,
                                                          const double* __restrict__ c1, const double* __restrict__ x2,
                                                          int64_t N2, const double* __restrict__ c2, int nb1, int nb2,
                                                          double* part, double* __restrict__ out1,
                                                          double* __restrict__ out2) {
    __shared__ double red[MOM_THREADS / 64];
    double o[4];
    const int b = blockIdx.x;
    if (b < nb1) {
        mom_block(x1, N1, c1 ? c1[0] / c1[2] : 0.0, b, nb1, red, o);
    } else {
        mom_block(x2, N2, c2 ? c2[0] / c2[2] : 0.0, b - nb1, nb2, red, o);
    }
    if (mom_publish(part, o, nb1 + nb2)) {
        mom_fold(part, 0, nb1, N1, out1);
        if (out2) mom_fold(part, nb1, nb1 + nb2, N2, out2);
        if (threadIdx.x == 0) *reinterpret_cast<unsigned*>(part + MOM2_TICKET) = 0u;
    }
}

// whitening of block blk of nblk (k_whiten's arithmetic) and the block partial of
// the f32 output's moments
__device__ __forceinline__ void whiten_block(const double* __restrict__ adv, int64_t T, double mean, double den,
                                             int blk, int nblk, float* __restrict__ adv32, double* __restrict__ w64,
                                             double* red, double (&o)[4]) {
    double s1 = 0.0, s2 = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    const int64_t stride = (int64_t)nblk * blockDim.x;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < T; i += stride) {
        const double w = (adv[i] - mean) / den;
        const float wf = (float)w;
        adv32[i] = wf;
        if (w64) w64[i] = w;
        const double v = (double)wf;
        s1 += v;
        s2 += v * v;
        mn = fmin(mn, v);
        mx = fmax(mx, v);
    }
    o[0] = block_sum<MOM_THREADS>(s1, red);
    o[1] = block_sum<MOM_THREADS>(s2, red);
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, k, 64));
        mx = fmax(mx, __shfl_xor(mx, k, 64));
    }
    __shared__ double mm[2][MOM_THREADS / 64];
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        mm[0][threadIdx.x >> 6] = mn;
        mm[1][threadIdx.x >> 6] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MOM_THREADS / 64; ++i) {
        mn = fmin(mn, mm[0][i]);
        mx = fmax(mx, mm[1][i]);
    }
    o[2] = mn;
    o[3] = mx;
}

// whitening (k_whiten) and, in the same launch, the moments of the f32 output
// (the surr_before numerator, npg_cg.py:113 with LR == 1)
__global__ void __launch_bounds__(MOM_THREADS) k_whiten_mom(const double* __restrict__ adv, int64_t T,
                                                            const double* __restrict__ m1,
                                                            const double* __restrict__ m2, double eps,
                                                            float* __restrict__ adv32, double* __restrict__ w64,
                                                            double* part, double* __restrict__ out) {
    __shared__ double red[MOM_THREADS / 64];
    const double mean = m1[0] / m1[2];
    const double sd = sqrt(m2[1] / m1[2]);
    const double den = sd + eps;
    double o[4];
    whiten_block(adv, T, mean, den, blockIdx.x, gridDim.x, adv32, w64, red, o);
    if (mom_publish(part, o, gridDim.x)) {
        mom_fold(part, 0, gridDim.x, T, out);
        if (threadIdx.x == 0) *reinterpret_cast<unsigned*>(part + MOM2_TICKET) = 0u;
    }
}

// adv32 = float((adv - mean) / (std + 1e-6)) (npg_cg.py:91; .float() at batch_reinforce.py:38)
__global__ void __launch_bounds__(256) k_whiten(const double* __restrict__ adv, int64_t T,
                                                const double* __restrict__ m1, const double* __restrict__ m2,
                                                double eps, float* __restrict__ adv32, double* __restrict__ w64) {
    const double mean = m1[0] / m1[2];
    const double sd = sqrt(m2[1] / m1[2]);
    const double den = sd + eps;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += stride) {
        const double w = (adv[i] - mean) / den;
        if (adv32) adv32[i] = (float)w;
        if (w64) w64[i] = w;
    }
}

// DAPG augmented advantages (dapg.py:65-70):
// all_adv = 1e-2 * concat(w / (std(w) + 1e-8), demo_coef * ones)
__global__ void __launch_bounds__(256) k_dapg_adv(const double* __restrict__ w64, int64_t T,
                                                  const double* __restrict__ mw1, const double* __restrict__ mw2,
                                                  int64_t T_demo, double demo_coef, float* __restrict__ adv_vpg) {
    const double sd = sqrt(mw2[1] / mw1[2]);
    const double den = sd + 1e-8;
    const float dv = (float)(1e-2 * demo_coef);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T + T_demo; i += stride)
        adv_vpg[i] = i < T ? (float)(1e-2 * (w64[i] / den)) : dv;
}

// LinearBaseline.predict for every path (baselines/linear_baseline.py:10-18,46-49):
// b_t = clip(o_t, -10, 10) . c[0:n] + (t/1000) c[n] + (t/1000)^2 c[n+1]
//       + (t/1000)^3 c[n+2] + c[n+3], t = index within the path.
// One wave per row (lanes across the observation, coalesced f64 loads), a
// grid-stride over rows; the row's path comes from a binary search of path_off.
template <typename TO>
__global__ void __launch_bounds__(256) k_linear_baseline(const TO* __restrict__ obs, int64_t T, int n,
                                                         const int64_t* __restrict__ off, int64_t P,
                                                         const double* __restrict__ coef, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t row = wave; row < T; row += nw) {
        double acc = 0.0;
        for (int j = lane; j < n; j += 64) {
            double o = obs[row * n + j];
            o = o < -10.0 ? -10.0 : (o > 10.0 ? 10.0 : o);
            acc += o * coef[j];
        }
        acc = wave_sum(acc);
        if (lane == 0) {
            int64_t lo = 0, hi = P;   // largest p with off[p] <= row
            while (hi - lo > 1) {
                const int64_t mid = (lo + hi) >> 1;
                if (off[mid] <= row) lo = mid; else hi = mid;
            }
            const double al = (double)(row - off[lo]) / 1000.0;
            acc += al * coef[n] + (al * al) * coef[n + 1] + pow(al, 3.0) * coef[n + 2] + coef[n + 3];
            out[row] = acc;
        }
    }
}

__global__ void __launch_bounds__(256) k_scale_vec(const float* __restrict__ gsum, int d, double scale,
                                                   float* __restrict__ g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < d) g[i] = (float)((double)gsum[i] * scale);
}

// dst[i] = src[idx[i]] (row copies; one wave per row, 16-B lanes when aligned)
template <typename V>
__global__ void __launch_bounds__(256) k_gather_rows(const V* __restrict__ src, int64_t row_v,
                                                     const int64_t* __restrict__ idx, int64_t n,
                                                     V* __restrict__ dst) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
        const V* s = src + idx[i] * row_v;
        V* d = dst + i * row_v;
        for (int64_t c = lane; c < row_v; c += 64) d[c] = s[c];
    }
}

// The same returns / advantages / path-return sums as k_gae by a wave-parallel
// scan (the north_star's "wavefront shuffles for the GAE prefix scan"): the
// recurrence y_t = x_t + c y_{t+1} is the composition of affine maps
// y -> x_t + c y, so one wave per path splits a window of up to 64 x GSC steps
// into 64 lane chunks, runs each chunk's recurrence from a zero carry (giving the
// chunk's map y -> a + c^len y), composes the 64 maps right to left with six
// __shfl_down steps, and fixes every element up with c^(distance) times the value
// entering its chunk.  Windows are walked from the path's end, carrying the
// value at the window start.  Not bit-identical to discount_sum (the products
// are regrouped): |error| <= ~1e-14 of the path's largest |y| at H = 1000
// (tests: rtol 1e-12 of the path maximum).  The path-return sum is a fixed-order
// wave reduction.  Selected by mjrl_gae_scan; mjrl_gae stays the exact default.
constexpr int GSC = 16;   // steps per lane per window (window = 1024 steps)

__device__ __forceinline__ void affine_scan_down(double& a, double& m, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double ao = __shfl_down(a, o, 64), mo = __shfl_down(m, o, 64);
        if (lane + o < 64) {
            a = a + m * ao;
            m = m * mo;
        }
    }
}

__global__ void __launch_bounds__(256) k_gae_scan(const double* __restrict__ rew, const double* __restrict__ base,
                                                  const int64_t* __restrict__ off,
                                                  const uint8_t* __restrict__ term, int64_t P, double gamma,
                                                  double gl, int use_gae, double* __restrict__ ret,
                                                  double* __restrict__ adv, double* __restrict__ path_ret) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < P; p += nw) {
        const int64_t b = off[p], e = off[p + 1];
        const double blast = e > b ? (term[p] ? 0.0 : base[e - 1]) : 0.0;
        double carry_r = 0.0, carry_a = 0.0, total = 0.0;
        for (int64_t w1 = e; w1 > b; w1 -= 64 * GSC) {
            const int64_t w0 = w1 - 64 * GSC > b ? w1 - 64 * GSC : b;
            const int cnt = (int)(w1 - w0);
            const int C = (cnt + 63) / 64;
            const int c0 = lane * C;
            const int len = c0 < cnt ? (cnt - c0 < C ? cnt - c0 : C) : 0;
            double r[GSC], yr[GSC], ya[GSC];
            double sr = 0.0, ar = 0.0, aa = 0.0, mr = 1.0, ma = 1.0;
#pragma unroll
            for (int k = 0; k < GSC; ++k) r[k] = k < len ? rew[w0 + c0 + k] : 0.0;
#pragma unroll
            for (int k = GSC - 1; k >= 0; --k) {
                if (k < len) {
                    const int64_t i = w0 + c0 + k;
                    const double bb = base[i];
                    const double bn = i + 1 < e ? base[i + 1] : blast;
                    const double td = use_gae ? (r[k] + gamma * bn) - bb : 0.0;
                    ar = r[k] + gamma * ar;
                    aa = td + gl * aa;
                    mr *= gamma;
                    ma *= gl;
                    yr[k] = ar;
                    ya[k] = aa;
                    sr += r[k];
                }
            }
            // maps of this lane's chunk: y_in -> a + m y_in; compose lanes right to left
            affine_scan_down(ar, mr, lane);
            affine_scan_down(aa, ma, lane);
            // value entering this lane's chunk from the right: lane + 1's composed map
            // applied to the window carry (lane 63: the carry itself)
            const double Yr = ar + mr * carry_r, Ya = aa + ma * carry_a;
            double nr = __shfl_down(Yr, 1, 64), na = __shfl_down(Ya, 1, 64);
            if (lane == 63 || c0 + len >= cnt) {
                nr = carry_r;
                na = carry_a;
            }
            double pr = gamma, pa = gl;
#pragma unroll
            for (int k = GSC - 1; k >= 0; --k) {
                if (k < len) {
                    const int64_t i = w0 + c0 + k;
                    const double rv = yr[k] + pr * nr;
                    ret[i] = rv;
                    adv[i] = use_gae ? ya[k] + pa * na : rv - base[i];
                    pr *= gamma;
                    pa *= gl;
                }
            }
            carry_r = __shfl(Yr, 0, 64);
            carry_a = __shfl(Ya, 0, 64);
            total += wave_sum_d(sr);
        }
        if (lane == 0) path_ret[p] = total;
    }
}

inline int grid_for(int64_t work, int per_block, int cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

inline int err(hipError_t e) { return e == hipSuccess ? MJRL_OK : (int)e; }

}  // namespace

extern "C" {

extern "C++" {
template <typename TO>
static int pack_batch(const TO* obs, const TO* act, int64_t T, const mjrl_shape* s, const float* in_shift,
                      const float* in_scale, float* xhat, float* act32, void* stream) {
    if (!s || T < 0 || (T > 0 && (!obs || !act || !xhat || !act32))) return MJRL_EINVAL;
    if ((in_shift == nullptr) != (in_scale == nullptr)) return MJRL_EINVAL;
    if (T == 0) return MJRL_OK;
    const int g = grid_for(T * (s->np / 4), 256, 2048);
    hipLaunchKernelGGL(k_pack_batch<TO>, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, act, T, s->n, s->m, s->np,
                       in_shift, in_scale, xhat, act32);
    return err(hipGetLastError());
}
}  // extern "C++"

extern "C++" {
template <typename TO>
static int pack_batch_split(const TO* obs, const TO* act, int64_t T, const mjrl_shape* s, const float* in_shift,
                            const float* in_scale, const float* xc, void* xs, float* xu, float* act32,
                            void* stream) {
    if (!s || T < 0 || (T > 0 && (!obs || !act || !xc || !xs || !xu || !act32))) return MJRL_EINVAL;
    if ((in_shift == nullptr) != (in_scale == nullptr)) return MJRL_EINVAL;
    if (s->np > 128 * PS_MAXP) return MJRL_ESHAPE;
    if (T == 0) return MJRL_OK;
    const int g = grid_for(T, 4, 8192);
    if constexpr (sizeof(TO) == 4) {
        if (s->n % 4 == 0 && (reinterpret_cast<uintptr_t>(obs) & 15) == 0 && s->np % 4 == 0 && s->np <= 256 * PQ_MAXQ) {
            hipLaunchKernelGGL(k_pack_split_q, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, act, T, s->n, s->m,
                               s->np, in_shift, in_scale, xc, (_Float16*)xs, xu, act32);
            return err(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(k_pack_split<TO>, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, act, T, s->n, s->m, s->np,
                       in_shift, in_scale, xc, (_Float16*)xs, xu, act32);
    return err(hipGetLastError());
}

// column maxima -> power-of-two column scales, in place (one workgroup)
__global__ void k_colscale(float* xc, int np) {
    for (int k = threadIdx.x; k < np; k += blockDim.x) xc[k] = col_scale(xc[k]);
}

// The same scales from per-column ranges [cmin, cmax] of the f32 observations
// (taken by the host staging pass, mjrl_host_stage_*): x -> (x - shift) / (scale
// + 1e-8) is the pack's f32 expression, monotone in x (each rounding is), so the
// column max of |xhat| over the batch is attained at cmin or cmax: the result is
// bit for bit k_colmax's.  An empty column range (cmin > cmax: no rows) gives 1.
__global__ void k_colscale_range(const float* __restrict__ cmin, const float* __restrict__ cmax, int n, int np,
                                 const float* __restrict__ in_shift, const float* __restrict__ in_scale,
                                 float* __restrict__ xc) {
    for (int k = threadIdx.x; k < np; k += blockDim.x) {
        float m = 0.f;
        if (k < n) {
            float lo = cmin[k], hi = cmax[k];
            if (lo <= hi) {
                if (in_shift) {
                    const float den = in_scale[k] + 1e-8f;
                    lo = (lo - in_shift[k]) / den;   // MuNet.forward:177, as the pack
                    hi = (hi - in_shift[k]) / den;
                }
                m = fmaxf(fabsf(lo), fabsf(hi));
            }
        } else if (k == n) {
            m = 1.f;   // the bias column
        }
        xc[k] = col_scale(m);
    }
}

// Sharded moments (the all-gather form of npg_cg.py:91, 97-102 over shards):
// g[world][rec] holds every rank's local pass-1 moments (mjrl_moments format, at
// 16 j + 0..5 for group j) and its pass-2 moments centred on the rank's OWN mean
// (16 j + 8..13).  Thread j folds group j over the ranks in rank order: N = sum
// n_r, S = sum S_r, mean = S / N, and the centred sum of squares about the global
// mean, M2 = sum_r [M2_r + 2 (m_r - mean) D_r + n_r (m_r - mean)^2] (m_r = S_r /
// n_r, D_r = sum (x - m_r): exact algebra, only rounding differs from one pass
// about the global mean; with one rank m_0 == mean and M2 = M2_0 bit for bit).
// out[16 j + 0..5] / out[16 j + 8..13] receive the global pass-1 / pass-2 moments.
__global__ void k_moments_combine(const double* __restrict__ g, int world, int rec, int ngroups,
                                  double* __restrict__ out) {
    const int j = threadIdx.x;
    if (j >= ngroups) return;
    double N = 0.0, S = 0.0, SS = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
    for (int r = 0; r < world; ++r) {
        const double* p = g + (int64_t)r * rec + 16 * j;
        S += p[0];
        SS += p[1];
        N += p[2];
        mn = fmin(mn, p[3]);
        mx = fmax(mx, p[4]);
    }
    const double mean = S / N;
    double D = 0.0, M2 = 0.0;
    for (int r = 0; r < world; ++r) {
        const double* p = g + (int64_t)r * rec + 16 * j;
        const double nr = p[2];
        if (!(nr > 0.0)) continue;
        const double dm = p[0] / nr - mean;
        M2 += p[9] + 2.0 * dm * p[8] + nr * dm * dm;
        D += p[8] + nr * dm;
    }
    double* o1 = out + 16 * j;
    double* o2 = o1 + 8;
    o1[0] = S; o1[1] = SS; o1[2] = N; o1[3] = mn; o1[4] = mx; o1[5] = -mn;
    o2[0] = D; o2[1] = M2; o2[2] = N; o2[3] = mn; o2[4] = mx; o2[5] = -mn;
}

template <typename TO>
static int obs_colscale(const TO* obs, int64_t T, const mjrl_shape* s, const float* in_shift, const float* in_scale,
                        float* xc, void* stream) {
    if (!s || T < 0 || !xc || (T > 0 && !obs)) return MJRL_EINVAL;
    if ((in_shift == nullptr) != (in_scale == nullptr)) return MJRL_EINVAL;
    if (s->np > 512 || s->n >= s->np) return MJRL_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(xc, 0, sizeof(float) * s->np, st);
    if (e != hipSuccess) return (int)e;
    const bool q4 = sizeof(TO) == 4 && s->n % 4 == 0 && (reinterpret_cast<uintptr_t>(obs) & 15) == 0;
    const int nv = q4 ? s->n / 4 : s->n;
    // 512 workgroups: 512 atomicMax per column (2048 took 56 vs 41 us at 125k rows,
    // the same 290-300 us at 1M: tools/colmax_probe.py, profiles/r03i/colmax_probe.txt)
    constexpr int NT = 512;
    const int rpp = NT / nv;
    const int g = T > 0 ? grid_for(T, rpp * 16, 512) : 1;
    if (q4)
        hipLaunchKernelGGL((k_colmax<TO, 4, NT>), dim3(g), dim3(NT), 0, st, obs, T, s->n, in_shift, in_scale,
                           reinterpret_cast<unsigned*>(xc));
    else
        hipLaunchKernelGGL((k_colmax<TO, 1, NT>), dim3(g), dim3(NT), 0, st, obs, T, s->n, in_shift, in_scale,
                           reinterpret_cast<unsigned*>(xc));
    hipLaunchKernelGGL(k_colscale, dim3(1), dim3(512), 0, st, xc, s->np);
    return err(hipGetLastError());
}
}  // extern "C++"

int mjrl_pack_batch(const double* obs, const double* act, int64_t T, const mjrl_shape* s, const float* in_shift,
                    const float* in_scale, float* xhat, float* act32, void* stream) {
    return pack_batch(obs, act, T, s, in_shift, in_scale, xhat, act32, stream);
}

int mjrl_pack_batch_f32(const float* obs, const float* act, int64_t T, const mjrl_shape* s, const float* in_shift,
                        const float* in_scale, float* xhat, float* act32, void* stream) {
    return pack_batch(obs, act, T, s, in_shift, in_scale, xhat, act32, stream);
}

int mjrl_obs_colscale(const double* obs, int64_t T, const mjrl_shape* s, const float* in_shift,
                      const float* in_scale, float* xc, void* stream) {
    return obs_colscale(obs, T, s, in_shift, in_scale, xc, stream);
}

int mjrl_obs_colscale_f32(const float* obs, int64_t T, const mjrl_shape* s, const float* in_shift,
                          const float* in_scale, float* xc, void* stream) {
    return obs_colscale(obs, T, s, in_shift, in_scale, xc, stream);
}

int mjrl_obs_colscale_range(const float* cmin, const float* cmax, const mjrl_shape* s, const float* in_shift,
                            const float* in_scale, float* xc, void* stream) {
    if (!s || !cmin || !cmax || !xc) return MJRL_EINVAL;
    if ((in_shift == nullptr) != (in_scale == nullptr)) return MJRL_EINVAL;
    if (s->np > 512 || s->n >= s->np) return MJRL_ESHAPE;
    hipLaunchKernelGGL(k_colscale_range, dim3(1), dim3(512), 0, (hipStream_t)stream, cmin, cmax, s->n, s->np, in_shift,
                       in_scale, xc);
    return err(hipGetLastError());
}

int mjrl_moments_combine(const double* gathered, int32_t world, int32_t rec, int32_t ngroups, double* out,
                         void* stream) {
    if (!gathered || !out || world < 1 || ngroups < 1 || ngroups > 64 || rec < 16 * ngroups) return MJRL_EINVAL;
    hipLaunchKernelGGL(k_moments_combine, dim3(1), dim3(64), 0, (hipStream_t)stream, gathered, world, rec, ngroups,
                       out);
    return err(hipGetLastError());
}

int mjrl_pack_batch_split(const double* obs, const double* act, int64_t T, const mjrl_shape* s,
                          const float* in_shift, const float* in_scale, const float* xc, void* xs, float* xu,
                          float* act32, void* stream) {
    return pack_batch_split(obs, act, T, s, in_shift, in_scale, xc, xs, xu, act32, stream);
}

int mjrl_pack_batch_split_f32(const float* obs, const float* act, int64_t T, const mjrl_shape* s,
                              const float* in_shift, const float* in_scale, const float* xc, void* xs, float* xu,
                              float* act32, void* stream) {
    return pack_batch_split(obs, act, T, s, in_shift, in_scale, xc, xs, xu, act32, stream);
}

int mjrl_gae_scan(const double* rew, const double* base, const int64_t* path_off, const uint8_t* terminated,
                  int64_t P, double gamma, double gae_lambda, int32_t use_gae, double* ret, double* adv,
                  double* path_ret, void* stream) {
    if (P < 0 || (P > 0 && (!rew || !base || !path_off || !terminated || !ret || !adv || !path_ret)))
        return MJRL_EINVAL;
    if (P == 0) return MJRL_OK;
    const double gl = gamma * gae_lambda;
    const int64_t g = (P + 3) / 4;   // four waves (paths) per workgroup
    hipLaunchKernelGGL(k_gae_scan, dim3((unsigned)(g < 8192 ? g : 8192)), dim3(256), 0, (hipStream_t)stream, rew,
                       base, path_off, terminated, P, gamma, gl, use_gae, ret, adv, path_ret);
    return err(hipGetLastError());
}

int mjrl_gae(const double* rew, const double* base, const int64_t* path_off, const uint8_t* terminated, int64_t P,
             double gamma, double gae_lambda, int32_t use_gae, double* ret, double* adv, double* path_ret,
             void* stream) {
    if (P < 0 || (P > 0 && (!rew || !base || !path_off || !terminated || !ret || !adv || !path_ret)))
        return MJRL_EINVAL;
    if (P == 0) return MJRL_OK;
    const double gl = gamma * gae_lambda;   // python: gamma*gae_lambda (process_samples.py:29)
    const int64_t g = (P + LP_PATHS - 1) / LP_PATHS;
    hipLaunchKernelGGL(k_gae_lp, dim3((unsigned)g), dim3(LP_T), 0, (hipStream_t)stream, rew, base, path_off,
                       terminated, P, gamma, gl, use_gae, ret, adv, path_ret);
    return err(hipGetLastError());
}

// The one-wave-per-path kernel (rounds 1-5), kept for A/B (tools/gae_probe.py).
int mjrl_gae_wave(const double* rew, const double* base, const int64_t* path_off, const uint8_t* terminated,
                  int64_t P, double gamma, double gae_lambda, int32_t use_gae, double* ret, double* adv,
                  double* path_ret, void* stream) {
    if (P < 0 || (P > 0 && (!rew || !base || !path_off || !terminated || !ret || !adv || !path_ret)))
        return MJRL_EINVAL;
    if (P == 0) return MJRL_OK;
    const double gl = gamma * gae_lambda;
    const int64_t g = (P + GAE_WAVES - 1) / GAE_WAVES;
    hipLaunchKernelGGL(k_gae, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(64 * GAE_WAVES), 0, (hipStream_t)stream, rew,
                       base, path_off, terminated, P, gamma, gl, use_gae, ret, adv, path_ret);
    return err(hipGetLastError());
}

static int moments_impl(bool f32, const void* x, int64_t N, const double* center, double* rpart, double* out,
                        void* stream) {
    if (N < 0 || !rpart || !out || (N > 0 && !x)) return MJRL_EINVAL;
    const int nb = grid_for(N, MOM_THREADS * 4, MOM_BLOCKS);
    if (f32)
        hipLaunchKernelGGL(k_moments_part<float>, dim3(nb), dim3(MOM_THREADS), 0, (hipStream_t)stream,
                           (const float*)x, N, center, rpart);
    else
        hipLaunchKernelGGL(k_moments_part<double>, dim3(nb), dim3(MOM_THREADS), 0, (hipStream_t)stream,
                           (const double*)x, N, center, rpart);
    hipLaunchKernelGGL(k_moments_final, dim3(1), dim3(64), 0, (hipStream_t)stream, rpart, nb, N, out);
    return err(hipGetLastError());
}

int mjrl_moments2(const double* x1, int64_t N1, const double* c1, const double* x2, int64_t N2, const double* c2,
                  double* rpart, double* out1, double* out2, void* stream) {
    if (N1 < 0 || N2 < 0 || !rpart || !out1 || (N1 > 0 && !x1) || (out2 && N2 > 0 && !x2)) return MJRL_EINVAL;
    const int nb1 = grid_for(N1, MOM_THREADS * 4, mom2_grid(N1));
    const int nb2 = out2 ? grid_for(N2, MOM_THREADS * 4, mom2_grid(N2)) : 0;
    hipLaunchKernelGGL(k_moments2, dim3(nb1 + nb2), dim3(MOM_THREADS), 0, (hipStream_t)stream, x1, N1, c1, x2, N2, c2,
                       nb1, nb2, rpart, out1, out2);
    return err(hipGetLastError());
}

int mjrl_whiten_moments(const double* adv, int64_t T, const double* m1, const double* m2, double eps, float* adv32,
                        double* w64, double* rpart, double* out, void* stream) {
    if (T < 0 || !adv || !m1 || !m2 || !adv32 || !rpart || !out) return MJRL_EINVAL;
    const int nb = grid_for(T, MOM_THREADS * 4, mom2_grid(T));
    hipLaunchKernelGGL(k_whiten_mom, dim3(nb), dim3(MOM_THREADS), 0, (hipStream_t)stream, adv, T, m1, m2, eps, adv32,
                       w64, rpart, out);
    return err(hipGetLastError());
}

int mjrl_moments(const double* x, int64_t N, const double* center, double* rpart, double* out, void* stream) {
    return moments_impl(false, x, N, center, rpart, out, stream);
}

int mjrl_moments_f32(const float* x, int64_t N, const double* center, double* rpart, double* out, void* stream) {
    return moments_impl(true, x, N, center, rpart, out, stream);
}

int mjrl_whiten(const double* adv, int64_t T, const double* m1, const double* m2, double eps, float* adv32,
                double* w64, void* stream) {
    if (T < 0 || !m1 || !m2 || (T > 0 && (!adv || (!adv32 && !w64)))) return MJRL_EINVAL;
    if (T == 0) return MJRL_OK;
    hipLaunchKernelGGL(k_whiten, dim3(grid_for(T, 256, 2048)), dim3(256), 0, (hipStream_t)stream, adv, T, m1, m2,
                       eps, adv32, w64);
    return err(hipGetLastError());
}

int mjrl_dapg_adv(const double* w64, int64_t T, const double* mw1, const double* mw2, int64_t T_demo,
                  double demo_coef, float* adv_vpg, void* stream) {
    if (T < 0 || T_demo < 0 || !mw1 || !mw2 || !adv_vpg || (T > 0 && !w64)) return MJRL_EINVAL;
    if (T + T_demo == 0) return MJRL_OK;
    hipLaunchKernelGGL(k_dapg_adv, dim3(grid_for(T + T_demo, 256, 2048)), dim3(256), 0, (hipStream_t)stream, w64,
                       T, mw1, mw2, T_demo, demo_coef, adv_vpg);
    return err(hipGetLastError());
}

extern "C++" {
template <typename TO>
static int linear_baseline(const TO* obs, int64_t T, int32_t n, const int64_t* path_off, int64_t P,
                           const double* coeffs, double* out, void* stream) {
    if (T < 0 || n <= 0 || P < 0 || (T > 0 && (!obs || !path_off || !coeffs || !out))) return MJRL_EINVAL;
    if (T == 0) return MJRL_OK;
    const int g = grid_for(T * 64, 256, 4096);
    hipLaunchKernelGGL(k_linear_baseline<TO>, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, T, n, path_off, P,
                       coeffs, out);
    return err(hipGetLastError());
}
}  // extern "C++"

int mjrl_linear_baseline(const double* obs, int64_t T, int32_t n, const int64_t* path_off, int64_t P,
                         const double* coeffs, double* out, void* stream) {
    return linear_baseline(obs, T, n, path_off, P, coeffs, out, stream);
}

int mjrl_linear_baseline_f32(const float* obs, int64_t T, int32_t n, const int64_t* path_off, int64_t P,
                             const double* coeffs, double* out, void* stream) {
    return linear_baseline(obs, T, n, path_off, P, coeffs, out, stream);
}

int mjrl_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t n, void* dst, void* stream) {
    if (n < 0 || row_bytes < 0 || row_bytes % 4 != 0 || (n > 0 && (!src || !idx || !dst))) return MJRL_EINVAL;
    if (n == 0 || row_bytes == 0) return MJRL_OK;
    const int g = grid_for(n, 4, 8192);   // 4 rows (waves) per workgroup
    const bool v16 = row_bytes % 16 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0;
    if (v16)
        hipLaunchKernelGGL(k_gather_rows<float4>, dim3(g), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)src, row_bytes / 16, idx, n, (float4*)dst);
    else
        hipLaunchKernelGGL(k_gather_rows<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)src,
                           row_bytes / 4, idx, n, (float*)dst);
    return err(hipGetLastError());
}

int mjrl_scale_vec(const float* gsum, int32_t d, double scale, float* g, void* stream) {
    if (d < 0 || (d > 0 && (!gsum || !g))) return MJRL_EINVAL;
    if (d == 0) return MJRL_OK;
    hipLaunchKernelGGL(k_scale_vec, dim3((d + 255) / 256), dim3(256), 0, (hipStream_t)stream, gsum, d, scale, g);
    return err(hipGetLastError());
}

}  // extern "C"
