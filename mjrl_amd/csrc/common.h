// common.h — shared device building blocks for the gfx950 update-path kernels.
//
// Everything here is written for CDNA4 directly: 64-lane waves, the exact-f32
// MFMA `v_mfma_f32_16x16x4_f32`, LDS-staged operands.  No CUDA shims.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mjrl_amd.h"

#ifdef MJRL_KX_PROF
// phase profile (profiling builds) of k_kx / k_fused: wave 0 of block 0 accumulates s_memtime cycles
// between stamps in (wave-uniform, scalar) registers, written once at the end;
// read with mjrl_debug_kx_prof
constexpr int KX_NPROF = 24;   // 0-14 phases, 15 launch preamble, 16 tail (slab writes), 17 launches, 18-23 preamble parts
__device__ unsigned long long g_kx_prof[KX_NPROF];
#define KX_STAMP(i)                                                     \
    do {                                                                \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
        kx_acc_[i] += now_ - kx_last_;                                  \
        kx_last_ = now_;                                                \
    } while (0)
#define KX_PRE(i) kx_pre_[i] = __builtin_amdgcn_s_memtime()
#else
#define KX_PRE(i) \
    do {          \
    } while (0)
#define KX_STAMP(i) \
    do {            \
    } while (0)
#endif

namespace mjrl {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;
constexpr int NTHREADS = 256;   // 4 waves per workgroup for the row / wgrad kernels

__device__ __forceinline__ floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

// D = A(16x4) * B(4x16) + C, exact f32 (a k-ordered fma chain).
// Lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; D[(l>>4)*4+r][l&15] = c[r].
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Four MFMAs over one 16-wide k group.  Lane group q = lane>>4 owns
// k = 16g + 4q + s for step s, so both operands come in as one float4 each
// (the same permutation on A and B keeps the product exact).
__device__ __forceinline__ floatx4 mfma_k16(const float4& a, const float4& b, floatx4 c) {
    c = mfma4(a.x, b.x, c);
    c = mfma4(a.y, b.y, c);
    c = mfma4(a.z, b.z, c);
    c = mfma4(a.w, b.w, c);
    return c;
}

// ---------------------------------------------------------------------------
// Split-f16 operands ("fp16x3"): an f32 value y of a block scaled by a power of
// two is carried as hi = f16(y) and lo = f16(y - hi) (round to nearest; y - hi is
// exact).  A product of two split operands is hi*hi + hi*lo + lo*hi, three
// v_mfma_f32_16x16x32_f16 into ONE f32 accumulator (f16 products are exact),
// dropping only lo*lo.  Three f16 MFMAs carry 8x the k of one
// v_mfma_f32_16x16x4_f32 in half its cycles: 5.3x the f32 matrix rate.
//
// Block scale with headroom: the block's max |y| goes to [2^14, 2^15), the top of
// the f16 range (not [1/2, 1)).  Element error of the pair, for every y of the block:
//     |hi + lo - y| <= 2^-23 |y| + 2^-25,
// the second term being lo's subnormal floor (f16 subnormals are 2^-24 apart).
// Relative to the block max B that is 2^-23 |y| + 2^-40 B: every element down to
// 2^-17 of its block max keeps 23 bits (f32 rounding is 2^-24), and the absolute
// floor sits 40 binades below the max, where a [1/2, 1) block had it at 2^-25 B
// (an element 1e-6 of its row max then lost everything).  Products stay far inside
// f32: |hi * hi| < 2^30, a K = 384 sum < 2^39.
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx4 mfma_h(const half8& a, const half8& b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// c += (ah + al)(bh + bl) - al bl
__device__ __forceinline__ floatx4 mfma_x3(const half8& ah, const half8& al, const half8& bh, const half8& bl,
                                           floatx4 c) {
    c = mfma_h(ah, bh, c);
    c = mfma_h(ah, bl, c);
    return mfma_h(al, bh, c);
}

constexpr int SPLIT_HR = 15;   // block max -> [2^(SPLIT_HR-1), 2^SPLIT_HR)

// Power-of-two scale for a block whose max |value| is M: returns s = 2^(15-E) with
// M * s in [2^14, 2^15) and sets inv = 1 / s = 2^(E-15) (s = inv = 1 for M == 0 /
// non-finite; blocks below 2^-111 keep s = 2^126).
__device__ __forceinline__ float pow2_scale(float M, float& inv) {
    if (!(M > 0.f) || !(M < 3.0e38f)) {
        inv = 1.f;
        return 1.f;
    }
    int E;
    frexpf(M, &E);
    E = E < -111 ? -111 : E;
    inv = ldexpf(1.f, E - SPLIT_HR);
    return ldexpf(1.f, SPLIT_HR - E);
}

// Split xhat rows (mjrl_rows.xs): column k carries xhat / xc[k] with xc[k] = 2^E the
// power of two with colmax[k] 2^-E in [1/2, 1) over the batch (1 for an all-zero
// column), then each row is scaled by its own power of two (xu[t], headroom as
// above).  Then |xc xu (hi + lo) - xhat| <= 2^-23 |xhat| + 2^-39 xc_k r_t, r_t =
// max_j |xhat[t][j]| / xc_j < 1, so at most 2^-23 |xhat| + 2^-38 colmax_k: a
// small-scale feature keeps 23 bits in rows dominated by large ones.
__device__ __forceinline__ float col_scale(float cmax) {
    if (!(cmax > 0.f) || !(cmax < 3.0e38f)) return 1.f;
    int E;
    frexpf(cmax, &E);
    E = E < -100 ? -100 : (E > 100 ? 100 : E);
    return ldexpf(1.f, E);
}

// Cached tanh activations (|a| <= 1) are split into their LDS images with the fixed
// scale 2^14 (the same headroom); consumers multiply by AHR_INV (exact).
constexpr float AHR = 16384.f;
constexpr float AHR_INV = 1.f / 16384.f;

typedef float float8v __attribute__((ext_vector_type(8)));
typedef short short8v __attribute__((ext_vector_type(8)));

typedef unsigned uint4v __attribute__((ext_vector_type(4)));

// lo = f16(y - hi) for 8 values (hi: 4 packed f16 pairs; y: f32): v_fma_mixlo_f16 /
// v_fma_mixhi_f16 compute hi * -1 + y exactly in f32 and round once to f16 (y - hi is
// exact, so this equals f16((float)(y - hi))), one instruction per value instead of an
// f16 -> f32 conversion, a subtraction and a conversion back.  One asm statement; it
// ends with the 2 wait states a VALU-written VGPR needs before an MFMA reads it (hipcc
// pads nothing for an asm producer, cdna_hip_programming.md §5.7 item 2).
__device__ __forceinline__ uint4v mix_lo8(const uint4v& h, const float8v& y) {
    uint4v l;
    asm("v_fma_mixlo_f16 %0, %4, -1.0, %8 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %4, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixlo_f16 %1, %5, -1.0, %10 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %1, %5, -1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixlo_f16 %2, %6, -1.0, %12 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %2, %6, -1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixlo_f16 %3, %7, -1.0, %14 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %3, %7, -1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
        "s_nop 1"
        : "=&v"(l[0]), "=&v"(l[1]), "=&v"(l[2]), "=&v"(l[3])
        : "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]),
          "v"(y[5]), "v"(y[6]), "v"(y[7]));
    return l;
}

// the same for one pair (results feed VALU code only: no MFMA wait states needed)
__device__ __forceinline__ unsigned mix_lo2(unsigned hi2, float y0, float y1) {
    unsigned t;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(t) : "v"(hi2), "v"(y0), "v"(y1));
    return t;
}

// hi / lo of y = v * s (packed v_cvt_pk_f16_f32, round to nearest; lo via mix_lo8)
__device__ __forceinline__ void split8(const float8v& v, float s, half8& hi, half8& lo) {
    const float8v y = v * s;
    hi = __builtin_convertvector(y, half8);
    lo = __builtin_bit_cast(half8, mix_lo8(__builtin_bit_cast(uint4v, hi), y));
}

// (float)hi + (float)lo for the two halves of packed f16 pairs (v_fma_mix_f32: hi * 1 + lo,
// exact in f32)
__device__ __forceinline__ float mix_add_lo(unsigned h2, unsigned l2) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(h2), "v"(l2));
    return r;
}
__device__ __forceinline__ float mix_add_hi(unsigned h2, unsigned l2) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(h2), "v"(l2));
    return r;
}
__device__ __forceinline__ float8v hilo8(const half8& hh, const half8& ll) {
    const uint4v h = __builtin_bit_cast(uint4v, hh), l = __builtin_bit_cast(uint4v, ll);
    float8v r;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        r[2 * p] = mix_add_lo(h[p], l[p]);
        r[2 * p + 1] = mix_add_hi(h[p], l[p]);
    }
    return r;
}

__device__ __forceinline__ float8v load8(const float* p) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    return float8v{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}

__device__ __forceinline__ float absmax8(const float8v& v) {
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
    return m;
}

// Exchange across 16-lane groups with the gfx950 lane-swap VALU ops (no LDS
// round trip): permlane16_swap(x, x) gives every lane {x[l], x[l ^ 16]} in
// (lower group, upper group) order, permlane32_swap(x, x) {x[l], x[l ^ 32]}
// likewise (checked by tools/permlane_check.hip).
__device__ __forceinline__ float max_over_groups(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// sum over the four 16-lane groups, the same fixed order in every lane
__device__ __forceinline__ float sum_over_groups(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4r+p addresses row r,
// columns 4p..4p+3 of a 4 x 16 block of 16-bit values; lane i receives column i
// (row r in element r).  EXEC must be all ones.
__device__ __forceinline__ short4v ds_read_tr16(const void* p) {
    typedef __attribute__((address_space(3))) short4v lds_short4;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(p));
}

// ---------------------------------------------------------------------------
// Wave decomposition of an output tile [BT x N] (BT = 16*RB rows, N = 16*CB cols)
// over the 4 waves of a workgroup: each wave owns NRW row blocks x NCW col blocks
// and loads one B (weight) fragment per col block per k-step, reused across its
// row blocks.
// ---------------------------------------------------------------------------
template <int RB, int CB, int NW = 4>
struct Split {
    // CB >= NW: wave w owns col blocks w, w + NW, ... over every row block;
    // CB < NW: NW / CB waves share a col block, each a strided set of row blocks
    static constexpr int WPC = CB >= NW ? 1 : NW / CB;                 // waves per col block
    static constexpr int NCW = CB >= NW ? CB / NW : 1;
    static constexpr int NRW = CB >= NW ? RB : (RB + WPC - 1) / WPC;
    static constexpr int CBS = CB >= NW ? NW : 1;                      // col block stride
    static constexpr int RBS = CB >= NW ? 1 : WPC;
    __device__ static int cb0(int w) { return CB >= NW ? w : w % CB; }
    __device__ static int rb0(int w) { return CB >= NW ? 0 : w / CB; }
};

// acc[i][j] += A[rows of rb(i)][k] * W[cols of cb(j)][k], k in [kb, ke) (multiples of 16).
// A: LDS row-major (lda floats), columns offset by a_col0 relative to k.
// W: global row-major [N][ldw] (weights, L2-resident).
template <int NRW, int NCW>
__device__ __forceinline__ void gemm_tile(floatx4 (&acc)[NRW][NCW], const float* As, int lda, int a_col0,
                                          int rb0, int rbs, int rb_lim, const float* __restrict__ W, int ldw,
                                          int cb0, int cbs, int kb, int ke, int lane) {
    const int r = lane & 15, q = lane >> 4;
#ifndef MJRL_GEMM_UNROLL
#define MJRL_GEMM_UNROLL 8   // k-steps in flight: 8 measured -6 % on k_rows<256> (c5), -1.5 % on k_rows<128> (c3) vs 2
#endif
#pragma unroll MJRL_GEMM_UNROLL
    for (int k = kb; k < ke; k += 16) {
        float4 b[NCW];
#pragma unroll
        for (int j = 0; j < NCW; ++j)
            b[j] = *reinterpret_cast<const float4*>(W + (size_t)((cb0 + j * cbs) * 16 + r) * ldw + k + 4 * q);
#pragma unroll
        for (int i = 0; i < NRW; ++i) {
            const int rb = rb0 + i * rbs;
            if (rb >= rb_lim) continue;
            const float4 a = *reinterpret_cast<const float4*>(As + (rb * 16 + r) * lda + (k - a_col0) + 4 * q);
#pragma unroll
            for (int j = 0; j < NCW; ++j) acc[i][j] = mfma_k16(a, b[j], acc[i][j]);
        }
    }
}

template <int NRW, int NCW>
__device__ __forceinline__ void zero_acc(floatx4 (&acc)[NRW][NCW]) {
#pragma unroll
    for (int i = 0; i < NRW; ++i)
#pragma unroll
        for (int j = 0; j < NCW; ++j) acc[i][j] = zero4();
}

// ---------------------------------------------------------------------------
// Deterministic block reductions (fixed tree order).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NT>
__device__ __forceinline__ double block_sum(double v, double* red /* LDS, >= NT/64 */) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) s += red[i];
    return s;
}

__host__ __device__ __forceinline__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// Debug build only (-DMJRL_DEVICE_CHECKS: python -m mjrl_amd.build --debug ->
// lib/libmjrl_amd_dbg.so): every weight-gradient slab index is checked against
// the scratch the caller sized with mjrl_scratch_size (wcap floats, passed in the
// kernel arguments), and a bad one prints the kernel's file:line, workgroup,
// index and bound, then traps.  Release builds compile the checks out.
// ---------------------------------------------------------------------------
#ifdef MJRL_DEVICE_CHECKS
#define MJRL_SLAB_CHECK(idx, cap)                                                                          \
    do {                                                                                                 \
        const int64_t i_ = (int64_t)(idx), c_ = (int64_t)(cap);                                          \
        if (i_ < 0 || i_ >= c_) {                                                                        \
            printf("MJRL_SLAB_CHECK %s:%d wg %d thread %d: slab index %lld outside [0, %lld)\n", __FILE__, \
                   __LINE__, (int)blockIdx.x, (int)threadIdx.x, (long long)i_, (long long)c_);            \
            __builtin_trap();                                                                            \
        }                                                                                                \
    } while (0)
#else
#define MJRL_SLAB_CHECK(idx, cap) ((void)0)
#endif

// ---------------------------------------------------------------------------
// Grid-wide fixed-order fold without a grid barrier: every workgroup stores its
// (already block-reduced) partial, and the LAST workgroup to take a ticket folds
// all nwg partials in index order (lane l: partials l, l + 64, ... then a fixed
// shuffle tree) — the same order on every run, whatever the scheduling.  Called
// by the 64 lanes of ONE wave per workgroup with the same value b in every lane.
// Returns true in the last workgroup (total valid in every lane of that wave);
// the ticket is reset there for the next launch.  Visibility: release fence
// before the ticket, acquire fence after it (MI355X_MICROARCH.md, inter-workgroup
// visibility).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool last_wg_fold(double b, double* parts, unsigned* ticket, int nwg, double& total) {
    const int lane = threadIdx.x & 63;
    unsigned tk = 0;
    if (lane == 0) {
        parts[blockIdx.x] = b;
        __threadfence();
        tk = atomicAdd(ticket, 1u);
    }
    tk = __shfl(tk, 0, 64);
    if (tk != (unsigned)(nwg - 1)) return false;
    __threadfence();
    double t = 0.0;
    for (int i = lane; i < nwg; i += 64) t += __hip_atomic_load(parts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    total = wave_sum(t);
    if (lane == 0) *ticket = 0u;
    return true;
}

// The z step of a CG iteration (cg_solve.py:11, npg_cg.py:73-74) fused into the
// epilogue of a gradient gather: z[f] = gsum[f] / T + damping p[f] on the mean
// block, c(sigma) p[f] + damping p[f] on the log-std block (closed form, DESIGN.md
// §2), and the partial of p.z.  p == nullptr: off.
struct CgZ {
    const float* p;
    float* z;
    float* cg;            // CG state (mjrl_cg_*): cg[8] ticket, cg + 16 double partials
    const float* ls;      // packed log_std
    double inv_T;
    float damping;
    int ls0;              // first log-std flat index (d - m)
};

__device__ __forceinline__ float cg_logstd_curv(float log_std) {
    const float sg = expf(log_std);
    const double uu = (double)sg * (double)sg;
    return (float)(4.0 * uu * (2.0 * uu - 1e-8) / ((2.0 * uu + 1e-8) * (2.0 * uu + 1e-8)));
}

// wave 0 of a gather workgroup: lane -> flat parameter f (< d), gs = the folded
// (f32-rounded) gradient sum of f.  Writes z and this workgroup's partial of p.z
// (cg[CG_PZ_PARTS + 2 blockIdx.x], a double); mjrl_cg_step_xr_p folds them.
constexpr int CG_PZ_PARTS = 1024;   // float offset of the fused gather's p.z partials in the CG state
// (pf, lsv: p[f] and, on the log-std block, log_std[f - ls0], loaded by the caller)
__device__ __forceinline__ void cgz_epilogue(const CgZ& c, int f, int d, float gs, float pf, float lsv,
                                             int slot = -1) {
    double pz = 0.0;
    if (f < d) {
        float hv;
        if (f >= c.ls0) {
            const float sg = expf(lsv);
            const double uu = (double)sg * (double)sg;
            const double cc = 4.0 * uu * (2.0 * uu - 1e-8) / ((2.0 * uu + 1e-8) * (2.0 * uu + 1e-8));
            hv = (float)(cc * (double)pf);
        } else {
            hv = (float)((double)gs * c.inv_T);
        }
        const float zf = __fadd_rn(hv, __fmul_rn(c.damping, pf));   // hvp_flat + regu_coef * vector
        c.z[f] = zf;
        pz = (double)pf * (double)zf;
    }
    pz = wave_sum(pz);
    if ((threadIdx.x & 63) == 0) reinterpret_cast<double*>(c.cg + CG_PZ_PARTS)[slot < 0 ? (int)blockIdx.x : slot] = pz;
}
__device__ __forceinline__ void cgz_load(const CgZ& c, int f, int d, float& pf, float& lsv) {
    pf = f < d ? c.p[f] : 0.f;
    lsv = f < d && f >= c.ls0 ? c.ls[f - c.ls0] : 0.f;
}
__device__ __forceinline__ void cgz_epilogue(const CgZ& c, int f, int d, float gs, int slot = -1) {
    float pf, lsv;
    cgz_load(c, f, d, pf, lsv);
    cgz_epilogue(c, f, d, gs, pf, lsv, slot);
}

// Offsets (in floats) of the packed parameter set — see pack_params.
struct Packed {
    int W0, W1, b1, W2, b2, W1T, W2T, ls, total;
    __host__ __device__ Packed(int h0, int h1, int np, int mp) {
        int o = 0;
        if (h0 == 0) {                 // linear: Wp [MP][NP] only
            W0 = o; o += mp * np;
            W1 = b1 = W2 = b2 = W1T = W2T = o;
        } else {
            W0 = o;  o += h0 * np;
            W1 = o;  o += h1 * h0;
            b1 = o;  o += h1;
            W2 = o;  o += mp * h1;
            b2 = o;  o += mp;
            W1T = o; o += h0 * h1;
            W2T = o; o += h1 * mp;
        }
        ls = o; o += mp;
        total = round_up(o, 4);
    }
};

// Packed positions of flat parameters (reference order W0, b0, W1, b1, W2, b2,
// log_std; gaussian_mlp.py:61-64) in the padded / transposed packed set above.
struct PackMap {
    int n, m, h0, h1, np, mp;
    Packed pk;
    __host__ __device__ PackMap(const mjrl_shape& s)
        : n(s.n), m(s.m), h0(s.h0), h1(s.h1), np(s.np), mp(s.mp), pk(s.h0, s.h1, s.np, s.mp) {}

    // Packed positions of flat parameter f (second = transpose copy or -1);
    // returns the log_std index j when f is a log-std entry, else -1.
    __device__ int map(int f, int& p1, int& p2) const {
        p2 = -1;
        int g = f;
        if (h0 == 0) {
            if (g < m * n) { p1 = pk.W0 + (g / n) * np + g % n; return -1; }
            if ((g -= m * n) < m) { p1 = pk.W0 + g * np + n; return -1; }
            g -= m;
            p1 = pk.ls + g;
            return g;
        }
        if (g < h0 * n) { p1 = pk.W0 + (g / n) * np + g % n; return -1; }
        if ((g -= h0 * n) < h0) { p1 = pk.W0 + g * np + n; return -1; }
        if ((g -= h0) < h1 * h0) {
            const int j = g / h0, k = g % h0;
            p1 = pk.W1 + g;
            p2 = pk.W1T + k * h1 + j;
            return -1;
        }
        if ((g -= h1 * h0) < h1) { p1 = pk.b1 + g; return -1; }
        if ((g -= h1) < m * h1) {
            const int j = g / h1, k = g % h1;
            p1 = pk.W2 + j * h1 + k;
            p2 = pk.W2T + k * mp + j;
            return -1;
        }
        if ((g -= m * h1) < m) { p1 = pk.b2 + g; return -1; }
        g -= m;
        p1 = pk.ls + g;
        return g;
    }
};

__device__ __forceinline__ void pack_one(const PackMap& pm, int f, float v, float* packed, bool clamp, float min_ls) {
    int p1, p2;
    const int j = pm.map(f, p1, p2);
    if (j >= 0 && clamp) v = v < min_ls ? min_ls : v;   // torch.clamp(log_std, min) (gaussian_mlp.py:74-78)
    packed[p1] = v;
    if (p2 >= 0) packed[p2] = v;
}

}  // namespace mjrl
