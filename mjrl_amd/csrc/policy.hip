// policy.hip — Gaussian-MLP / linear policy passes over the timestep batch.
//
// Three launches per pass:
//   k_rows<H0,H1,MP,MODE>  persistent, one 64-row (32 for 256-wide layers) tile of
//                          timesteps at a time; the whole per-row chain runs out of
//                          LDS on v_mfma_f32_16x16x4_f32:
//                            FWD  forward + LL + VPG upstream + backprop to every layer
//                            FVP  JVP of the tangent + Gauss-Newton weight + backprop
//                            EVAL forward at new params + likelihood ratio + KL
//   k_wgrad                split-K over timesteps: weight gradients G^T A per layer
//                          (bias gradients ride along: the obs bias column / column sums)
//   k_gather               fixed-order sum of the slabs into the flat d-vector
//
// Reference math: mjrl/policies/gaussian_mlp.py:100-182, gaussian_linear.py:98-175,
// mjrl/algos/batch_reinforce.py:37-55, mjrl/algos/npg_cg.py:55-74.
#include <math.h>
#include <stdlib.h>

#include "common.h"

using namespace mjrl;

namespace {

enum { FWD = 0, FVP = 1, EVAL = 2 };

struct RowArgs {
    int64_t T;            // rows processed by this call
    int np, m;
    const float* xhat;
    const float* act;
    const float* adv;     // EVAL: surrogate advantages
    const float* adv_vpg; // FWD: advantages driving the gradient
    float* a0;
    float* a1;
    float* mu0;
    float* ll0;
    float* gu0;
    float* gu1;
    float* gp;
    const float* P;       // packed theta (new)
    const float* V;       // FVP: packed tangent;  EVAL: packed old theta (log_std)
    const float* out_shift;
    const float* out_scale;
    double* rpart;        // per-workgroup partials
    const int32_t* done;
    float llc;            // -0.5 * m * log(2 pi) rounded to f32
    const void* xs;       // split-f16 xhat rows [T][hi NP | lo NP] (k_kx), or null
    const float* xu;      // [T] power-of-two row scales of xs
    const float* xc;      // [NP] power-of-two column scales of xs
    // FWD with the batch assembly fused in (k_kx<.., FWD, true>): the staged f32
    // observations [T][n_obs] (identity input normalisation), converted to the split
    // rows in the tile publish, which also writes them to xs_w / xu_w
    const float* obs32;
    _Float16* xs_w;
    float* xu_w;
    int n_obs;
};

// rows per k_rows tile for a hidden width.  128-wide layers: 32 rows keep the f32
// activation buffers (4 x BT x (H + 4) floats) at 70 KB, two workgroups per CU —
// the HalfCheetah FVP 388 -> 298 us against 64 rows and one workgroup; 256-wide
// layers: 32 rows (16 rows, two workgroups per CU, measured 1 % slower)
__host__ __device__ constexpr int rows_bt(int hmax) { return hmax >= 128 ? 32 : 64; }
// threads per k_rows workgroup.  256-wide layers: one 138 KB workgroup per CU of
// 16 waves (four per SIMD, 128 VGPRs each); 128-wide: two 70 KB workgroups of 8
// waves.  Measured against 4 waves: door DAPG FVP 415 -> 369 us (8 waves) -> 353
// us (16); HalfCheetah TRPO FVP 298 -> 251 us (8).  The phase-1 staging and the
// row pass leave threads beyond the tile's elements idle.
__host__ __device__ constexpr int rows_nt(int hmax) { return hmax >= 256 ? 1024 : (hmax >= 128 ? 512 : NTHREADS); }

template <int H0, int H1, int MP>
struct Layout {
    static constexpr bool LIN = (H0 == 0);
    static constexpr int HMAX = H0 > H1 ? H0 : H1;
    static constexpr int BT = rows_bt(HMAX);
    static constexpr int RB = BT / 16;
    static constexpr int LD0 = LIN ? 0 : H0 + 4;
    static constexpr int LD1 = LIN ? 0 : H1 + 4;
    static constexpr int LDP = MP + 4;
    static constexpr int KC = 64;
    static constexpr int LDX = KC + 4;
    static constexpr int oD0 = 0;
    static constexpr int oA0 = oD0 + BT * LD0;
    static constexpr int oD1 = oA0 + BT * LD0;
    static constexpr int oA1 = oD1 + BT * LD1;
    static constexpr int oGP = oA1 + BT * LD1;
    static constexpr int XS = 2 * BT * LDX;
    static constexpr bool XS_ALIAS = !LIN && 2 * BT * LD1 >= XS;
    static constexpr int oXS = XS_ALIAS ? oD1 : oGP + BT * LDP;
    static constexpr int end1 = XS_ALIAS ? oGP + BT * LDP : oXS + XS;
    static constexpr int NT = rows_nt(HMAX);
    static constexpr int total = end1 > 2 * NT ? end1 : 2 * NT;   // >= row_pass_final's doubles
    static constexpr int bytes = total * 4;
};

__device__ __forceinline__ float tanh_f(float x) { return tanhf(x); }

// sum_j log_std_j in action order (the -sum(log_std) term of log_likelihood)
__device__ __forceinline__ float ls_sum(const float* __restrict__ P_ls, int m) {
    // sum(log_std) front to back; the loads of a 16-chunk are issued together
    // (adding the zero padding is exact)
    float s = 0.f;
    for (int j0 = 0; j0 < m; j0 += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = j0 + u < m ? P_ls[j0 + u] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
    }
    return s;
}

// Per-row pass of FWD / EVAL over a tile of BT rows whose output-layer values
// sit in GPs[BT][ldp] (gaussian_mlp.py:100-140 log_likelihood, mean_LL,
// likelihood_ratio, kl_old_new; batch_reinforce.py:37-55).
// Element-parallel over (row, action): thread tid owns action j = tid % MP of
// rows (tid + u NT) / MP, so the MP lanes of a row sit in one wave and the sums
// over actions are a fixed shuffle tree inside the row's lanes (no barrier).
//   FWD : mu0 <- mean; GPs <- adv z / sigma * out_scale (zero for j >= m and rows
//         past T); ll0 <- log-likelihood; acc0 += adv (z^2 - 1) (log-std VPG, action j).
//   EVAL: acc0 += exp(LL_new - LL_old) adv, acc1 += KL(old || new) (lanes j = 0).
// The per-thread partials are folded once per launch by row_pass_final.
// The per-row inputs of row_pass (actions, old means, old log-likelihoods,
// advantages) for this thread's elements, loaded ahead of the pass by a caller
// with registers to spare (the EVAL pass of k_kx loads them at the top of the
// tile, so the row pass no longer waits on them).
template <int BT, int MP, int NT>
struct RowPre {
    static constexpr int NE = BT * MP;
    static constexpr int PER = NE >= NT ? NE / NT : 1;
    float av[PER], mo[PER], l0[PER], ad[PER];
};

template <int MODE, int BT, int MP, int NT>
__device__ __forceinline__ void row_pre_load(const RowArgs& a, int64_t row_base, int tid, RowPre<BT, MP, NT>& pre) {
    using R = RowPre<BT, MP, NT>;
    const int m = a.m;
    const int64_t T = a.T;
    const int j = tid % MP;
    // unconditional loads from clamped indices, no selects: row_pass reads an element
    // only where it is valid (gr < T, j < m; j == 0 for the per-row values), and a
    // load under a branch would make every later vmcnt wait conservative (it waited
    // for the next tile's xhat loads)
    const int jc = j < m ? j : 0;
#pragma unroll
    for (int u = 0; u < R::PER; ++u) {
        const bool in = R::NE >= NT || tid + u * NT < R::NE;
        const int row = in ? (tid + u * NT) / MP : 0;
        const int64_t gr = in ? row_base + row : T;
        const int64_t gc = gr < T ? gr : T - 1;
        pre.av[u] = a.act[gc * m + jc];
        pre.mo[u] = MODE == EVAL ? a.mu0[gc * m + jc] : 0.f;
        pre.l0[u] = MODE == EVAL ? a.ll0[gc] : 0.f;
        pre.ad[u] = MODE == FWD ? a.adv_vpg[gc] : a.adv[gc];
    }
}

// The row pass's per-launch constants of this thread's action j (log-stds, out_scale),
// loaded once before the tile loop by callers that keep them in registers: a
// per-tile load would make the row pass wait (in-order vmcnt) on every global load
// issued before it, the next tile's xhat prefetch included.
struct RowConst {
    float lsn, sn, os, lso, so;
};

template <int MODE, int MP>
__device__ __forceinline__ RowConst row_const(const RowArgs& a, const float* __restrict__ P_ls, int tid) {
    const int j = tid % MP;
    const bool act_j = j < a.m;
    RowConst c;
    c.lsn = act_j ? P_ls[j] : 0.f;
    c.sn = expf(c.lsn);
    c.os = 1.f;
    c.lso = 0.f;
    c.so = 1.f;
    if (MODE == FWD) {
        if (a.out_scale && act_j) c.os = a.out_scale[j];
    } else {
        c.lso = act_j ? a.V[(P_ls - a.P) + j] : 0.f;
        c.so = expf(c.lso);
    }
    return c;
}

template <int MODE, int BT, int MP, int NT, bool STORE_GP, bool PRE = false>
__device__ __forceinline__ void row_pass(const RowArgs& a, const float* __restrict__ P_ls, float sls,
                                         int64_t row_base, float* GPs, int ldp, double& acc0, double& acc1,
                                         int tid, const RowPre<BT, MP, NT>* pre = nullptr,
                                         const RowConst* rc = nullptr) {
    constexpr int NE = BT * MP;                        // (row, action) elements of the tile
    constexpr int PER = NE >= NT ? NE / NT : 1;        // more threads than elements: the rest idle
    static_assert(NT % MP == 0 && (NE >= NT ? PER * NT == NE : NT % NE == 0) && MP <= 64, "row lanes in one wave");
    const int m = a.m;
    const int64_t T = a.T;
    const int j = tid % MP;
    const bool act_j = j < m;
    const RowConst c = rc ? *rc : row_const<MODE, MP>(a, P_ls, tid);
    const float lsn = c.lsn, sn = c.sn, os = c.os, lso = c.lso, so = c.so;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const bool in = NE >= NT || tid + u * NT < NE;
        const int row = in ? (tid + u * NT) / MP : 0;
        const int64_t gr = in ? row_base + row : T;        // an idle thread acts as a row past T
        const bool valid = gr < T && act_j;
        float* g = GPs + row * ldp + j;
        const float mu = in ? *g : 0.f;
        const float av = PRE ? pre->av[u] : (valid ? a.act[gr * m + j] : 0.f);
        float mo = 0.f, adv = 0.f;
        if (MODE == EVAL) mo = PRE ? pre->mo[u] : (valid ? a.mu0[gr * m + j] : 0.f);
        if (MODE == FWD) adv = PRE ? pre->ad[u] : (gr < T ? a.adv_vpg[gr] : 0.f);
        const float zs = valid ? (av - mu) / sn : 0.f;
        float z2 = zs * zs;
        float kl = 0.f;
        if (MODE == FWD) {
            if (valid) {
                a.mu0[gr * m + j] = mu;
                acc0 += (double)(adv * (z2 - 1.f));
            }
            const float gv = valid ? adv * (zs / sn) * os : 0.f;
            if (in) *g = gv;
            if (STORE_GP && gr < T) a.gp[gr * MP + j] = gv;
        } else if (valid) {
            const float dm = mo - mu;
            const float nr = (dm * dm + so * so) - sn * sn;
            const float dr = 2.f * sn * sn + 1e-8f;
            kl = (nr / dr + lsn) - lso;
        }
#pragma unroll
        for (int o = MP / 2; o > 0; o >>= 1) {
            z2 += __shfl_xor(z2, o, 64);
            if (MODE == EVAL) kl += __shfl_xor(kl, o, 64);
        }
        if (j == 0 && gr < T) {
            const float ll = ((-0.5f * z2) + (-sls)) + a.llc;
            if (MODE == FWD) {
                a.ll0[gr] = ll;
            } else {
                const float lr = expf(ll - (PRE ? pre->l0[u] : a.ll0[gr]));
                acc0 += (double)(lr * (PRE ? pre->ad[u] : a.adv[gr]));
                acc1 += (double)kl;
            }
        }
    }
}

// Fold the launch's row-pass partials (fixed order): FWD -> rpart[blk][MP]
// (log-std VPG sums), EVAL -> rpart[blk][2] (surrogate and KL sums).
// red: LDS scratch of NT doubles; the caller has synchronised the block.
template <int MODE, int MP, int NT>
__device__ __forceinline__ void row_pass_final(double acc0, double acc1, double* red, double* __restrict__ rpart,
                                               int64_t blk, int tid) {
    if (MODE == FWD) {
        red[tid] = acc0;
        __syncthreads();
        if (tid < MP) {
            double s = 0.0;
            for (int k = 0; k < NT / MP; ++k) s += red[k * MP + tid];
            rpart[blk * MP + tid] = s;
        }
    } else {
        if (tid % MP == 0) {
            red[tid / MP] = acc0;
            red[NT / MP + tid / MP] = acc1;
        }
        __syncthreads();
        if (tid == 0) {
            double s = 0.0, k = 0.0;
            for (int i = 0; i < NT / MP; ++i) {
                s += red[i];
                k += red[NT / MP + i];
            }
            rpart[blk * 2 + 0] = s;
            rpart[blk * 2 + 1] = k;
        }
    }
}

template <int H0, int H1, int MP, int MODE>
__global__ void __launch_bounds__((Layout<H0, H1, MP>::NT), (Layout<H0, H1, MP>::bytes > 81920 ? 1 : 2))
    k_rows(RowArgs a) {
    using L = Layout<H0, H1, MP>;
    constexpr int BT = L::BT, RB = L::RB, NT = L::NT, NW = NT / 64;
    constexpr int N1 = L::LIN ? MP : H0;
    using S1 = Split<RB, N1 / 16, NW>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* D0 = smem + L::oD0;
    float* A0s = smem + L::oA0;
    float* D1 = smem + L::oD1;
    float* A1s = smem + L::oA1;
    float* GPs = smem + L::oGP;
    float* XS = smem + L::oXS;

    // FVP: a converged CG loop (cg_solve.py:19-20); EVAL: a TRPO trial the device line
    // search no longer needs (mjrl_policy_eval_if)
    if ((MODE == FVP || MODE == EVAL) && a.done && *a.done) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, q = lane >> 4;
    const int np = a.np, m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;

    const float* P = a.P;
    const Packed pk(H0, H1, np, MP);
    // per-lane output-column constants for the output layer
    // FWD / EVAL row-pass partials (row_pass), folded at the end of the launch
    double racc0 = 0.0, racc1 = 0.0;
    const float sls = MODE == FVP ? 0.f : ls_sum(P + pk.ls, m);

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row_base = tile * BT;

        // ---------------- phase 1: [BT x N1] = xhat[BT x np] * W^T, K = np ----------------
        floatx4 acc1[S1::NRW][S1::NCW];
        zero_acc(acc1);
        {
            const float* W = (MODE == FVP ? a.V : P) + pk.W0;
            constexpr int NQ = BT * (L::KC / 4);              // float4 pieces of a staged chunk
            constexpr int PER = NQ >= NT ? NQ / NT : 1;
            static_assert(NQ < NT ? NT % NQ == 0 : PER * NT == NQ, "phase-1 staging");
            float4 st[PER];
            const int nch = (np + L::KC - 1) / L::KC;
            auto gload = [&](int c) {
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const int idx = tid + u * NT;
                    const int row = idx / (L::KC / 4), c4 = idx % (L::KC / 4);
                    const int col = c * L::KC + c4 * 4;
                    const int64_t gr = row_base + row;
                    st[u] = (idx < NQ && gr < T && col < np) ? *reinterpret_cast<const float4*>(a.xhat + gr * np + col)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            };
            gload(0);
            for (int c = 0; c < nch; ++c) {
                float* xs = XS + (c & 1) * BT * L::LDX;
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const int idx = tid + u * NT;
                    const int row = idx / (L::KC / 4), c4 = idx % (L::KC / 4);
                    if (idx < NQ) *reinterpret_cast<float4*>(xs + row * L::LDX + c4 * 4) = st[u];
                }
                __syncthreads();
                if (c + 1 < nch) gload(c + 1);
                const int kb = c * L::KC;
                const int ke = kb + L::KC < np ? kb + L::KC : np;
                gemm_tile(acc1, xs, L::LDX, kb, S1::rb0(w), S1::RBS, RB, W, np, S1::cb0(w), S1::CBS, kb, ke, lane);
            }
            __syncthreads();
        }

        if constexpr (L::LIN) {
            // ---------------- linear policy: phase 1 is the output layer -----------
#pragma unroll
            for (int i = 0; i < S1::NRW; ++i) {
                const int rb = S1::rb0(w) + i * S1::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S1::NCW; ++j) {
                    const int col = (S1::cb0(w) + j * S1::CBS) * 16 + r16;
                    const float ls = P[pk.ls + col];
                    const float os = a.out_scale ? (col < m ? a.out_scale[col] : 1.f) : 1.f;
                    const float osh = a.out_shift ? (col < m ? a.out_shift[col] : 0.f) : 0.f;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * q + rr;
                        const float v = acc1[i][j][rr];
                        if (MODE == FVP) {
                            const float sg = expf(ls);
                            const float wq = os * os * (2.f / (2.f * sg * sg + 1e-8f));
                            const float g = col < m ? wq * v : 0.f;
                            const int64_t gr = row_base + row;
                            if (gr < T) a.gp[gr * MP + col] = g;
                        } else {
                            GPs[row * L::LDP + col] = col < m ? v * os + osh : 0.f;
                        }
                    }
                }
            }
        } else {
            // ---------------- epilogue 1 ----------------
#pragma unroll
            for (int i = 0; i < S1::NRW; ++i) {
                const int rb = S1::rb0(w) + i * S1::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S1::NCW; ++j) {
                    const int col = (S1::cb0(w) + j * S1::CBS) * 16 + r16;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * q + rr;
                        const int64_t gr = row_base + row;
                        const float v = acc1[i][j][rr];
                        if (MODE == FVP) {
                            const float av = gr < T ? a.a0[gr * H0 + col] : 0.f;
                            D0[row * L::LD0 + col] = (1.f - av * av) * v;
                            A0s[row * L::LD0 + col] = av;
                        } else {
                            const float av = tanh_f(v);
                            A0s[row * L::LD0 + col] = av;
                            if (MODE == FWD && gr < T) a.a0[gr * H0 + col] = av;
                        }
                    }
                }
            }
            __syncthreads();

            // ---------------- phase 2: [BT x H1], K = H0 ----------------
            using S2 = Split<RB, H1 / 16, NW>;
            floatx4 acc2[S2::NRW][S2::NCW];
            zero_acc(acc2);
            if (MODE == FVP) {
                gemm_tile(acc2, D0, L::LD0, 0, S2::rb0(w), S2::RBS, RB, P + pk.W1, H0, S2::cb0(w), S2::CBS, 0, H0,
                          lane);
                gemm_tile(acc2, A0s, L::LD0, 0, S2::rb0(w), S2::RBS, RB, a.V + pk.W1, H0, S2::cb0(w), S2::CBS, 0,
                          H0, lane);
            } else {
                gemm_tile(acc2, A0s, L::LD0, 0, S2::rb0(w), S2::RBS, RB, P + pk.W1, H0, S2::cb0(w), S2::CBS, 0, H0,
                          lane);
            }
            // epilogue 2
#pragma unroll
            for (int i = 0; i < S2::NRW; ++i) {
                const int rb = S2::rb0(w) + i * S2::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S2::NCW; ++j) {
                    const int col = (S2::cb0(w) + j * S2::CBS) * 16 + r16;
                    const float bias = (MODE == FVP ? a.V : P)[pk.b1 + col];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * q + rr;
                        const int64_t gr = row_base + row;
                        const float v = acc2[i][j][rr] + bias;
                        if (MODE == FVP) {
                            const float av = gr < T ? a.a1[gr * H1 + col] : 0.f;
                            D1[row * L::LD1 + col] = (1.f - av * av) * v;
                            A1s[row * L::LD1 + col] = av;
                        } else {
                            const float av = tanh_f(v);
                            A1s[row * L::LD1 + col] = av;
                            if (MODE == FWD && gr < T) a.a1[gr * H1 + col] = av;
                        }
                    }
                }
            }
            __syncthreads();

            // ---------------- phase 3: [BT x MP], K = H1 ----------------
            using S3 = Split<RB, MP / 16, NW>;
            floatx4 acc3[S3::NRW][S3::NCW];
            zero_acc(acc3);
            if (MODE == FVP) {
                gemm_tile(acc3, D1, L::LD1, 0, S3::rb0(w), S3::RBS, RB, P + pk.W2, H1, S3::cb0(w), S3::CBS, 0, H1,
                          lane);
                gemm_tile(acc3, A1s, L::LD1, 0, S3::rb0(w), S3::RBS, RB, a.V + pk.W2, H1, S3::cb0(w), S3::CBS, 0,
                          H1, lane);
            } else {
                gemm_tile(acc3, A1s, L::LD1, 0, S3::rb0(w), S3::RBS, RB, P + pk.W2, H1, S3::cb0(w), S3::CBS, 0, H1,
                          lane);
            }
#pragma unroll
            for (int i = 0; i < S3::NRW; ++i) {
                const int rb = S3::rb0(w) + i * S3::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S3::NCW; ++j) {
                    const int col = (S3::cb0(w) + j * S3::CBS) * 16 + r16;
                    const float bias = (MODE == FVP ? a.V : P)[pk.b2 + col];
                    const float os = a.out_scale ? (col < m ? a.out_scale[col] : 1.f) : 1.f;
                    const float osh = a.out_shift ? (col < m ? a.out_shift[col] : 0.f) : 0.f;
                    float wq = 0.f;
                    if (MODE == FVP) {
                        const float sg = expf(P[pk.ls + col]);
                        wq = os * os * (2.f / (2.f * sg * sg + 1e-8f));
                    }
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * q + rr;
                        const float v = acc3[i][j][rr] + bias;
                        if (MODE == FVP) {
                            const float g = col < m ? wq * v : 0.f;
                            GPs[row * L::LDP + col] = g;
                            const int64_t gr = row_base + row;
                            if (gr < T) a.gp[gr * MP + col] = g;
                        } else {
                            GPs[row * L::LDP + col] = col < m ? v * os + osh : 0.f;
                        }
                    }
                }
            }
        }
        __syncthreads();

        // ---------------- per-row pass: log-likelihood, VPG upstream, LR, KL -------------
        if (MODE != FVP) {
            row_pass<MODE, BT, MP, NT, true>(a, P + pk.ls, sls, row_base, GPs, L::LDP, racc0, racc1, tid);
            __syncthreads();
        }

        if constexpr (!L::LIN) {
            if (MODE != EVAL) {
                // ---------------- phase 4: ga1 = g * W2, K = MP ----------------
                using S2 = Split<RB, H1 / 16, NW>;
                floatx4 acc4[S2::NRW][S2::NCW];
                zero_acc(acc4);
                gemm_tile(acc4, GPs, L::LDP, 0, S2::rb0(w), S2::RBS, RB, P + pk.W2T, MP, S2::cb0(w), S2::CBS, 0, MP,
                          lane);
#pragma unroll
                for (int i = 0; i < S2::NRW; ++i) {
                    const int rb = S2::rb0(w) + i * S2::RBS;
                    if (rb >= RB) continue;
#pragma unroll
                    for (int j = 0; j < S2::NCW; ++j) {
                        const int col = (S2::cb0(w) + j * S2::CBS) * 16 + r16;
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int row = rb * 16 + 4 * q + rr;
                            const float av = A1s[row * L::LD1 + col];
                            const float g = (1.f - av * av) * acc4[i][j][rr];
                            D1[row * L::LD1 + col] = g;
                            const int64_t gr = row_base + row;
                            if (gr < T) a.gu1[gr * H1 + col] = g;
                        }
                    }
                }
                __syncthreads();
                // ---------------- phase 5: ga0 = gu1 * W1, K = H1 ----------------
                floatx4 acc5[S1::NRW][S1::NCW];
                zero_acc(acc5);
                gemm_tile(acc5, D1, L::LD1, 0, S1::rb0(w), S1::RBS, RB, P + pk.W1T, H1, S1::cb0(w), S1::CBS, 0, H1,
                          lane);
#pragma unroll
                for (int i = 0; i < S1::NRW; ++i) {
                    const int rb = S1::rb0(w) + i * S1::RBS;
                    if (rb >= RB) continue;
#pragma unroll
                    for (int j = 0; j < S1::NCW; ++j) {
                        const int col = (S1::cb0(w) + j * S1::CBS) * 16 + r16;
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int row = rb * 16 + 4 * q + rr;
                            const float av = A0s[row * L::LD0 + col];
                            const int64_t gr = row_base + row;
                            if (gr < T) a.gu0[gr * H0 + col] = (1.f - av * av) * acc5[i][j][rr];
                        }
                    }
                }
                __syncthreads();
            }
        }
    }

    if (MODE != FVP) {
        static_assert(L::total >= 2 * NT, "row_pass_final scratch");
        __syncthreads();
        row_pass_final<MODE, MP, NT>(racc0, racc1, reinterpret_cast<double*>(smem), a.rpart, blockIdx.x, tid);
    }
}

// ---------------------------------------------------------------------------
// Weight gradients: C[N][K] = sum_t G[t][n] * A[t][k], split over T into S slices.
// ---------------------------------------------------------------------------
struct WJob {
    const float* G;
    const float* A;
    int ldg, lda, N, K;
    int nbN, nbK, bias;
    int64_t off;    // float offset of slice 0's [N][K] slab in wpart
    int64_t boff;   // float offset of slice 0's [N] bias slab
};

struct WArgs {
    WJob job[3];
    int njobs;
    int start[4];   // prefix sums of blocks per slice per job
    int S;
    int64_t T;
    int64_t rows_per_slice;
    float* wpart;
    const int32_t* done;
    int64_t wcap;   // floats of the scratch's slabs (MJRL_SLAB_CHECK)
};

constexpr int WB = 64;        // output block edge
constexpr int WT = 64;        // rows per staged tile
constexpr int WLD = WB + 16;  // LDS row stride (floats): rows 4 apart land 16 banks apart

// (A split-f16 version — transposed LDS tiles, per-(32-row step, column) scales —
// measured slower: HalfCheetah 87 -> 126 us, door 94 -> 134 us per launch, from
// the transposing LDS writes and the per-step splits; profiles/r03g/rejected/.)
__global__ void __launch_bounds__(NTHREADS, 2) k_wgrad(WArgs a) {
    if (a.done && *a.done) return;
    __shared__ __attribute__((aligned(16))) float Gs[WT * WLD];
    __shared__ __attribute__((aligned(16))) float As[WT * WLD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, q = lane >> 4;
    const int jb = blockIdx.x / a.S, s = blockIdx.x % a.S;
    int ji = 0;
    while (ji + 1 < a.njobs && jb >= a.start[ji + 1]) ++ji;
    const WJob& J = a.job[ji];
    const int local = jb - a.start[ji];
    const int nb = local / J.nbK, kb = local % J.nbK;
    const int n0 = nb * WB, k0 = kb * WB;
    const int64_t r0 = (int64_t)s * a.rows_per_slice;
    int64_t r1 = r0 + a.rows_per_slice;
    if (r1 > a.T) r1 = a.T;

    floatx4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = zero4();
    double bsum = 0.0;
    const bool do_bias = J.bias && kb == 0;

    // staging: 64 rows x 64 cols of G and of A = 1024 float4 each, 4 per thread
    float4 g4[4], a4[4];
    auto gload = [&](int64_t t0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = tid + u * NTHREADS;
            const int row = idx >> 4, c4 = (idx & 15) * 4;
            const int64_t t = t0 + row;
            const bool rv = t < r1;
            g4[u] = (rv && n0 + c4 < J.N) ? *reinterpret_cast<const float4*>(J.G + t * J.ldg + n0 + c4)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
            a4[u] = (rv && k0 + c4 < J.K) ? *reinterpret_cast<const float4*>(J.A + t * J.lda + k0 + c4)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    if (r0 < r1) gload(r0);
    for (int64_t t0 = r0; t0 < r1; t0 += WT) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = tid + u * NTHREADS;
            const int row = idx >> 4, c4 = (idx & 15) * 4;
            *reinterpret_cast<float4*>(Gs + row * WLD + c4) = g4[u];
            *reinterpret_cast<float4*>(As + row * WLD + c4) = a4[u];
        }
        __syncthreads();
        if (t0 + WT < r1) gload(t0 + WT);
        if (n0 + 16 * w < J.N) {
#pragma unroll 4
            for (int tt = 0; tt < WT; tt += 4) {
                const float ga = Gs[(tt + q) * WLD + 16 * w + r16];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float ab = As[(tt + q) * WLD + 16 * i + r16];
                    acc[i] = mfma4(ga, ab, acc[i]);
                }
            }
        }
        if (do_bias && tid < WB) {
            double cs = 0.0;
            for (int row = 0; row < WT; ++row) cs += (double)Gs[row * WLD + tid];
            bsum += cs;
        }
    }
    // write this slice's partial block
    float* out = a.wpart + J.off + (int64_t)s * J.N * J.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = k0 + 16 * i + r16;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int n = n0 + 16 * w + 4 * q + rr;
            if (n < J.N && k < J.K) {
                MJRL_SLAB_CHECK(J.off + (int64_t)s * J.N * J.K + (int64_t)n * J.K + k, a.wcap);
                out[(int64_t)n * J.K + k] = acc[i][rr];
            }
        }
    }
    if (do_bias && tid < WB && n0 + tid < J.N) {
        MJRL_SLAB_CHECK(J.boff + (int64_t)s * J.N + n0 + tid, a.wcap);
        a.wpart[J.boff + (int64_t)s * J.N + n0 + tid] = (float)bsum;
    }
}

// ---------------------------------------------------------------------------
// All three weight gradients of one row slice in ONE workgroup (MLP, H0 = H1 = H):
//   gW0[H][NP] += gu0^T xhat,  gW1[H][H] += gu1^T a0 (+ gb1),  gW2[MP][H] += gp^T a1 (+ gb2)
// k_wgrad gives each 64 x 64 output block its own workgroup, so every row tile of
// gu1 / a0 / ... is fetched once per block that reads it (HalfCheetah: 2x the
// bytes it needs, and half the CUs at its 128 slices).  Here a workgroup stages
// each row tile of the six inputs into LDS once (register prefetch of the next
// tile under this tile's MFMAs) and every output block of all three products is
// an accumulator in some wave: wave w owns the 16-row strips w + NW t of gW1 and
// gW0 (a strip's gu fragment feeds all its column blocks) and BW2 blocks of gW2.
// Slabs in the flat chunk-major layout of k_kx (k_gather_flat), fixed order.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int wall_ld(int w) {   // LDS row stride: w <= ld, ld % 64 in {16, 48}
    return (w % 64 == 0) ? w + 16 : (w % 64 <= 16 ? w - w % 64 + 16 : (w % 64 <= 48 ? w - w % 64 + 48 : w - w % 64 + 80));
}

// v where c holds, else zero, component by component (a select of the whole float4
// made the compiler select between two stack addresses and reload through scratch)
__device__ __forceinline__ float4 sel4(bool c, float4 v) {
    return make_float4(c ? v.x : 0.f, c ? v.y : 0.f, c ? v.z : 0.f, c ? v.w : 0.f);
}

template <int H, int MP, int NPBM>
struct WallCfg {
    static constexpr int NW = H / 16 < 8 ? H / 16 : 8;   // waves
    static constexpr int NT = 64 * NW;
    static constexpr int SPW = (H / 16) / NW;            // gW1 / gW0 strips per wave
    static constexpr int BW2 = (MP / 16) * (H / 16) / NW;   // gW2 blocks per wave
    static constexpr int BT = 32;                        // rows per staged tile
    static constexpr int LDH = wall_ld(H), LDP = wall_ld(MP), LDX = wall_ld(16 * NPBM);
    static constexpr int oG0 = 0, oG1 = oG0 + BT * LDH, oGP = oG1 + BT * LDH, oX = oGP + BT * LDP,
                         oA0 = oX + BT * LDX, oA1 = oA0 + BT * LDH, total = oA1 + BT * LDH;
    static constexpr int bytes = total * 4;
};

struct WallArgs {
    const float *gu0, *gu1, *gp, *x, *a0, *a1;
    int n, m, np, S;
    int64_t T, rows_per_slice;
    float* wpart;   // flat slab layout (k_gather_flat)
    const int32_t* done;
    int64_t wcap;   // floats of the scratch's slabs (MJRL_SLAB_CHECK)
};

// PART 0: all three products (the kernel below); 1: gW1 + gb1 only, 2: gW0, gW2 + gb2
// only (the two-workgroups-per-slice split measured for 256-wide layers, not used)
template <int H, int MP, int NPBM, int PART>
__device__ __forceinline__ void wall_body(const WallArgs& a, int s, float* sm) {
    using C = WallCfg<H, MP, NPBM>;
    constexpr int BT = C::BT, NW = C::NW, SPW = C::SPW, BW2 = C::BW2, HB = H / 16;
    constexpr bool J1 = PART != 2, J02 = PART != 1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int np = a.np, npb = np / 16;
    const int64_t r0 = (int64_t)s * a.rows_per_slice;
    const int64_t r1 = r0 + a.rows_per_slice < a.T ? r0 + a.rows_per_slice : a.T;

    // Staging of a tile: every load unconditional (rows past the slice clamped to its
    // last row, masked to zero when stored to LDS; surplus threads of the narrow gp /
    // x pieces re-read a valid piece and store nothing), so no load sits under a
    // branch and none waits for another (in-order vmcnt; a branchy per-piece decode
    // measured 114 vs 87 us for k_wgrad).  H-wide inputs: PH float4 per thread, a
    // compile-time row / column decode.
    constexpr int PH = BT * H / 4 / C::NT;   // float4 per thread of one H-wide input
    static_assert(PH * C::NT == BT * H / 4, "H-wide staging");
    constexpr int QP = BT * MP / 4, PP = (QP + C::NT - 1) / C::NT;                // gp pieces
    constexpr int PX = (BT * 16 * NPBM / 4 + C::NT - 1) / C::NT;               // x pieces (np <= 16 NPBM)
    const int qx = BT * np / 4;
    int prow[PP], pc4[PP], xrow[PX], xc4[PX];
#pragma unroll
    for (int u = 0; u < PP; ++u) {
        const int i = tid + u * C::NT, ic = i < QP ? i : QP - 1;
        prow[u] = ic / (MP / 4);
        pc4[u] = ic % (MP / 4);
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
        const int i = tid + u * C::NT, ic = i < qx ? i : qx - 1;
        xrow[u] = ic / (np / 4);
        xc4[u] = ic % (np / 4);
    }
    struct Stage {
        float4 g0[PH], g1[PH], a0[PH], a1[PH], p[PP], x[PX];
    };
    Stage stA;
    auto hload = [&](float4 (&dst)[PH], const float* src, int64_t t0) __attribute__((always_inline)) {
        const int64_t tl = r1 - 1;
#pragma unroll
        for (int u = 0; u < PH; ++u) {
            const int i = tid + u * C::NT, row = i / (H / 4), c4 = i % (H / 4);
            const int64_t t = t0 + row < tl ? t0 + row : tl;
            dst[u] = *reinterpret_cast<const float4*>(src + t * H + 4 * c4);
        }
    };
    auto hstore = [&](const float4 (&v)[PH], int off, int64_t t0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < PH; ++u) {
            const int i = tid + u * C::NT, row = i / (H / 4), c4 = i % (H / 4);
            *reinterpret_cast<float4*>(sm + off + row * C::LDH + 4 * c4) = sel4(t0 + row < r1, v[u]);
        }
    };
    auto gload = [&](Stage& st, int64_t t0) __attribute__((always_inline)) {
        const int64_t tl = r1 - 1;
        if constexpr (J02) hload(st.g0, a.gu0, t0);
        if constexpr (J1) hload(st.g1, a.gu1, t0);
        if constexpr (J1) hload(st.a0, a.a0, t0);
        if constexpr (J02) hload(st.a1, a.a1, t0);
        if constexpr (J02) {
#pragma unroll
            for (int u = 0; u < PP; ++u) {
                const int64_t tp = t0 + prow[u] < tl ? t0 + prow[u] : tl;
                st.p[u] = *reinterpret_cast<const float4*>(a.gp + tp * MP + 4 * pc4[u]);
            }
#pragma unroll
            for (int u = 0; u < PX; ++u) {
                const int64_t tx = t0 + xrow[u] < tl ? t0 + xrow[u] : tl;
                st.x[u] = *reinterpret_cast<const float4*>(a.x + tx * np + 4 * xc4[u]);
            }
        }
    };
    auto sstore = [&](const Stage& st, int64_t t0) __attribute__((always_inline)) {
        if constexpr (J02) hstore(st.g0, C::oG0, t0);
        if constexpr (J1) hstore(st.g1, C::oG1, t0);
        if constexpr (J1) hstore(st.a0, C::oA0, t0);
        if constexpr (J02) hstore(st.a1, C::oA1, t0);
        if constexpr (J02) {
#pragma unroll
            for (int u = 0; u < PP; ++u)
                if (tid + u * C::NT < QP)
                    *reinterpret_cast<float4*>(sm + C::oGP + prow[u] * C::LDP + 4 * pc4[u]) = sel4(t0 + prow[u] < r1, st.p[u]);
#pragma unroll
            for (int u = 0; u < PX; ++u)
                if (tid + u * C::NT < qx)
                    *reinterpret_cast<float4*>(sm + C::oX + xrow[u] * C::LDX + 4 * xc4[u]) = sel4(t0 + xrow[u] < r1, st.x[u]);
        }
    };

    constexpr int S1 = J1 ? SPW : 0, S0 = J02 ? SPW : 0, B2 = J02 ? BW2 : 0;
    floatx4 acc1[S1 ? S1 : 1][HB], acc0[S0 ? S0 : 1][NPBM], acc2[B2 ? B2 : 1];
#pragma unroll
    for (int t = 0; t < SPW; ++t) {
#pragma unroll
        for (int kb = 0; kb < HB; ++kb) acc1[t < S1 ? t : 0][kb] = zero4();
#pragma unroll
        for (int kb = 0; kb < NPBM; ++kb) acc0[t < S0 ? t : 0][kb] = zero4();
    }
#pragma unroll
    for (int b = 0; b < BW2; ++b) acc2[b < B2 ? b : 0] = zero4();
    double bsum = 0.0;   // thread c < H: gb1[c]; H <= c < H + MP: gb2[c - H]
    const bool bias_thr = (J1 && tid < H) || (J02 && tid >= H && tid < H + MP);

    // One k-step's operands (4 rows): read from LDS one k-step ahead of the MFMAs that
    // use them (the scheduler otherwise waited on each read right before its MFMA).
    struct Ops {
        float av[J1 ? HB : 1], g1[S1 ? S1 : 1], xv[NPBM], g0[S0 ? S0 : 1], gp[B2 ? B2 : 1], a1[B2 ? B2 : 1];
    };
    auto rd = [&](Ops& o, int kk) __attribute__((always_inline)) {
        const int row = 4 * kk + q;
        if constexpr (J1) {
#pragma unroll
            for (int kb = 0; kb < HB; ++kb) o.av[kb] = sm[C::oA0 + row * C::LDH + 16 * kb + r16];
#pragma unroll
            for (int t = 0; t < S1; ++t) o.g1[t] = sm[C::oG1 + row * C::LDH + 16 * (w + NW * t) + r16];
        }
        if constexpr (J02) {
#pragma unroll
            for (int kb = 0; kb < NPBM; ++kb) o.xv[kb] = kb < npb ? sm[C::oX + row * C::LDX + 16 * kb + r16] : 0.f;
#pragma unroll
            for (int t = 0; t < S0; ++t) o.g0[t] = sm[C::oG0 + row * C::LDH + 16 * (w + NW * t) + r16];
#pragma unroll
            for (int b = 0; b < B2; ++b) {
                const int blk = w * BW2 + b, sb = blk / HB, kb = blk % HB;
                o.gp[b] = sm[C::oGP + row * C::LDP + 16 * sb + r16];
                o.a1[b] = sm[C::oA1 + row * C::LDH + 16 * kb + r16];
            }
        }
    };
    auto mm = [&](const Ops& o) __attribute__((always_inline)) {
        if constexpr (J1) {
#pragma unroll
            for (int t = 0; t < S1; ++t)
#pragma unroll
                for (int kb = 0; kb < HB; ++kb) acc1[t][kb] = mfma4(o.g1[t], o.av[kb], acc1[t][kb]);
        }
        if constexpr (J02) {
#pragma unroll
            for (int t = 0; t < S0; ++t)
#pragma unroll
                for (int kb = 0; kb < NPBM; ++kb)
                    if (kb < npb) acc0[t][kb] = mfma4(o.g0[t], o.xv[kb], acc0[t][kb]);
#pragma unroll
            for (int b = 0; b < B2; ++b) acc2[b] = mfma4(o.gp[b], o.a1[b], acc2[b]);
        }
    };
    constexpr bool PIPE = SPW * (HB + NPBM) + BW2 <= 11;   // a second operand set fits the registers
    auto tile = [&]() __attribute__((always_inline)) {
        Ops o0, o1;
        if constexpr (PIPE) {
            rd(o0, 0);
#pragma unroll   // fully: a rolled loop's induction registers took prefetch registers (copies waiting on HBM)
            for (int kk = 0; kk < BT / 4; kk += 2) {
                rd(o1, kk + 1);
                __builtin_amdgcn_sched_barrier(0);
                mm(o0);
                __builtin_amdgcn_sched_barrier(0);
                if (kk + 2 < BT / 4) rd(o0, kk + 2);
                __builtin_amdgcn_sched_barrier(0);
                mm(o1);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BT / 4; ++kk) {
                rd(o0, kk);
                mm(o0);
            }
        }
        if (bias_thr) {   // bias sums: rows in order, fp64 (the LDS reads batched ahead of the adds)
            const float* col = tid < H ? sm + C::oG1 + tid : sm + C::oGP + (tid - H);
            const int ld = tid < H ? C::LDH : C::LDP;
            double cs = 0.0;
#pragma unroll
            for (int rb = 0; rb < BT; rb += 8) {   // eight reads in flight at a time
                float v[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = col[(rb + r) * ld];
#pragma unroll
                for (int r = 0; r < 8; ++r) cs += (double)v[r];
            }
            bsum += cs;
        }
    };
    // one tile of register prefetch under the current tile's MFMAs (a second stage
    // measured no faster: 71.6 vs 71.3 us; its registers hold the next k-step's
    // operands instead)
    if (r0 < r1) gload(stA, r0);
    for (int64_t t0 = r0; t0 < r1; t0 += BT) {
        __syncthreads();
        sstore(stA, t0);
        __syncthreads();
        gload(stA, t0 + BT);   // unconditional (rows clamped): a branch made the compiler copy prefetch registers at the join, waiting on HBM
        tile();
    }
    // this slice's slab in the flat, parameter-chunk-major layout of k_kx:
    // wpart[f / 64][S][64] for flat parameter f (reference order W0, b0, W1, b1, W2, b2,
    // gaussian_mlp.py:61-64), so k_gather_flat folds each 64-parameter chunk from one
    // contiguous run; padded columns / rows are not stored
    const int n = a.n, m = a.m;
    const int fb0 = H * n, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + m * H;
    float* wp = a.wpart + (int64_t)s * 64;
    const int64_t cs = (int64_t)a.S * 64;
    auto put = [&](int f, float v) {
        MJRL_SLAB_CHECK((int64_t)s * 64 + (int64_t)(f >> 6) * cs + (f & 63), a.wcap);
        wp[(int64_t)(f >> 6) * cs + (f & 63)] = v;
    };
    if constexpr (J1) {
#pragma unroll
        for (int t = 0; t < S1; ++t) {
            const int n0 = 16 * (w + NW * t) + 4 * q;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int j = n0 + rr;
                if constexpr (H % 64 == 0) {
                    // fW1 = H (n + 1) is a multiple of 64: row j of gW1 is H / 64 whole chunks,
                    // so column k lands in chunk fW1 / 64 + j H / 64 + k / 64 at k % 64 (one
                    // address per row, immediate offsets for the 16-column steps)
                    float* rowp = wp + (int64_t)((fW1 >> 6) + j * (H / 64)) * cs + r16;
#pragma unroll
                    for (int kb = 0; kb < HB; ++kb) {
                        MJRL_SLAB_CHECK((rowp - a.wpart) + (kb >> 2) * cs + 16 * (kb & 3), a.wcap);
                        rowp[(kb >> 2) * cs + 16 * (kb & 3)] = acc1[t][kb][rr];
                    }
                } else {
#pragma unroll
                    for (int kb = 0; kb < HB; ++kb) put(fW1 + j * H + 16 * kb + r16, acc1[t][kb][rr]);
                }
            }
        }
        if (tid < H) put(fb1 + tid, (float)bsum);
    }
    if constexpr (J02) {
#pragma unroll
        for (int t = 0; t < S0; ++t) {
            const int n0 = 16 * (w + NW * t) + 4 * q;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                for (int kb = 0; kb < NPBM; ++kb) {
                    const int k = 16 * kb + r16, h = n0 + rr;
                    if (k < n) put(h * n + k, acc0[t][kb][rr]);
                    else if (k == n) put(fb0 + h, acc0[t][kb][rr]);   // the bias column: b0
                }
        }
#pragma unroll
        for (int b = 0; b < B2; ++b) {
            const int blk = w * BW2 + b, sb = blk / HB, kb = blk % HB;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int j = 16 * sb + 4 * q + rr;
                if (j < m) put(fW2 + j * H + 16 * kb + r16, acc2[b][rr]);
            }
        }
        if (tid >= H && tid < H + m) put(fb2 + (tid - H), (float)bsum);
    }
}

template <int H, int MP, int NPBM>
__global__ void __launch_bounds__((WallCfg<H, MP, NPBM>::NT)) k_wgrad_all(WallArgs a) {
    if (a.done && *a.done) return;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    wall_body<H, MP, NPBM, 0>(a, blockIdx.x, sm);
}

// ---------------------------------------------------------------------------
// Gather: gsum[f] = sum over slices (fixed order) of the slab element feeding
// flat parameter f (reference order, gaussian_mlp.py:61-64).
// ---------------------------------------------------------------------------
struct GArgs {
    int n, m, h0, h1, np, mp, d, S;
    int64_t off0, off1, off2, boff1, boff2;
    const float* wpart;
    int64_t wcap;           // floats of the scratch's slabs (MJRL_SLAB_CHECK)
    const double* lspart;   // FWD: per-row-kernel-WG log-std partials [G][mp]; null for FVP
    int G;
    float* gsum;
    const int32_t* done;
    CgZ cz;   // fused CG z step (cz.p == nullptr: plain gather)
};

// Block = 16 waves over 64 consecutive flat parameters: lane -> parameter, wave w
// loads its contiguous share of the slices (all loads in flight at once) and sums
// them in slice order; wave 0 adds the sixteen wave partials in order
// (deterministic, fp64).
constexpr int GATHER_WAVES = 16;
constexpr int GATHER_PER = 16;   // slices per wave per batch (S <= 256: one batch)

__global__ void __launch_bounds__(64 * GATHER_WAVES) k_gather(GArgs a) {
    if (a.done && *a.done) return;
    __shared__ double part[GATHER_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int f = blockIdx.x * 64 + lane;
    int64_t src = -1, stride = 0;
    int lsj = -1;
    int g = f;
    if (f >= a.d) {
    } else if (a.h0 == 0) {
        if (g < a.m * a.n) {
            src = a.off0 + (int64_t)(g / a.n) * a.np + g % a.n;
            stride = (int64_t)a.mp * a.np;
        } else if ((g -= a.m * a.n) < a.m) {
            src = a.off0 + (int64_t)g * a.np + a.n;
            stride = (int64_t)a.mp * a.np;
        } else {
            lsj = g - a.m;
        }
    } else {
        const int s0 = a.h0 * a.n, s1 = a.h0, s2 = a.h1 * a.h0, s3 = a.h1, s4 = a.m * a.h1, s5 = a.m;
        if (g < s0) {
            src = a.off0 + (int64_t)(g / a.n) * a.np + g % a.n;
            stride = (int64_t)a.h0 * a.np;
        } else if ((g -= s0) < s1) {
            src = a.off0 + (int64_t)g * a.np + a.n;
            stride = (int64_t)a.h0 * a.np;
        } else if ((g -= s1) < s2) {
            src = a.off1 + g;
            stride = (int64_t)a.h1 * a.h0;
        } else if ((g -= s2) < s3) {
            src = a.boff1 + g;
            stride = a.h1;
        } else if ((g -= s3) < s4) {
            src = a.off2 + g;   // [mp][h1] with rows < m contiguous as [m][h1]
            stride = (int64_t)a.mp * a.h1;
        } else if ((g -= s4) < s5) {
            src = a.boff2 + g;
            stride = a.mp;
        } else {
            lsj = g - s5;
        }
    }
    double acc = 0.0;
    if (src >= 0) {
        const int per = (a.S + GATHER_WAVES - 1) / GATHER_WAVES;
        const int s0 = w * per, s1 = min(a.S, s0 + per);
        const float* p = a.wpart + src;
        if (s1 > s0) MJRL_SLAB_CHECK(src + (int64_t)(s1 - 1) * stride, a.wcap);
        for (int sb = s0; sb < s1; sb += GATHER_PER) {
            float v[GATHER_PER];
#pragma unroll
            for (int j = 0; j < GATHER_PER; ++j) v[j] = sb + j < s1 ? p[(int64_t)(sb + j) * stride] : 0.f;
#pragma unroll
            for (int j = 0; j < GATHER_PER; ++j) acc += (double)v[j];
        }
    } else if (lsj >= 0 && a.lspart) {
        const int per = (a.G + GATHER_WAVES - 1) / GATHER_WAVES;
        const int b0 = w * per, b1 = min(a.G, b0 + per);
        for (int b = b0; b < b1; ++b) acc += a.lspart[(int64_t)b * a.mp + lsj];
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
        float gs = 0.f;
        if (f < a.d) {
            double t = part[0][lane];
#pragma unroll
            for (int j = 1; j < GATHER_WAVES; ++j) t += part[j][lane];
            gs = (float)t;
            a.gsum[f] = gs;
        }
        if (a.cz.p) cgz_epilogue(a.cz, f, a.d, gs);
    }
}

// Gather of the flat slab layout of k_kx: block c folds wpart[c][0..S)[64] — one
// contiguous run — for flat parameters 64c..64c+63 (waves take 16 slices each,
// loads all in flight, fixed-order fp64 sums); log-std entries (FWD) from lspart.
__global__ void __launch_bounds__(64 * GATHER_WAVES) k_gather_flat(const float* __restrict__ wpart, int S, int d_mu,
                                                                   int d, const double* __restrict__ lspart, int G,
                                                                   int mp, float* __restrict__ gsum,
                                                                   const int32_t* __restrict__ done, CgZ cz,
                                                                   int64_t wcap) {
    __shared__ double part[GATHER_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int f = blockIdx.x * 64 + lane;
    float pf = 0.f, lsv = 0.f;   // the CG z step's operands, in flight with the slab loads
    if (w == 0 && cz.p) cgz_load(cz, f, d, pf, lsv);
    double acc = 0.0;
    if (f < d_mu) {
        const int per = (S + GATHER_WAVES - 1) / GATHER_WAVES;
        const int s0 = w * per, s1 = min(S, s0 + per);
        const float* p = wpart + (int64_t)blockIdx.x * S * 64 + lane;
        if (s1 > s0) MJRL_SLAB_CHECK((int64_t)blockIdx.x * S * 64 + lane + (int64_t)(s1 - 1) * 64, wcap);
        for (int sb = s0; sb < s1; sb += GATHER_PER) {
            float v[GATHER_PER];
#pragma unroll
            for (int j = 0; j < GATHER_PER; ++j) v[j] = sb + j < s1 ? p[(int64_t)(sb + j) * 64] : 0.f;
#pragma unroll
            for (int j = 0; j < GATHER_PER; ++j) acc += (double)v[j];
        }
    } else if (f < d && lspart) {
        const int lsj = f - d_mu;
        const int per = (G + GATHER_WAVES - 1) / GATHER_WAVES;
        const int b0 = w * per, b1 = min(G, b0 + per);
        for (int b = b0; b < b1; ++b) acc += lspart[(int64_t)b * mp + lsj];
    }
    part[w][lane] = acc;
    // a converged CG loop: nothing is stored (checked after the slab loads, whose
    // results the store above consumed, so the flag's load overlaps them)
    if (done && *done) return;
    __syncthreads();
    if (w == 0) {
        float gs = 0.f;
        if (f < d) {
            double t = part[0][lane];
#pragma unroll
            for (int j = 1; j < GATHER_WAVES; ++j) t += part[j][lane];
            gs = (float)t;
            gsum[f] = gs;
        }
        if (cz.p) cgz_epilogue(cz, f, d, gs, pf, lsv);
    }
}

__global__ void __launch_bounds__(64) k_eval_final(const double* __restrict__ rpart, int G, double* __restrict__ sums,
                                                   const int32_t* __restrict__ skip) {
    if (skip && *skip) return;
    // one wave: lane l folds partials l, l+64, ... in order, then a fixed shuffle tree
    double s = 0.0, k = 0.0;
    for (int b = threadIdx.x; b < G; b += 64) {
        s += rpart[2 * b];
        k += rpart[2 * b + 1];
    }
    s = wave_sum(s);
    k = wave_sum(k);
    if (threadIdx.x == 0) {
        sums[0] = s;
        sums[1] = k;
    }
}

}  // namespace

#include "fused.h"
#include "ks.h"
#include "kx.h"

namespace {

// ---------------------------------------------------------------------------
// host side: dispatch, grids, scratch sizes
// ---------------------------------------------------------------------------
constexpr int ROW_GRID_CAP = 512;
constexpr int WGRAD_SLICES_CAP = 128;   // 32 / 64 / 256 measured slower on the HalfCheetah / door shapes

inline int bt_for(int h0, int h1) { return rows_bt(h0 > h1 ? h0 : h1); }

inline int row_grid(const mjrl_shape* s, int64_t T) {
    const int bt = bt_for(s->h0, s->h1);
    int64_t nt = (T + bt - 1) / bt;
    if (nt < 1) nt = 1;
    return (int)(nt < ROW_GRID_CAP ? nt : ROW_GRID_CAP);
}

inline int wgrad_slices(int64_t T) {
    int64_t nt = (T + WT - 1) / WT;
    if (nt < 1) nt = 1;
    return (int)(nt < WGRAD_SLICES_CAP ? nt : WGRAD_SLICES_CAP);
}

struct JobSet {
    int njobs;
    WJob job[3];
    int64_t floats;   // per full set (all slices)
};

int64_t slab_floats(const mjrl_shape* s, int S);

JobSet make_jobs(const mjrl_shape* s, const mjrl_rows* r, int S) {
    JobSet js{};
    auto add = [&](const float* G, int ldg, const float* A, int lda, int N, int K, int bias) {
        WJob& j = js.job[js.njobs++];
        j.G = G; j.ldg = ldg; j.A = A; j.lda = lda; j.N = N; j.K = K;
        j.nbN = (N + WB - 1) / WB; j.nbK = (K + WB - 1) / WB; j.bias = bias;
        j.off = js.floats;
        js.floats += (int64_t)S * N * K;
        j.boff = js.floats;
        if (bias) js.floats += (int64_t)S * N;
    };
    if (s->h0 == 0) {
        add(r ? r->gp : nullptr, s->mp, r ? r->xhat : nullptr, s->np, s->mp, s->np, 0);
    } else {
        add(r ? r->gu0 : nullptr, s->h0, r ? r->xhat : nullptr, s->np, s->h0, s->np, 0);
        add(r ? r->gu1 : nullptr, s->h1, r ? r->a0 : nullptr, s->h0, s->h1, s->h0, 1);
        add(r ? r->gp : nullptr, s->mp, r ? r->a1 : nullptr, s->h1, s->mp, s->h1, 1);
    }
    return js;
}

template <int H0, int H1, int MP, int MODE>
int launch_rows_t(const RowArgs& ra, int grid, hipStream_t st) {
    using L = Layout<H0, H1, MP>;
    auto fn = k_rows<H0, H1, MP, MODE>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, L::bytes);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(L::NT), L::bytes, st, ra);
    return (int)hipGetLastError();
}

template <int MODE>
int launch_rows(const mjrl_shape* s, const RowArgs& ra, int grid, hipStream_t st) {
#define MJRL_ROWS_CASE(H0_, H1_, MP_) \
    if (s->h0 == H0_ && s->h1 == H1_ && s->mp == MP_) return launch_rows_t<H0_, H1_, MP_, MODE>(ra, grid, st);
#define MJRL_ROWS_MP(H0_, H1_) MJRL_ROWS_CASE(H0_, H1_, 16) MJRL_ROWS_CASE(H0_, H1_, 32) MJRL_ROWS_CASE(H0_, H1_, 64)
    MJRL_ROWS_MP(0, 0)
    MJRL_ROWS_MP(32, 32)
    MJRL_ROWS_MP(64, 64)
    MJRL_ROWS_MP(128, 128)
    MJRL_ROWS_MP(256, 256)
#undef MJRL_ROWS_MP
#undef MJRL_ROWS_CASE
    return MJRL_ESHAPE;
}

bool shape_supported(int h0, int h1, int mp) {
    if (mp != 16 && mp != 32 && mp != 64) return false;
    if (h0 == 0 && h1 == 0) return true;
    return h0 == h1 && (h0 == 32 || h0 == 64 || h0 == 128 || h0 == 256);
}

RowArgs row_args(const mjrl_shape* s, const mjrl_rows* r, int64_t T) {
    RowArgs ra{};
    ra.T = T;
    ra.np = s->np;
    ra.m = s->m;
    ra.xhat = r->xhat; ra.act = r->act; ra.adv = r->adv; ra.adv_vpg = r->adv_vpg;
    ra.a0 = r->a0; ra.a1 = r->a1; ra.mu0 = r->mu0; ra.ll0 = r->ll0;
    ra.gu0 = r->gu0; ra.gu1 = r->gu1; ra.gp = r->gp;
    ra.xs = r->xs; ra.xu = r->xu; ra.xc = r->xc;
    ra.llc = (float)(-0.5 * (double)s->m * log(2.0 * M_PI));
    return ra;
}

bool fused_supported(const mjrl_shape* s) {
    if (s->h0 != s->h1 || (s->h0 != 32 && s->h0 != 64)) return false;
    if (s->mp != 16 && s->mp != 32) return false;
    const int nch = (s->np + 63) / 64;
    return nch >= 1 && nch <= 6;
}

inline int fused_grid(int64_t T) {
    int64_t nt = (T + 63) / 64;
    if (nt < 1) nt = 1;
    return (int)(nt < FGRID_CAP ? nt : FGRID_CAP);
}

// the K-split kernel (ks.h): MLP(64,64), m <= 32, NP = 32 * KG, NP a multiple of 64
bool ks_supported(const mjrl_shape* s) {
    if (s->h0 != 64 || s->h1 != 64 || (s->mp != 16 && s->mp != 32) || s->np % 32) return false;
    const int kg = s->np / 32;
    return kg == 2 || kg == 4 || kg == 6 || kg == 8 || kg == 12;
}

// persistent grid of the 32-row-tile kernels: at most FGRID_CAP workgroups, as few
// as give every workgroup the same (largest) tile count: the critical path is
// ceil(tiles / FGRID_CAP) tiles either way, and each workgroup fewer is one weight-
// gradient slab fewer for the gather (125k rows: 3907 tiles on 245 workgroups,
// not 256)
inline int ks_grid(int64_t T) {
    int64_t nt = (T + 31) / 32;
    if (nt < 1) nt = 1;
    if (nt <= FGRID_CAP) return (int)nt;
    const int64_t per = (nt + FGRID_CAP - 1) / FGRID_CAP;
    return (int)((nt + per - 1) / per);
}

// which accumulate kernel runs for (shape, T): 2 = K-split, 1 = fused, 0 = rows + wgrad
inline int acc_path(const mjrl_shape* s, int64_t T) {
    if (T <= 0) return 0;
    if (ks_supported(s)) return 2;
    return fused_supported(s) ? 1 : 0;
}

// slices of the weight-gradient slabs the accumulate step produces for (shape, T)
// k_wgrad_all (the MLP weight gradients of a slice in one workgroup): shapes, tile
// rows, slices (at most one per CU, equal tile counts)
inline int wall_npbm(const mjrl_shape* s) {
    const int npb = s->np / 16;
    return npb <= 2 ? 2 : (npb <= 4 ? 4 : (npb <= 8 ? 8 : 0));
}
bool wall_off() {   // MJRL_AMD_WGRAD_OLD (read once): the per-block k_wgrad instead, for A/B runs
    static const bool v = getenv("MJRL_AMD_WGRAD_OLD") && getenv("MJRL_AMD_WGRAD_OLD")[0] == '1';
    return v;
}
bool wall_supported(const mjrl_shape* s) {
    if (wall_off() || s->h0 == 0 || s->h0 != s->h1 || s->np % 16 || !wall_npbm(s)) return false;
    if (s->mp != 16 && s->mp != 32 && s->mp != 64) return false;
    // 256-wide layers keep k_wgrad: one workgroup's accumulators for all three products
    // do not fit its registers, and gW1 alone against gW0 + gW2 on two workgroups per
    // slice measured no faster (door DAPG 94 us either way, profiles/r03i/wgrad_all.txt)
    if (s->h0 == 128 && s->mp == 64 && wall_npbm(s) == 8) return false;   // spills (77 VGPRs): k_wgrad
    return s->h0 == 128 || ((s->h0 == 32 || s->h0 == 64) && s->mp == 64);
}
inline int wall_cap(const mjrl_shape*) { return 256; }   // one slice per CU at most
inline int wall_slices(const mjrl_shape* s, int64_t T) {
    const int bt = 32;
    int64_t tiles = (T + bt - 1) / bt;
    if (tiles < 1) tiles = 1;
    const int cap = wall_cap(s);
    const int64_t tps = (tiles + cap - 1) / cap;
    return (int)((tiles + tps - 1) / tps);
}
inline int rows_slices(const mjrl_shape* s, int64_t T) { return wall_supported(s) ? wall_slices(s, T) : wgrad_slices(T); }

inline int grad_slices(const mjrl_shape* s, int64_t T) {
    const int p = acc_path(s, T);
    return p == 2 ? ks_grid(T) : (p == 1 ? fused_grid(T) : rows_slices(s, T));
}

// the split-f16 first layer additionally needs NP % 128 == 0 (chunk swizzle)
bool ksx_supported(const mjrl_shape* s) { return ks_supported(s) && s->np % 128 == 0; }

template <int MP, int KG, int MODE>
int launch_ks_t(const RowArgs& ra, const FOut& fo, int grid, hipStream_t st) {
    using L = KLayout<MP, KG>;
    auto fn = k_ks<MP, KG, MODE>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, L::bytes);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(KT), L::bytes, st, ra, fo);
    return (int)hipGetLastError();
}

template <int MP, int KG, int MODE, bool PACK = false>
int launch_kx_t(const RowArgs& ra, const FOut& fo, int grid, hipStream_t st) {
    using L = XLayout<MP, KG>;
    auto fn = k_kx<MP, KG, MODE, PACK>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, L::bytes);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(KT), L::bytes, st, ra, fo);
    return (int)hipGetLastError();
}

// rows given as split-f16 (ra.xs) run the all-split kernel k_kx; f32 xhat the
// exact-f32 k_ks
template <int MODE>
int launch_ks(const mjrl_shape* s, const RowArgs& ra, const FOut& fo, int grid, hipStream_t st) {
    const int kg = s->np / 32;
    if (ra.xs) {
#define MJRL_K(MP_, KG_) \
    if (s->mp == MP_ && kg == KG_) return launch_kx_t<MP_, KG_, MODE>(ra, fo, grid, st);
#define MJRL_KN(MP_) MJRL_K(MP_, 4) MJRL_K(MP_, 8) MJRL_K(MP_, 12)
        MJRL_KN(16)
        MJRL_KN(32)
#undef MJRL_KN
#undef MJRL_K
        return MJRL_ESHAPE;
    }
#define MJRL_K(MP_, KG_) \
    if (s->mp == MP_ && kg == KG_) return launch_ks_t<MP_, KG_, MODE>(ra, fo, grid, st);
#define MJRL_KN(MP_) MJRL_K(MP_, 2) MJRL_K(MP_, 4) MJRL_K(MP_, 6) MJRL_K(MP_, 8) MJRL_K(MP_, 12)
    MJRL_KN(16)
    MJRL_KN(32)
#undef MJRL_KN
#undef MJRL_K
    return MJRL_ESHAPE;
}

template <int H, int MP, int NCH, int MODE>
int launch_fused_t(const RowArgs& ra, const FOut& fo, int grid, hipStream_t st) {
    using L = FLayout<H, H, MP, NCH, MODE>;
    auto fn = k_fused<H, H, MP, NCH, MODE>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, L::bytes);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(FT), L::bytes, st, ra, fo);
    return (int)hipGetLastError();
}

template <int MODE>
int launch_fused(const mjrl_shape* s, const RowArgs& ra, const FOut& fo, int grid, hipStream_t st) {
    const int nch = (s->np + 63) / 64;
#define MJRL_F(H_, MP_, N_) \
    if (s->h0 == H_ && s->mp == MP_ && nch == N_) return launch_fused_t<H_, MP_, N_, MODE>(ra, fo, grid, st);
#define MJRL_FN(H_, MP_) MJRL_F(H_, MP_, 1) MJRL_F(H_, MP_, 2) MJRL_F(H_, MP_, 3) MJRL_F(H_, MP_, 4) \
    MJRL_F(H_, MP_, 5) MJRL_F(H_, MP_, 6)
    MJRL_FN(64, 16)
    MJRL_FN(64, 32)
    MJRL_FN(32, 16)
    MJRL_FN(32, 32)
#undef MJRL_FN
#undef MJRL_F
    return MJRL_ESHAPE;
}

int run_fused(int mode, const mjrl_shape* s, const mjrl_rows* r, int64_t T, const RowArgs& ra,
              const mjrl_scratch* sc, hipStream_t st) {
    const bool ks = acc_path(s, T) == 2;
    const int G = ks ? ks_grid(T) : fused_grid(T);
    JobSet js = make_jobs(s, r, G);
    FOut fo{};
    fo.wpart = sc->wpart;
    fo.wcap = slab_floats(s, sc->slices);
    fo.off0 = js.job[0].off;
    fo.off1 = js.job[1].off;
    fo.boff1 = js.job[1].boff;
    fo.off2 = js.job[2].off;
    fo.boff2 = js.job[2].boff;
    fo.n = s->n;
    fo.m = s->m;
    if (ks) {
        if (mode == FWD) return launch_ks<FWD>(s, ra, fo, G, st);
        return launch_ks<FVP>(s, ra, fo, G, st);
    }
    return mode == FWD ? launch_fused<FWD>(s, ra, fo, G, st) : launch_fused<FVP>(s, ra, fo, G, st);
}

// FWD with the fused batch assembly (k_kx<.., FWD, true>): the same workgroups and
// slabs as run_fused's k_kx FWD
int run_fwd_pack(const mjrl_shape* s, const mjrl_rows* r, int64_t T, const RowArgs& ra, const mjrl_scratch* sc,
                 hipStream_t st) {
    const int G = ks_grid(T);
    JobSet js = make_jobs(s, r, G);
    FOut fo{};
    fo.wpart = sc->wpart;
    fo.wcap = slab_floats(s, sc->slices);
    fo.off0 = js.job[0].off;
    fo.off1 = js.job[1].off;
    fo.boff1 = js.job[1].boff;
    fo.off2 = js.job[2].off;
    fo.boff2 = js.job[2].boff;
    fo.n = s->n;
    fo.m = s->m;
    const int kg = s->np / 32;
#define MJRL_K(MP_, KG_) \
    if (s->mp == MP_ && kg == KG_) return launch_kx_t<MP_, KG_, FWD, true>(ra, fo, G, st);
#define MJRL_KN(MP_) MJRL_K(MP_, 4) MJRL_K(MP_, 8) MJRL_K(MP_, 12)
    MJRL_KN(16)
    MJRL_KN(32)
#undef MJRL_KN
#undef MJRL_K
    return MJRL_ESHAPE;
}

int run_gather(const mjrl_shape* s, const mjrl_rows* r, int64_t T, const mjrl_scratch* sc, const double* lspart,
               const int32_t* done, float* gsum, hipStream_t st, CgZ cz = CgZ{}) {
    const int S = grad_slices(s, T);
    const int p = acc_path(s, T);
    if (p == 2 || p == 1 || (p == 0 && wall_supported(s))) {   // k_kx / k_ks / k_fused / k_wgrad_all: flat slabs
        const int d_mu = s->d - s->m;
        const int G = p == 2 ? ks_grid(T) : (p == 1 ? fused_grid(T) : row_grid(s, T));   // log-std partial rows
        hipLaunchKernelGGL(k_gather_flat, dim3((s->d + 63) / 64), dim3(64 * GATHER_WAVES), 0, st, sc->wpart, S, d_mu,
                           s->d, lspart, G, s->mp, gsum, done, cz, slab_floats(s, sc->slices));
        return (int)hipGetLastError();
    }
    JobSet js = make_jobs(s, r, S);
    GArgs ga{};
    ga.n = s->n; ga.m = s->m; ga.h0 = s->h0; ga.h1 = s->h1; ga.np = s->np; ga.mp = s->mp; ga.d = s->d; ga.S = S;
    ga.off0 = js.job[0].off;
    if (s->h0) {
        ga.off1 = js.job[1].off; ga.boff1 = js.job[1].boff;
        ga.off2 = js.job[2].off; ga.boff2 = js.job[2].boff;
    }
    ga.wpart = sc->wpart;
    ga.wcap = slab_floats(s, sc->slices);
    ga.lspart = lspart;
    {
        const int p = acc_path(s, T);
        ga.G = p == 2 ? ks_grid(T) : (p == 1 ? fused_grid(T) : row_grid(s, T));
    }
    ga.gsum = gsum;
    ga.done = done;
    ga.cz = cz;
    hipLaunchKernelGGL(k_gather, dim3((s->d + 63) / 64), dim3(64 * GATHER_WAVES), 0, st, ga);
    return (int)hipGetLastError();
}

// floats of S weight-gradient slabs: the per-job layout of make_jobs or the flat,
// parameter-chunk-major layout of k_kx / k_wgrad_all, whichever is larger
int64_t slab_floats(const mjrl_shape* s, int S) {
    const int64_t jobs = make_jobs(s, nullptr, S).floats;
    const int64_t flat = (int64_t)S * 64 * ((s->d + 63) / 64);
    return jobs > flat ? jobs : flat;
}

template <int H, int MP, int NPBM>
int launch_wall_t(const WallArgs& wa, int S, hipStream_t st) {
    using C = WallCfg<H, MP, NPBM>;
    auto fn = k_wgrad_all<H, MP, NPBM>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, C::bytes);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(S), dim3(C::NT), C::bytes, st, wa);
    return (int)hipGetLastError();
}

int run_wgrad_all(const mjrl_shape* s, const mjrl_rows* r, int64_t T, const mjrl_scratch* sc, const int32_t* done,
                  hipStream_t st) {
    const int S = wall_slices(s, T);
    if (S > sc->slices) return MJRL_EINVAL;   // scratch not sized by mjrl_scratch_size for >= T rows
    WallArgs wa{};
    wa.gu0 = r->gu0; wa.gu1 = r->gu1; wa.gp = r->gp; wa.x = r->xhat; wa.a0 = r->a0; wa.a1 = r->a1;
    wa.n = s->n;
    wa.m = s->m;
    wa.np = s->np;
    wa.S = S;
    wa.T = T;
    const int bt = 32;
    const int64_t tiles = (T + bt - 1) / bt;
    wa.rows_per_slice = ((tiles + S - 1) / S) * bt;
    wa.wpart = sc->wpart;
    wa.wcap = slab_floats(s, sc->slices);
    wa.done = done;
    const int nb = wall_npbm(s);
#define MJRL_W(H_, MP_, NB_) \
    if (s->h0 == H_ && s->mp == MP_ && nb == NB_) return launch_wall_t<H_, MP_, NB_>(wa, S, st);
#define MJRL_WN(H_, MP_) MJRL_W(H_, MP_, 2) MJRL_W(H_, MP_, 4) MJRL_W(H_, MP_, 8)
    MJRL_WN(128, 16) MJRL_WN(128, 32) MJRL_W(128, 64, 2) MJRL_W(128, 64, 4)
    MJRL_WN(32, 64) MJRL_WN(64, 64)
#undef MJRL_WN
#undef MJRL_W
    return MJRL_ESHAPE;
}

int run_wgrad_only(const mjrl_shape* s, const mjrl_rows* r, int64_t T, const mjrl_scratch* sc, const int32_t* done,
                   hipStream_t st) {
    if (T > 0 && wall_supported(s)) return run_wgrad_all(s, r, T, sc, done, st);
    const int S = wgrad_slices(T);
    JobSet js = make_jobs(s, r, S);
    WArgs wa{};
    wa.njobs = js.njobs;
    int tot = 0;
    for (int j = 0; j < js.njobs; ++j) {
        wa.job[j] = js.job[j];
        wa.start[j] = tot;
        tot += js.job[j].nbN * js.job[j].nbK;
    }
    wa.start[js.njobs] = tot;
    wa.S = S;
    wa.T = T;
    const int64_t tiles = (T + WT - 1) / WT;
    wa.rows_per_slice = ((tiles + S - 1) / S) * WT;
    wa.wpart = sc->wpart;
    wa.wcap = slab_floats(s, sc->slices);
    wa.done = done;
    if (T > 0) {
        hipLaunchKernelGGL(k_wgrad, dim3(tot * S), dim3(NTHREADS), 0, st, wa);
    } else {
        hipMemsetAsync(sc->wpart, 0, js.floats * sizeof(float), st);
    }
    return (int)hipGetLastError();
}

bool rows_ok(const mjrl_shape* s, const mjrl_rows* r) {
    if (!s || !r || r->T < 0) return false;
    // split-f16 rows (xs + xu) only feed the K-split kernel; every other path reads f32 xhat
    if (r->xs ? (!r->xu || !r->xc || !ksx_supported(s)) : !r->xhat) return false;
    if (s->h0 && (!r->a0 || !r->a1 || !r->gu0 || !r->gu1)) return false;
    return r->gp != nullptr;
}

}  // namespace

extern "C" {

#ifdef MJRL_KX_PROF
// debug builds only: copy out and clear the k_kx phase profile (16 counters)
int mjrl_debug_kx_prof(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kx_prof), sizeof(unsigned long long) * KX_NPROF);
    if (e != hipSuccess) return (int)e;
    unsigned long long z[KX_NPROF] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_kx_prof), z, sizeof(z));
}
#endif

// What this library was built with (bits): a timing-ablation build (any
// MJRL_KX_ABL_*: results wrong by construction), the phase-profiling build, the
// device-checks (slab guard) build.  UpdateEngine refuses an ablation build unless
// asked for one (tools/fvp_time.py).
int mjrl_build_flags(void) {
    int f = 0;
#if defined(MJRL_KX_ABL_NOP1) || defined(MJRL_KX_ABL_NOP6) || defined(MJRL_KX_ABL_NOCHAIN) || \
    defined(MJRL_KX_ABL_NOCOLS) || defined(MJRL_GAE_ABL_NOLOAD) || defined(MJRL_GAE_ABL_NOCHAIN) ||   \
    defined(MJRL_GAE_ABL_NOFWD)
    f |= MJRL_BUILD_ABLATION;
#endif
#ifdef MJRL_KX_PROF
    f |= MJRL_BUILD_PROF;
#endif
#ifdef MJRL_DEVICE_CHECKS
    f |= MJRL_BUILD_CHECKS;
#endif
    return f;
}

int mjrl_shape_init(mjrl_shape* s, int32_t n, int32_t m, int32_t h0, int32_t h1) {
    if (!s || n <= 0 || m <= 0 || h0 < 0 || h1 < 0) return MJRL_EINVAL;
    s->n = n;
    s->m = m;
    s->h0 = h0;
    s->h1 = h1;
    s->np = round_up(n + 1, 16);
    s->mp = m <= 16 ? 16 : (m <= 32 ? 32 : (m <= 64 ? 64 : round_up(m, 16)));
    if (h0 == 0)
        s->d = m * n + m + m;
    else
        s->d = h0 * n + h0 + h1 * h0 + h1 + m * h1 + m + m;
    s->packed = Packed(h0, h1, s->np, s->mp).total;
    return shape_supported(h0, h1, s->mp) ? MJRL_OK : MJRL_ESHAPE;
}

int mjrl_scratch_size(const mjrl_shape* s, int64_t T, int64_t* wpart_floats, int64_t* rpart_doubles,
                      int32_t* slices) {
    if (!s || T < 0 || !wpart_floats || !rpart_doubles || !slices) return MJRL_EINVAL;
    int S = wgrad_slices(T) > fused_grid(T) ? wgrad_slices(T) : fused_grid(T);
    // k_wgrad_all's slice count is not monotonic in T (equal tile counts per slice):
    // size for its cap, so a scratch sized for T holds every pass over T' <= T rows
    if (T > 0 && wall_supported(s) && wall_cap(s) > S) S = wall_cap(s);
    // ks_grid balances tiles per workgroup and is not monotonic in T (8192 tiles:
    // 256 workgroups, 8224: 129): size for its cap, min(tiles, FGRID_CAP)
    const int64_t nt = (T + 31) / 32;
    const int kcap = (int)(nt < 1 ? 1 : (nt < FGRID_CAP ? nt : FGRID_CAP));
    if (kcap > S) S = kcap;
    *slices = S;
    *wpart_floats = slab_floats(s, S);
    const int64_t rp = (int64_t)ROW_GRID_CAP * (s->mp > 2 ? s->mp : 2);
    *rpart_doubles = rp + 4 * 256 + 16;
    return MJRL_OK;
}

int mjrl_vpg_accumulate(const mjrl_shape* s, const mjrl_rows* rows, const float* packed_theta,
                        const float* out_shift, const float* out_scale, const mjrl_scratch* sc, void* stream) {
    if (!rows_ok(s, rows) || !packed_theta || !sc || !rows->act || !rows->adv_vpg || !rows->mu0 || !rows->ll0)
        return MJRL_EINVAL;
    if (!shape_supported(s->h0, s->h1, s->mp)) return MJRL_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    const int64_t T = rows->T;
    RowArgs ra = row_args(s, rows, T);
    ra.P = packed_theta;
    ra.out_shift = out_shift;
    ra.out_scale = out_scale;
    ra.rpart = sc->rpart;
    if (T == 0) {
        hipMemsetAsync(sc->wpart, 0, slab_floats(s, grad_slices(s, 0)) * sizeof(float), st);
        hipMemsetAsync(sc->rpart, 0, sizeof(double) * row_grid(s, 0) * s->mp, st);
        return (int)hipGetLastError();
    }
    if (acc_path(s, T)) return run_fused(FWD, s, rows, T, ra, sc, st);
    int e = launch_rows<FWD>(s, ra, row_grid(s, T), st);
    if (e) return e;
    return run_wgrad_only(s, rows, T, sc, nullptr, st);
}

int mjrl_vpg_accumulate_pack(const mjrl_shape* s, const mjrl_rows* rows, const float* obs, const float* packed_theta,
                             const float* out_shift, const float* out_scale, const mjrl_scratch* sc, void* stream) {
    if (!rows_ok(s, rows) || !rows->xs || !obs || !packed_theta || !sc || !rows->act || !rows->adv_vpg ||
        !rows->mu0 || !rows->ll0)
        return MJRL_EINVAL;
    if (!ksx_supported(s) || s->n % 4 || (reinterpret_cast<uintptr_t>(obs) & 15) ||
        (reinterpret_cast<uintptr_t>(rows->xs) & 15))
        return MJRL_ESHAPE;
    const int64_t T = rows->T;
    if (T == 0) return mjrl_vpg_accumulate(s, rows, packed_theta, out_shift, out_scale, sc, stream);
    hipStream_t st = (hipStream_t)stream;
    RowArgs ra = row_args(s, rows, T);
    ra.P = packed_theta;
    ra.out_shift = out_shift;
    ra.out_scale = out_scale;
    ra.rpart = sc->rpart;
    ra.obs32 = obs;
    ra.xs_w = (_Float16*)rows->xs;
    ra.xu_w = const_cast<float*>(rows->xu);
    ra.n_obs = s->n;
    return run_fwd_pack(s, rows, T, ra, sc, st);
}

int mjrl_policy_vpg_pack(const mjrl_shape* s, const mjrl_rows* rows, const float* obs, const float* packed_theta,
                         const float* out_shift, const float* out_scale, const mjrl_scratch* sc, float* gsum,
                         void* stream) {
    int e = mjrl_vpg_accumulate_pack(s, rows, obs, packed_theta, out_shift, out_scale, sc, stream);
    if (e) return e;
    return mjrl_gather_grads(s, rows, rows->T, sc, 1, nullptr, gsum, stream);
}

int mjrl_fvp_accumulate(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_fvp, const float* packed_theta,
                        const float* packed_v, const float* out_scale, const int32_t* done, const mjrl_scratch* sc,
                        void* stream) {
    if (!rows_ok(s, rows) || !packed_theta || !packed_v || !sc || T_fvp < 0 || T_fvp > rows->T) return MJRL_EINVAL;
    if (!shape_supported(s->h0, s->h1, s->mp)) return MJRL_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    RowArgs ra = row_args(s, rows, T_fvp);
    ra.P = packed_theta;
    ra.V = packed_v;
    ra.out_scale = out_scale;
    ra.done = done;
    if (T_fvp == 0) {
        hipMemsetAsync(sc->wpart, 0, slab_floats(s, grad_slices(s, 0)) * sizeof(float), st);
        return (int)hipGetLastError();
    }
    if (acc_path(s, T_fvp)) return run_fused(FVP, s, rows, T_fvp, ra, sc, st);
    int e = launch_rows<FVP>(s, ra, row_grid(s, T_fvp), st);
    if (e) return e;
    return run_wgrad_only(s, rows, T_fvp, sc, done, st);
}

int mjrl_gather_grads(const mjrl_shape* s, const mjrl_rows* rows, int64_t T, const mjrl_scratch* sc,
                      int32_t with_log_std, const int32_t* done, float* gsum, void* stream) {
    if (!rows_ok(s, rows) || !sc || !gsum || T < 0 || T > rows->T) return MJRL_EINVAL;
    if (!shape_supported(s->h0, s->h1, s->mp)) return MJRL_ESHAPE;
    return run_gather(s, rows, T, sc, with_log_std ? sc->rpart : nullptr, done, gsum, (hipStream_t)stream);
}

int mjrl_policy_vpg(const mjrl_shape* s, const mjrl_rows* rows, const float* packed_theta, const float* out_shift,
                    const float* out_scale, const mjrl_scratch* sc, float* gsum, void* stream) {
    int e = mjrl_vpg_accumulate(s, rows, packed_theta, out_shift, out_scale, sc, stream);
    if (e) return e;
    return mjrl_gather_grads(s, rows, rows->T, sc, 1, nullptr, gsum, stream);
}

int mjrl_policy_fvp(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_fvp, const float* packed_theta,
                    const float* packed_v, const float* out_scale, const mjrl_scratch* sc, const int32_t* done,
                    float* gsum, void* stream) {
    if (!sc || !gsum) return MJRL_EINVAL;
    int e = mjrl_fvp_accumulate(s, rows, T_fvp, packed_theta, packed_v, out_scale, done, sc, stream);
    if (e) return e;
    return mjrl_gather_grads(s, rows, T_fvp, sc, 0, done, gsum, stream);
}

int mjrl_gather_cg_z(const mjrl_shape* s, const mjrl_rows* rows, int64_t T, const mjrl_scratch* sc,
                     const int32_t* done, float* gsum, double inv_T, float damping, const float* packed_theta,
                     const float* p, float* z, float* cg, void* stream) {
    if (!rows_ok(s, rows) || !sc || !gsum || !packed_theta || !p || !z || !cg || T < 0 || T > rows->T)
        return MJRL_EINVAL;
    if (!shape_supported(s->h0, s->h1, s->mp)) return MJRL_ESHAPE;
    if ((s->d + 63) / 64 > (MJRL_CG_STATE - CG_PZ_PARTS) / 2) return MJRL_EINVAL;   // partials beyond the CG state
    const Packed pk(s->h0, s->h1, s->np, s->mp);
    CgZ cz{p, z, cg, packed_theta + pk.ls, inv_T, damping, s->d - s->m};
    return run_gather(s, rows, T, sc, nullptr, done, gsum, (hipStream_t)stream, cz);
}

int mjrl_fused_path(const mjrl_shape* s) { return s ? acc_path(s, 1) : 0; }

int mjrl_split_supported(const mjrl_shape* s) { return s && ksx_supported(s) ? 1 : 0; }

static int policy_eval(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval, const float* packed_theta_new,
                       const float* packed_theta_old, const float* out_shift, const float* out_scale,
                       const mjrl_scratch* sc, double* sums, const int32_t* skip, void* stream);

int mjrl_policy_eval(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval, const float* packed_theta_new,
                     const float* packed_theta_old, const float* out_shift, const float* out_scale,
                     const mjrl_scratch* sc, double* sums, void* stream) {
    return policy_eval(s, rows, T_eval, packed_theta_new, packed_theta_old, out_shift, out_scale, sc, sums, nullptr,
                       stream);
}

int mjrl_policy_eval_if(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval, const float* packed_theta_new,
                        const float* packed_theta_old, const float* out_shift, const float* out_scale,
                        const mjrl_scratch* sc, double* sums, const int32_t* skip, void* stream) {
    if (!skip) return MJRL_EINVAL;
    return policy_eval(s, rows, T_eval, packed_theta_new, packed_theta_old, out_shift, out_scale, sc, sums, skip,
                       stream);
}

static int policy_eval(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval, const float* packed_theta_new,
                       const float* packed_theta_old, const float* out_shift, const float* out_scale,
                       const mjrl_scratch* sc, double* sums, const int32_t* skip, void* stream) {
    if (!rows_ok(s, rows) || !packed_theta_new || !packed_theta_old || !sc || !sums || T_eval < 0 ||
        T_eval > rows->T || !rows->adv || !rows->mu0 || !rows->ll0)
        return MJRL_EINVAL;
    if (!shape_supported(s->h0, s->h1, s->mp)) return MJRL_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    RowArgs ra = row_args(s, rows, T_eval);
    ra.P = packed_theta_new;
    ra.V = packed_theta_old;
    ra.out_shift = out_shift;
    ra.out_scale = out_scale;
    ra.rpart = sc->rpart;
    ra.done = skip;   // EVAL: the whole pass is skipped while *skip != 0
    // forward-only: the K-split kernel in EVAL mode where it applies, else the row kernel
    const bool ks = ks_supported(s);
    const int G = ks ? ks_grid(T_eval) : row_grid(s, T_eval);
    if (T_eval > 0) {
        int e = ks ? launch_ks<EVAL>(s, ra, FOut{}, G, st) : launch_rows<EVAL>(s, ra, G, st);
        if (e) return e;
    } else {
        hipMemsetAsync(sc->rpart, 0, sizeof(double) * 2 * G, st);
    }
    hipLaunchKernelGGL(k_eval_final, dim3(1), dim3(64), 0, st, sc->rpart, G, sums, skip);
    return (int)hipGetLastError();
}

}  // extern "C"
