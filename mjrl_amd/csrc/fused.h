// fused.h — persistent fused VPG / FVP kernel for hidden widths <= 64
// (included by policy.hip: shares RowArgs, gemm_tile and the k_gather slab layout).
//
// One 512-thread workgroup (8 waves) per CU walks 64-row tiles of timesteps.
// Per tile everything stays on chip:
//   phase 1   xhat tile streamed in 64-column chunks through LDS (double
//             buffered through registers) x W0 (or the tangent dW0) -> [64 x H0]
//   phase 2-5 the row chain of k_rows (JVP / forward, GN weight / log-lik,
//             backprop) with every intermediate in LDS
//   grads     gW2 += gp^T a1, gW1 += gu1^T a0, gb1 / gb2 column sums, and
//             gW0 += gu0^T xhat with the tile re-streamed (L2-hot) — all
//             accumulated in REGISTERS across the workgroup's tiles
// and each workgroup writes its slab at the end in the flat, parameter-chunk-major
// layout of k_kx, so k_gather_flat folds them (each 64-parameter chunk one
// contiguous run).
// Replaces k_rows<FWD|FVP> + k_wgrad: the gu0 / gu1 / gp round trip through HBM
// and k_wgrad's re-reads disappear.
#pragma once

namespace {

constexpr int FT = 512;          // threads per workgroup (8 waves)
constexpr int FGRID_CAP = 256;   // one persistent workgroup per CU

// Output tiles [RB x CB] (16x16 each) over 8 waves: each wave owns NRW row
// blocks x NCW col blocks; waves sharing a col block reuse its B fragment.
template <int RB, int CB>
struct Split8 {
    static constexpr int WPC = CB >= 8 ? 1 : 8 / CB;   // waves per col block
    static constexpr int NCW = CB >= 8 ? CB / 8 : 1;
    static constexpr int NRW = CB >= 8 ? RB : (RB / WPC > 0 ? RB / WPC : 1);
    static constexpr int CBS = CB >= 8 ? 8 : 1;
    static constexpr int RBS = CB >= 8 ? 1 : WPC;
    __device__ static int cb0(int w) { return CB >= 8 ? w : w % CB; }
    __device__ static int rb0(int w) { return CB >= 8 ? 0 : w / CB; }
};

// LDS: the tile's activations / upstreams, the xhat chunk buffer(s) (one when the
// observations fit one 64-column chunk: the gW0 sums then reuse phase 1's chunk),
// and — where they fit in the 160 KB — row-major images of W1 and W2 (and the
// tangent's in FVP mode; phases 4 / 5 read them transposed for W2^T / W1^T) and of
// the first layer's W0 (one chunk), loaded once per launch: every phase's weight
// operand is then an LDS read instead of an L2 round trip on the tile's critical path.
template <int H0, int H1, int MP, int NCH, int MODE>
struct FLayout {
    static constexpr int BT = 64;
    static constexpr int LD0 = H0 + 4, LD1 = H1 + 4, LDP = MP + 4, KC = 64, LDX = KC + 4;
    static constexpr int LW0 = KC + 4, LW1 = H0 + 4, LW2 = H1 + 4;
    static constexpr int NV = MODE == FVP ? 2 : 1;   // P's images (+ the tangent's)
    static constexpr int oD0 = 0;
    static constexpr int oA0 = oD0 + BT * LD0;
    static constexpr int oD1 = oA0 + BT * LD0;
    static constexpr int oA1 = oD1 + BT * LD1;
    static constexpr int oGP = oA1 + BT * LD1;
    static constexpr int oXS = oGP + BT * LDP;
    static constexpr int oW1 = oXS + (NCH == 1 ? 1 : 2) * BT * LDX;
    static constexpr int oW1V = oW1 + H1 * LW1;
    static constexpr int oW2 = oW1 + NV * H1 * LW1;
    static constexpr int oW2V = oW2 + MP * LW2;
    static constexpr int oW0 = oW2 + NV * MP * LW2;
    static constexpr int LDS_CAP = 160 * 1024 / 4;
    static constexpr bool IMG = oW0 <= LDS_CAP;
    static constexpr bool IMG0 = IMG && NCH == 1 && oW0 + H0 * LW0 <= LDS_CAP;
    static constexpr int total = IMG0 ? oW0 + H0 * LW0 : (IMG ? oW0 : oW1);
    static constexpr int bytes = total * 4;
    static_assert(LD0 >= MP, "log-std scratch lives in D0");
    static_assert(total <= LDS_CAP, "LDS");
};

// A [ROWS][COLS] row-major weight block (global, row stride ld_src) to an LDS image
// (row stride ld_dst): all of a thread's 16-byte loads in flight before its stores.
template <int ROWS, int COLS>
struct ImgCopy {
    static constexpr int N4 = ROWS * COLS / 4, IT = (N4 + FT - 1) / FT;
    static_assert(COLS % 4 == 0, "16-byte rows");
    float4 v[IT];
    __device__ __forceinline__ void load(const float* __restrict__ src, int ld_src, int col_lim, int tid) {
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int idx = tid + u * FT;
            const int row = idx / (COLS / 4), c = (idx % (COLS / 4)) * 4;
            v[u] = (idx < N4 && c < col_lim) ? *reinterpret_cast<const float4*>(src + row * ld_src + c)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __device__ __forceinline__ void store(float* dst, int ld_dst, int tid) const {
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int idx = tid + u * FT;
            if (idx < N4) *reinterpret_cast<float4*>(dst + (idx / (COLS / 4)) * ld_dst + (idx % (COLS / 4)) * 4) = v[u];
        }
    }
};

// gemm_tile with the weight operand read TRANSPOSED from a row-major LDS image:
// acc[i][j] += sum_k A[rows of rb(i)][k] * Wt[k][cols of cb(j)], k in [0, ke).
template <int NRW, int NCW>
__device__ __forceinline__ void gemm_tile_t(floatx4 (&acc)[NRW][NCW], const float* As, int lda, int rb0, int rbs,
                                            int rb_lim, const float* Wt, int ldt, int cb0, int cbs, int ke,
                                            int lane) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll MJRL_GEMM_UNROLL
    for (int k = 0; k < ke; k += 16) {
        float4 b[NCW];
#pragma unroll
        for (int j = 0; j < NCW; ++j) {
            const float* pb = Wt + (k + 4 * q) * ldt + (cb0 + j * cbs) * 16 + r;
            b[j] = make_float4(pb[0], pb[ldt], pb[2 * ldt], pb[3 * ldt]);
        }
#pragma unroll
        for (int i = 0; i < NRW; ++i) {
            const int rb = rb0 + i * rbs;
            if (rb >= rb_lim) continue;
            const float4 a = *reinterpret_cast<const float4*>(As + (rb * 16 + r) * lda + k + 4 * q);
#pragma unroll
            for (int j = 0; j < NCW; ++j) acc[i][j] = mfma_k16(a, b[j], acc[i][j]);
        }
    }
}

struct FOut {
    float* wpart;
    int64_t off0, off1, boff1, off2, boff2;   // per-job slab offsets (make_jobs; unused by the flat writers)
    int n, m;                                 // k_kx / k_ks / k_fused: flat layout wpart[f / 64][S][64] (k_gather_flat)
    int64_t wcap;                             // floats of the scratch's slabs (MJRL_SLAB_CHECK)
};

// acc[i][j] += sum_{t<64} G[t][n-block] * A[t][k-block], both row-major in LDS.
template <int NRW, int NCW>
__device__ __forceinline__ void wgrad_lds(floatx4 (&acc)[NRW][NCW], const float* G, int ldg, const float* A,
                                          int lda, int nb0, int nbs, int nb_lim, int kb0, int kbs, int kb_lim,
                                          int lane) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll 4
    for (int t = 0; t < 64; t += 4) {
        float ga[NRW], ab[NCW];
#pragma unroll
        for (int i = 0; i < NRW; ++i) {
            const int nb = nb0 + i * nbs;
            ga[i] = nb < nb_lim ? G[(t + q) * ldg + nb * 16 + r] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < NCW; ++j) {
            const int kb = kb0 + j * kbs;
            ab[j] = kb < kb_lim ? A[(t + q) * lda + kb * 16 + r] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < NRW; ++i)
#pragma unroll
            for (int j = 0; j < NCW; ++j) acc[i][j] = mfma4(ga[i], ab[j], acc[i][j]);
    }
}

// The body of k_fused: this workgroup's tiles (blockIdx.x + k gridDim.x), then its
// slab.
template <int H0, int H1, int MP, int NCH, int MODE>
__device__ __forceinline__ void fused_body(const RowArgs& a, const FOut& o) {
    using L = FLayout<H0, H1, MP, NCH, MODE>;
    constexpr int BT = L::BT, RB = 4, KC = L::KC;
    using S1 = Split8<RB, H0 / 16>;
    using S2 = Split8<RB, H1 / 16>;
    using S3 = Split8<RB, MP / 16>;
    using W0S = Split8<H0 / 16, KC / 16>;
    using W1S = Split8<H1 / 16, H0 / 16>;
    using W2S = Split8<MP / 16, H1 / 16>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* D0 = smem + L::oD0;
    float* A0s = smem + L::oA0;
    float* D1 = smem + L::oD1;
    float* A1s = smem + L::oA1;
    float* GPs = smem + L::oGP;
    float* XS = smem + L::oXS;

#ifdef MJRL_KX_PROF
    // phase profile (profiling builds, the k_kx counters): wave 0 of workgroup 0
    unsigned long long kx_acc_[KX_NPROF] = {0};
    unsigned long long kx_last_ = __builtin_amdgcn_s_memtime();
    kx_acc_[17] = 1;
#endif
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, q = lane >> 4;
    const int np = a.np, m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;
    const float* P = a.P;
    const float* V = MODE == FVP ? a.V : a.P;   // weights of the first-layer GEMM / biases
    const Packed pk(H0, H1, np, MP);

    floatx4 g0[NCH][W0S::NRW][W0S::NCW];
    floatx4 g1[W1S::NRW][W1S::NCW];
    floatx4 g2[W2S::NRW][W2S::NCW];
#pragma unroll
    for (int c = 0; c < NCH; ++c) zero_acc(g0[c]);
    zero_acc(g1);
    zero_acc(g2);
    float b1acc = 0.f, b2acc = 0.f;
    double racc0 = 0.0, racc1 = 0.0;   // row-pass partials (FWD), folded at the end
    const float sls = MODE == FWD ? ls_sum(P + pk.ls, m) : 0.f;

    constexpr int PER = BT * (KC / 4) / FT;   // float4 per thread per chunk
    float4 st[PER];
    auto gload = [&](int64_t row_base, int c) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = tid + u * FT;
            const int row = idx / (KC / 4), c4 = idx % (KC / 4);
            const int col = c * KC + c4 * 4;
            const int64_t gr = row_base + row;
            st[u] = (gr < T && col < np) ? *reinterpret_cast<const float4*>(a.xhat + gr * np + col)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto lstore = [&](float* xs) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = tid + u * FT;
            const int row = idx / (KC / 4), c4 = idx % (KC / 4);
            *reinterpret_cast<float4*>(xs + row * L::LDX + c4 * 4) = st[u];
        }
    };

    bool pre = false;
    // FVP: this lane's cached activations for epilogues 1 / 2 of a tile (the
    // tile's first loads)
    float pa0[S1::NRW][S1::NCW][4], pa1[S2::NRW][S2::NCW][4];
    auto paload = [&](int64_t row_base) {
        if (MODE != FVP) return;
#pragma unroll
        for (int i = 0; i < S1::NRW; ++i)
#pragma unroll
            for (int j = 0; j < S1::NCW; ++j)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int rb = S1::rb0(w) + i * S1::RBS;
                    const int64_t gr = row_base + rb * 16 + 4 * q + rr;
                    const int col = (S1::cb0(w) + j * S1::CBS) * 16 + r16;
                    pa0[i][j][rr] = (rb < RB && gr < T) ? a.a0[gr * H0 + col] : 0.f;
                }
#pragma unroll
        for (int i = 0; i < S2::NRW; ++i)
#pragma unroll
            for (int j = 0; j < S2::NCW; ++j)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int rb = S2::rb0(w) + i * S2::RBS;
                    const int64_t gr = row_base + rb * 16 + 4 * q + rr;
                    const int col = (S2::cb0(w) + j * S2::CBS) * 16 + r16;
                    pa1[i][j][rr] = (rb < RB && gr < T) ? a.a1[gr * H1 + col] : 0.f;
                }
    };
    // weight images (once per launch; the barrier is the first tile's)
    const float* W0b = V + pk.W0;   // phase 1's weights (row stride np)
    int ldw0 = np;
    const float* W1p = P + pk.W1;   // phase 2 / 5 (row stride H0)
    const float* W1v = V + pk.W1;
    int ldw1 = H0;
    const float* W2p = P + pk.W2;   // phase 3 / 4 (row stride H1)
    const float* W2v = V + pk.W2;
    int ldw2 = H1;
    if constexpr (L::IMG) {
        ImgCopy<H1, H0> c1, c1v;
        ImgCopy<MP, H1> c2, c2v;
        ImgCopy<H0, L::KC> c0;
        c1.load(W1p, H0, H0, tid);
        c2.load(W2p, H1, H1, tid);
        if (MODE == FVP) {
            c1v.load(W1v, H0, H0, tid);
            c2v.load(W2v, H1, H1, tid);
        }
        if (L::IMG0) c0.load(W0b, np, np, tid);
        if (blockIdx.x < ntiles) {   // the first tile's first chunk, in flight with the images
            gload((int64_t)blockIdx.x * BT, 0);
            pre = true;
        }
        c1.store(smem + L::oW1, L::LW1, tid);
        c2.store(smem + L::oW2, L::LW2, tid);
        if (MODE == FVP) {
            c1v.store(smem + L::oW1V, L::LW1, tid);
            c2v.store(smem + L::oW2V, L::LW2, tid);
        }
        if (L::IMG0) c0.store(smem + L::oW0, L::LW0, tid);
        W1p = smem + L::oW1;
        W1v = MODE == FVP ? smem + L::oW1V : W1p;
        W2p = smem + L::oW2;
        W2v = MODE == FVP ? smem + L::oW2V : W2p;
        ldw1 = L::LW1;
        ldw2 = L::LW2;
        if (L::IMG0) {
            W0b = smem + L::oW0;
            ldw0 = L::LW0;
        }
    }
    // a converged CG loop (cg_solve.py:19-20): checked once the preamble's loads have
    // been consumed, so the flag's load overlaps them
    // FVP: a converged CG loop (cg_solve.py:19-20); EVAL: a TRPO trial the device line
    // search no longer needs (mjrl_policy_eval_if)
    if ((MODE == FVP || MODE == EVAL) && a.done && *a.done) return;

    KX_STAMP(15);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row_base = tile * BT;

        paload(row_base);
        KX_STAMP(0);
        // ---------------- phase 1: [64 x H0] = xhat * W0^T (or dW0^T) ----------------
        floatx4 acc1[S1::NRW][S1::NCW];
        zero_acc(acc1);
        if (!pre) gload(row_base, 0);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            float* xs = XS + (c & 1) * BT * L::LDX;
            lstore(xs);
            __syncthreads();
            if (c + 1 < NCH) gload(row_base, c + 1);
            const int kb = c * KC;
            const int ke = kb + KC < np ? kb + KC : np;
            gemm_tile(acc1, xs, L::LDX, kb, S1::rb0(w), S1::RBS, RB, W0b, ldw0, S1::cb0(w), S1::CBS, kb, ke, lane);
        }
        KX_STAMP(1);
        // epilogue 1
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
                        const float av = pa0[i][j][rr];
                        D0[row * L::LD0 + col] = (1.f - av * av) * v;
                        A0s[row * L::LD0 + col] = av;
                    } else {
                        const float av = tanhf(v);
                        A0s[row * L::LD0 + col] = av;
                        if (gr < T) a.a0[gr * H0 + col] = av;
                    }
                }
            }
        }
        __syncthreads();
        KX_STAMP(2);

        // ---------------- phase 2: [64 x H1], K = H0 ----------------
        {
            floatx4 acc2[S2::NRW][S2::NCW];
            zero_acc(acc2);
            if (MODE == FVP) {
                gemm_tile(acc2, D0, L::LD0, 0, S2::rb0(w), S2::RBS, RB, W1p, ldw1, S2::cb0(w), S2::CBS, 0, H0, lane);
                gemm_tile(acc2, A0s, L::LD0, 0, S2::rb0(w), S2::RBS, RB, W1v, ldw1, S2::cb0(w), S2::CBS, 0, H0, lane);
            } else {
                gemm_tile(acc2, A0s, L::LD0, 0, S2::rb0(w), S2::RBS, RB, W1p, ldw1, S2::cb0(w), S2::CBS, 0, H0, lane);
            }
#pragma unroll
            for (int i = 0; i < S2::NRW; ++i) {
                const int rb = S2::rb0(w) + i * S2::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S2::NCW; ++j) {
                    const int col = (S2::cb0(w) + j * S2::CBS) * 16 + r16;
                    const float bias = V[pk.b1 + col];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * q + rr;
                        const int64_t gr = row_base + row;
                        const float v = acc2[i][j][rr] + bias;
                        if (MODE == FVP) {
                            const float av = pa1[i][j][rr];
                            D1[row * L::LD1 + col] = (1.f - av * av) * v;
                            A1s[row * L::LD1 + col] = av;
                        } else {
                            const float av = tanhf(v);
                            A1s[row * L::LD1 + col] = av;
                            if (gr < T) a.a1[gr * H1 + col] = av;
                        }
                    }
                }
            }
        }
        __syncthreads();
        KX_STAMP(3);

        // ---------------- phase 3: [64 x MP], K = H1 ----------------
        {
            floatx4 acc3[S3::NRW][S3::NCW];
            zero_acc(acc3);
            if (MODE == FVP) {
                gemm_tile(acc3, D1, L::LD1, 0, S3::rb0(w), S3::RBS, RB, W2p, ldw2, S3::cb0(w), S3::CBS, 0, H1, lane);
                gemm_tile(acc3, A1s, L::LD1, 0, S3::rb0(w), S3::RBS, RB, W2v, ldw2, S3::cb0(w), S3::CBS, 0, H1, lane);
            } else {
                gemm_tile(acc3, A1s, L::LD1, 0, S3::rb0(w), S3::RBS, RB, W2p, ldw2, S3::cb0(w), S3::CBS, 0, H1, lane);
            }
#pragma unroll
            for (int i = 0; i < S3::NRW; ++i) {
                const int rb = S3::rb0(w) + i * S3::RBS;
                if (rb >= RB) continue;
#pragma unroll
                for (int j = 0; j < S3::NCW; ++j) {
                    const int col = (S3::cb0(w) + j * S3::CBS) * 16 + r16;
                    const float bias = V[pk.b2 + col];
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
                        const bool valid = row_base + row < T;
                        const float v = acc3[i][j][rr] + bias;
                        if (MODE == FVP)
                            GPs[row * L::LDP + col] = (col < m && valid) ? wq * v : 0.f;
                        else
                            GPs[row * L::LDP + col] = col < m ? v * os + osh : 0.f;
                    }
                }
            }
        }
        __syncthreads();
        KX_STAMP(4);

        // ---------------- FWD: log-likelihood, caches, VPG upstream ----------------
        if (MODE == FWD) {
            row_pass<MODE, BT, MP, FT, false>(a, P + pk.ls, sls, row_base, GPs, L::LDP, racc0, racc1, tid);
            __syncthreads();
        }

        KX_STAMP(5);
        // ---------------- phase 4: gu1 = (1 - a1^2) (g W2) ----------------
        {
            floatx4 acc4[S2::NRW][S2::NCW];
            zero_acc(acc4);
            if constexpr (L::IMG)   // W2^T: the W2 image read transposed
                gemm_tile_t(acc4, GPs, L::LDP, S2::rb0(w), S2::RBS, RB, W2p, ldw2, S2::cb0(w), S2::CBS, MP, lane);
            else
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
                        D1[row * L::LD1 + col] = row_base + row < T ? (1.f - av * av) * acc4[i][j][rr] : 0.f;
                    }
                }
            }
        }
        __syncthreads();
        KX_STAMP(6);

        // ---------------- phase 5: gu0 = (1 - a0^2) (gu1 W1) ----------------
        {
            floatx4 acc5[S1::NRW][S1::NCW];
            zero_acc(acc5);
            if constexpr (L::IMG)   // W1^T: the W1 image read transposed
                gemm_tile_t(acc5, D1, L::LD1, S1::rb0(w), S1::RBS, RB, W1p, ldw1, S1::cb0(w), S1::CBS, H1, lane);
            else
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
                        D0[row * L::LD0 + col] = row_base + row < T ? (1.f - av * av) * acc5[i][j][rr] : 0.f;
                    }
                }
            }
        }
        __syncthreads();
        KX_STAMP(7);

        // ---------------- weight gradients, accumulated in registers ----------------
        wgrad_lds(g2, GPs, L::LDP, A1s, L::LD1, W2S::rb0(w), W2S::RBS, MP / 16, W2S::cb0(w), W2S::CBS, H1 / 16,
                  lane);
        wgrad_lds(g1, D1, L::LD1, A0s, L::LD0, W1S::rb0(w), W1S::RBS, H1 / 16, W1S::cb0(w), W1S::CBS, H0 / 16,
                  lane);
        KX_STAMP(8);
        if (tid < H1) {
            float s = 0.f;
            for (int row = 0; row < BT; ++row) s += D1[row * L::LD1 + tid];
            b1acc += s;
        } else if (tid < H1 + MP) {
            float s = 0.f;
            for (int row = 0; row < BT; ++row) s += GPs[row * L::LDP + tid - H1];
            b2acc += s;
        }
        KX_STAMP(9);
        // gW0 += gu0^T xhat: re-stream the tile's chunks (L2-hot); the last chunk
        // prefetches the next tile's first chunk
        const int64_t next = tile + gridDim.x;
        if constexpr (NCH == 1) {
            // the tile's only chunk is still in XS (phase 1's): no re-stream
            if (next < ntiles) gload(next * BT, 0);
            const int kb_lim = np / 16 < KC / 16 ? np / 16 : KC / 16;
            wgrad_lds(g0[0], D0, L::LD0, XS, L::LDX, W0S::rb0(w), W0S::RBS, H0 / 16, W0S::cb0(w), W0S::CBS, kb_lim,
                      lane);
        } else {
            gload(row_base, 0);
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                float* xs = XS + (c & 1) * BT * L::LDX;
                lstore(xs);
                __syncthreads();
                if (c + 1 < NCH) {
                    gload(row_base, c + 1);
                } else if (next < ntiles) {
                    gload(next * BT, 0);
                }
                const int kb_lim = (np - c * KC) / 16 < KC / 16 ? (np - c * KC) / 16 : KC / 16;
                wgrad_lds(g0[c], D0, L::LD0, xs, L::LDX, W0S::rb0(w), W0S::RBS, H0 / 16, W0S::cb0(w), W0S::CBS,
                          kb_lim, lane);
            }
        }
        pre = next < ntiles;
        __syncthreads();
        KX_STAMP(10);
    }

    // ---------------- this workgroup's slab (slice = blockIdx.x) in the flat,
    // parameter-chunk-major layout wpart[f / 64][S][64] (k_gather_flat): flat parameter
    // f in the reference order W0, b0, W1, b1, W2, b2 (gaussian_mlp.py:61-64); padded
    // columns / rows are not stored.  When the slab fits, it is staged in LDS in flat
    // order (the tile buffers are free after the loop's last barrier) and leaves in
    // 16-byte stores, as k_kx's does ----------------
    const int64_t blk = blockIdx.x;
    const int nobs = o.n, mact = o.m;
    const int fb0 = H0 * nobs, fW1 = fb0 + H0, fb1 = fW1 + H1 * H0, fW2 = fb1 + H1, fb2 = fW2 + mact * H1;
    const int dmu = fb2 + mact;
    const bool stage = dmu <= L::total;
    float* wp = o.wpart + blk * 64;
    const int64_t cs = (int64_t)gridDim.x * 64;
    auto put = [&](int f, float v) {
        if (stage) {
            smem[f] = v;
        } else {
            MJRL_SLAB_CHECK(blk * 64 + (int64_t)(f >> 6) * cs + (f & 63), o.wcap);
            wp[(int64_t)(f >> 6) * cs + (f & 63)] = v;
        }
    };
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int i = 0; i < W0S::NRW; ++i)
#pragma unroll
            for (int j = 0; j < W0S::NCW; ++j)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int n = (W0S::rb0(w) + i * W0S::RBS) * 16 + 4 * q + rr;
                    const int k = c * KC + (W0S::cb0(w) + j * W0S::CBS) * 16 + r16;
                    if (n < H0 && k < nobs) put(n * nobs + k, g0[c][i][j][rr]);
                    else if (n < H0 && k == nobs) put(fb0 + n, g0[c][i][j][rr]);   // the bias column: b0
                }
#pragma unroll
    for (int i = 0; i < W1S::NRW; ++i)
#pragma unroll
        for (int j = 0; j < W1S::NCW; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = (W1S::rb0(w) + i * W1S::RBS) * 16 + 4 * q + rr;
                const int k = (W1S::cb0(w) + j * W1S::CBS) * 16 + r16;
                if (n < H1 && k < H0) put(fW1 + n * H0 + k, g1[i][j][rr]);
            }
#pragma unroll
    for (int i = 0; i < W2S::NRW; ++i)
#pragma unroll
        for (int j = 0; j < W2S::NCW; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = (W2S::rb0(w) + i * W2S::RBS) * 16 + 4 * q + rr;
                const int k = (W2S::cb0(w) + j * W2S::CBS) * 16 + r16;
                if (n < mact && k < H1) put(fW2 + n * H1 + k, g2[i][j][rr]);
            }
    if (tid < H1)
        put(fb1 + tid, b1acc);
    else if (tid < H1 + mact)
        put(fb2 + (tid - H1), b2acc);
    KX_STAMP(11);
    if (stage) {
        __syncthreads();
        KX_STAMP(12);
        for (int f0 = 4 * tid; f0 < dmu; f0 += 4 * FT) {
            const int64_t gi = ((int64_t)(f0 >> 6) * gridDim.x + blk) * 64 + (f0 & 63);   // f0 % 4 == 0: one chunk
            if (f0 + 3 < dmu) {
                MJRL_SLAB_CHECK(gi + 3, o.wcap);
                *reinterpret_cast<float4*>(o.wpart + gi) = *reinterpret_cast<const float4*>(smem + f0);
            } else {
                for (int e = 0; f0 + e < dmu; ++e) {
                    MJRL_SLAB_CHECK(gi + e, o.wcap);
                    o.wpart[gi + e] = smem[f0 + e];
                }
            }
        }
    }
    if (MODE == FWD) {
        static_assert(L::total >= 2 * FT, "row_pass_final scratch");
        __syncthreads();
        row_pass_final<MODE, MP, FT>(racc0, racc1, reinterpret_cast<double*>(smem), a.rpart, blk, tid);
    }
#ifdef MJRL_KX_PROF
    KX_STAMP(16);
    if (blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < KX_NPROF; ++i) g_kx_prof[i] += kx_acc_[i];
#endif
}

template <int H0, int H1, int MP, int NCH, int MODE>
__global__ void __launch_bounds__(FT, 1) k_fused(RowArgs a, FOut o) {
    fused_body<H0, H1, MP, NCH, MODE>(a, o);
}

}  // namespace
