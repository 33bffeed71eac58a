// ks.h — persistent fused FWD / FVP / EVAL kernel for the MLP(64,64) policy with a
// wide observation (NP = 32*KG, up to 384: Humanoid), included by policy.hip.
//
// One 512-thread workgroup (8 waves) per CU walks 32-row tiles of timesteps with
// NO global load inside the tile loop except the tile's xhat (and, for FVP, the
// cached activations):
//   - wave w owns hidden block cb = w&3 and observation half kh = w>>2: its slice of
//     W0 (FWD / EVAL) or of the tangent dW0 (FVP) — 16 x NP/2 — lives in
//     REGISTERS as MFMA B fragments for the whole launch, and so does its slice of
//     the gW0 accumulator;
//   - W1 / dW1 / W2 / dW2 live in LDS for the whole launch;
//   - the 32-row xhat tile sits in LDS for both the first-layer GEMM and the gW0
//     update; the next tile's lines are pulled into L2 meanwhile.
// Phase 1 computes per-half partial sums, folded through LDS; phases 2-5 are the
// row chain of k_rows; gW1 / gW2 / biases accumulate in registers too.  Slabs
// are written at the end in k_gather's layout.
//
// The split-f16 form of this tile walk, with every product on f16 MFMA, is k_kx
// (kx.h); this kernel is the exact-f32 path (precision = 'f32').
#pragma once

namespace {

constexpr int KT = 512;

template <int MP, int KG>
struct KLayout {
    static constexpr int H = 64, BT = 32, RB = 2;
    static constexpr int NP = 32 * KG, KH = NP / 2;
    static constexpr int LDX = NP + 16;   // rows 4 apart fall 16 banks apart for the b32 gW0 reads
    static constexpr int LD = H + 4, LDP = MP + 4;
    static_assert(KT == BT * H / 4, "tanh_tile: one float4 per thread");
    static constexpr int XFLOATS = BT * LDX;
    static constexpr int oXT = 0;
    static constexpr int oD0 = oXT + XFLOATS;
    static constexpr int oA0 = oD0 + BT * LD;
    static constexpr int oD1 = oA0 + BT * LD;
    static constexpr int oA1 = oD1 + BT * LD;
    static constexpr int oGP = oA1 + BT * LD;
    static constexpr int oW1 = oGP + BT * LDP;     // [64][LD]  W1  (out x in)
    static constexpr int odW1 = oW1 + H * LD;      // [64][LD]  dW1 (FVP)
    static constexpr int oW2 = odW1 + H * LD;      // [MP][LD]  W2p
    static constexpr int odW2 = oW2 + MP * LD;     // [MP][LD]  dW2p (FVP)
    static constexpr int total = odW2 + MP * LD;
    static constexpr int bytes = total * 4;
    static_assert(bytes <= 160 * 1024, "LDS");
    static constexpr int XPER = BT * NP / 4 / KT;  // 16-byte pieces of the xhat tile per thread
    static_assert(XPER * KT * 4 == BT * NP, "NP must be a multiple of 64");
};

// XOR swizzle of the 16-byte chunks of row `row` in k_kx's xhat images (rows of
// NP halves, a multiple of 256 B): ds_read_b128 of 16 rows (lane groups
// {0-3,12-15,20-27}, ... of MI355X_MICROARCH.md §LDS) and ds_read_b64_tr_b16 of
// rows {8q + 4h + 0..3} (32-lane halves) both touch 64 distinct banks (found by
// exhaustive search over XOR-linear maps, tools/swizzle_search.py).
__device__ __forceinline__ int chunk_swz(int row) {
    return ((row & 1) << 1) | (((row >> 1) & 1) << 2) | (((row >> 3) & 1) << 3);
}

// acc += A[rows][k] (LDS, row-major) x B where B(k, n) = Bs[n][k] (LDS, row-major by n)
template <int NR>
__device__ __forceinline__ void mm_lds_nk(floatx4 (&acc)[NR], const float* As, int lda, int rb0, int rbs,
                                          const float* Bs, int ldb, int cb, int K, int lane) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int k = 0; k < K; k += 16) {
        const float4 b = *reinterpret_cast<const float4*>(Bs + (cb * 16 + r) * ldb + k + 4 * q);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const float4 a = *reinterpret_cast<const float4*>(As + ((rb0 + i * rbs) * 16 + r) * lda + k + 4 * q);
            acc[i] = mfma_k16(a, b, acc[i]);
        }
    }
}

// acc += A[rows][k] (LDS) x B where B(k, n) = Bt[k][n] (LDS, row-major by k)
template <int NR>
__device__ __forceinline__ void mm_lds_kn(floatx4 (&acc)[NR], const float* As, int lda, int rb0, int rbs,
                                          const float* Bt, int ldb, int cb, int K, int lane) {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int k = 0; k < K; k += 16) {
        float4 b;
        b.x = Bt[(k + 4 * q + 0) * ldb + cb * 16 + r];
        b.y = Bt[(k + 4 * q + 1) * ldb + cb * 16 + r];
        b.z = Bt[(k + 4 * q + 2) * ldb + cb * 16 + r];
        b.w = Bt[(k + 4 * q + 3) * ldb + cb * 16 + r];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const float4 a = *reinterpret_cast<const float4*>(As + ((rb0 + i * rbs) * 16 + r) * lda + k + 4 * q);
            acc[i] = mfma_k16(a, b, acc[i]);
        }
    }
}

// Activation of one [32][64] tile: A = tanh(U) in LDS and (FWD) the a0 / a1
// cache rows in HBM, one float4 per thread (row-contiguous, coalesced stores).
__device__ __forceinline__ void tanh_tile(const float* U, float* A, float* cache, int64_t row_base, int64_t T,
                                          int tid) {
    constexpr int LD = 68;
    const int row = tid >> 4, c = (tid & 15) * 4;
    const float4 u = *reinterpret_cast<const float4*>(U + row * LD + c);
    const float4 v = make_float4(tanhf(u.x), tanhf(u.y), tanhf(u.z), tanhf(u.w));
    *reinterpret_cast<float4*>(A + row * LD + c) = v;
    const int64_t gr = row_base + row;
    if (cache && gr < T) *reinterpret_cast<float4*>(cache + gr * 64 + c) = v;
}

template <int MP, int KG, int MODE>
__global__ void __launch_bounds__(KT, 1) k_ks(RowArgs a, FOut o) {
    using L = KLayout<MP, KG>;
    constexpr int H = 64, BT = L::BT, NP = L::NP, KH = L::KH;
    constexpr bool GRAD = MODE != EVAL;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* XT = smem + L::oXT;
    float* D0 = smem + L::oD0;
    float* A0s = smem + L::oA0;
    float* D1 = smem + L::oD1;
    float* A1s = smem + L::oA1;
    float* GPs = smem + L::oGP;
    float* sW1 = smem + L::oW1;
    float* sdW1 = smem + L::odW1;
    float* sW2 = smem + L::oW2;
    float* sdW2 = smem + L::odW2;

    // FVP: a converged CG loop (cg_solve.py:19-20); EVAL: a TRPO trial the device line
    // search no longer needs (mjrl_policy_eval_if)
    if ((MODE == FVP || MODE == EVAL) && a.done && *a.done) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, q = lane >> 4;
    const int cb = w & 3, kh = w >> 2;
    const int m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;
    const float* P = a.P;
    const Packed pk(H, H, NP, MP);
    const float* W0src = (MODE == FVP ? a.V : P) + pk.W0;

    // ---- launch preamble: weights to LDS, this wave's W0 / dW0 slice to registers ----
    for (int i = tid; i < H * H; i += KT) {
        const int row = i / H, col = i % H;
        sW1[row * L::LD + col] = P[pk.W1 + i];
        if (MODE == FVP) sdW1[row * L::LD + col] = a.V[pk.W1 + i];
    }
    for (int i = tid; i < MP * H; i += KT) {
        const int row = i / H, col = i % H;
        sW2[row * L::LD + col] = P[pk.W2 + i];
        if (MODE == FVP) sdW2[row * L::LD + col] = a.V[pk.W2 + i];
    }
    float4 wb[KG];   // B fragments W0[cb*16 + r][kh*KH + 16g + 4q .. +3]
#pragma unroll
    for (int g = 0; g < KG; ++g)
        wb[g] = *reinterpret_cast<const float4*>(W0src + (cb * 16 + r16) * NP + kh * KH + 16 * g + 4 * q);

    // accumulators (FWD / FVP)
    floatx4 g0[KG];   // gW0[cb*16 ..][kh*KH + 16g ..]
#pragma unroll
    for (int g = 0; g < KG; ++g) g0[g] = zero4();
    floatx4 g1[2];    // gW1 tiles (nb = cb, kb = kh + 2j)
    g1[0] = zero4();
    g1[1] = zero4();
    floatx4 g2 = zero4();   // gW2 tile (nb = w>>2 < MP/16, kb = w&3)
    float b1acc = 0.f, b2acc = 0.f;
    double racc0 = 0.0, racc1 = 0.0;   // row-pass partials (FWD / EVAL), folded at the end
    const float sls = MODE == FVP ? 0.f : ls_sum(P + pk.ls, m);

    // tile-invariant per-lane constants of the epilogues
    const float bias1 = (MODE == FVP ? a.V : P)[pk.b1 + cb * 16 + r16];
    const int cbo3 = w % (MP / 16), rb3 = w / (MP / 16);
    const int col3 = cbo3 * 16 + r16;
    const float bias3 = (MODE == FVP ? a.V : P)[pk.b2 + col3];
    const float os3 = a.out_scale ? (col3 < m ? a.out_scale[col3] : 1.f) : 1.f;
    const float osh3 = a.out_shift ? (col3 < m ? a.out_shift[col3] : 0.f) : 0.f;
    float wq3 = 0.f;
    if (MODE == FVP) {
        const float sg = expf(P[pk.ls + col3]);
        wq3 = os3 * os3 * (2.f / (2.f * sg * sg + 1e-8f));
    }

    float touch = 0.f;
    __syncthreads();   // weights in LDS

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        // Per-lane indices through a zero the compiler cannot see through: every
        // lane-dependent address of the tile body is recomputed per tile (a few VALU)
        // instead of being hoisted out of the loop into live registers (it spilled).
        int opq = 0;
        asm volatile("" : "+v"(opq));
        const int ltid = tid + opq, llane = lane + opq, lr16 = r16 + opq, lq = q + opq;
        const int64_t row_base = tile * BT;
        const int nrow = (int)(T - row_base < BT ? T - row_base : BT);   // valid rows of this tile
        // ---- publish this tile's xhat (L2-warm from the previous tile's touch) ----
        asm volatile("" ::"v"(touch));
        {
            float4 xr[L::XPER];
#pragma unroll
            for (int u = 0; u < L::XPER; ++u) {
                const int idx = ltid + u * KT;
                const int row = idx / (NP / 4), c4 = idx % (NP / 4);
                const int64_t gr = row_base + row;
                xr[u] = gr < T ? *reinterpret_cast<const float4*>(a.xhat + gr * NP + c4 * 4)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < L::XPER; ++u) {
                const int idx = ltid + u * KT;
                const int row = idx / (NP / 4), c4 = idx % (NP / 4);
                *reinterpret_cast<float4*>(XT + row * L::LDX + c4 * 4) = xr[u];
            }
        }
        // FVP: cached activations for this llane's epilogue-1 / -2 elements
        float pa0[2][4], pa1[4];
        if (MODE == FVP) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int64_t gr = row_base + i * 16 + 4 * lq + rr;
                    pa0[i][rr] = (kh == 0 && gr < T) ? a.a0[gr * H + cb * 16 + lr16] : 0.f;
                }
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int64_t gr = row_base + kh * 16 + 4 * lq + rr;
                pa1[rr] = gr < T ? a.a1[gr * H + cb * 16 + lr16] : 0.f;
            }
        }
        __syncthreads();
        // pull the next tile's xhat lines into L2 (one dword per 128-B line; the
        // value is only kept alive until the next publish, 1 VGPR)
        {
            const int64_t nt = tile + gridDim.x;
            constexpr int LPR = 4 * NP / 128;   // lines per row
            if (nt < ntiles && ltid < BT * LPR) {
                const int64_t gr = nt * BT + ltid / LPR;
                if (gr < T) touch = a.xhat[gr * NP + (ltid % LPR) * 32];
            }
        }

        // ---- phase 1: partial [32 x 16] over this wave's observation half ----
        floatx4 acc1[2] = {zero4(), zero4()};
#pragma unroll
        for (int g = 0; g < KG; ++g) {
            const int k = kh * KH + 16 * g + 4 * lq;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float4 x = *reinterpret_cast<const float4*>(XT + (i * 16 + lr16) * L::LDX + k);
                acc1[i] = mfma_k16(x, wb[g], acc1[i]);
            }
            if ((g & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound the hoisting of LDS reads
        }
        // fold the two halves: kh = 1 publishes, kh = 0 finishes
        if (kh == 1) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) D0[(i * 16 + 4 * lq + rr) * L::LD + cb * 16 + lr16] = acc1[i][rr];
        }
        __syncthreads();
        if (kh == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = i * 16 + 4 * lq + rr;
                    const int col = cb * 16 + lr16;
                    const float v = acc1[i][rr] + D0[row * L::LD + col];
                    if (MODE == FVP) {
                        const float av = pa0[i][rr];
                        D0[row * L::LD + col] = (1.f - av * av) * v;
                        A0s[row * L::LD + col] = av;
                    } else {
                        D0[row * L::LD + col] = v;   // pre-activation; tanh below
                    }
                }
        }
        __syncthreads();
        if (MODE != FVP) {
            tanh_tile(D0, A0s, MODE == FWD ? a.a0 : nullptr, row_base, T, ltid);
            __syncthreads();
        }

        // ---- phase 2: [32 x 64], K = 64; wave -> (rb = kh, cb) ----
        {
            floatx4 acc[1] = {zero4()};
            if (MODE == FVP) {
                mm_lds_nk(acc, D0, L::LD, kh, 1, sW1, L::LD, cb, H, llane);
                mm_lds_nk(acc, A0s, L::LD, kh, 1, sdW1, L::LD, cb, H, llane);
            } else {
                mm_lds_nk(acc, A0s, L::LD, kh, 1, sW1, L::LD, cb, H, llane);
            }
            const int col = cb * 16 + lr16;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = kh * 16 + 4 * lq + rr;
                const float v = acc[0][rr] + bias1;
                if (MODE == FVP) {
                    const float av = pa1[rr];
                    D1[row * L::LD + col] = (1.f - av * av) * v;
                    A1s[row * L::LD + col] = av;
                } else {
                    D1[row * L::LD + col] = v;
                }
            }
        }
        __syncthreads();
        if (MODE != FVP) {
            tanh_tile(D1, A1s, MODE == FWD ? a.a1 : nullptr, row_base, T, ltid);
            __syncthreads();
        }

        // ---- phase 3: [32 x MP], K = 64; tiles (rb, cbo) over the first 2*MP/16 waves ----
        if (w < 2 * (MP / 16)) {
            floatx4 acc[1] = {zero4()};
            if (MODE == FVP) {
                mm_lds_nk(acc, D1, L::LD, rb3, 1, sW2, L::LD, cbo3, H, llane);
                mm_lds_nk(acc, A1s, L::LD, rb3, 1, sdW2, L::LD, cbo3, H, llane);
            } else {
                mm_lds_nk(acc, A1s, L::LD, rb3, 1, sW2, L::LD, cbo3, H, llane);
            }
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = rb3 * 16 + 4 * lq + rr;
                const bool valid = row < nrow;
                const float v = acc[0][rr] + bias3;
                if (MODE == FVP)
                    GPs[row * L::LDP + col3] = (col3 < m && valid) ? wq3 * v : 0.f;
                else
                    GPs[row * L::LDP + col3] = col3 < m ? v * os3 + osh3 : 0.f;
            }
        }
        __syncthreads();

        // ---- per-row pass (FWD: log-lik, caches, VPG upstream; EVAL: LR, KL) ----
        if (MODE != FVP) {
            row_pass<MODE, BT, MP, KT, false>(a, P + pk.ls, sls, row_base, GPs, L::LDP, racc0, racc1, ltid);
            __syncthreads();
        }
        if (MODE == EVAL) continue;   // forward only

        {
            // ---- phase 4: gu1 = (1 - a1^2) (g W2); wave -> (rb = kh, cb) ----
            {
                floatx4 acc[1] = {zero4()};
                mm_lds_kn(acc, GPs, L::LDP, kh, 1, sW2, L::LD, cb, MP, llane);
                const int col = cb * 16 + lr16;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = kh * 16 + 4 * lq + rr;
                    const float av = A1s[row * L::LD + col];
                    D1[row * L::LD + col] = row < nrow ? (1.f - av * av) * acc[0][rr] : 0.f;
                }
            }
            __syncthreads();
            // ---- phase 5: gu0 = (1 - a0^2) (gu1 W1) ----
            {
                floatx4 acc[1] = {zero4()};
                mm_lds_kn(acc, D1, L::LD, kh, 1, sW1, L::LD, cb, H, llane);
                const int col = cb * 16 + lr16;
                float g[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = kh * 16 + 4 * lq + rr;
                    const float av = A0s[row * L::LD + col];
                    g[rr] = row < nrow ? (1.f - av * av) * acc[0][rr] : 0.f;
                }
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) D0[(kh * 16 + 4 * lq + rr) * L::LD + col] = g[rr];
            }
            __syncthreads();
            // ---- weight gradients (registers) ----
#pragma unroll 1
            for (int t = 0; t < BT; t += 4) {
                {
                    const float gu = D0[(t + lq) * L::LD + cb * 16 + lr16];
#pragma unroll
                    for (int g = 0; g < KG; ++g) {
                        g0[g] = mfma4(gu, XT[(t + lq) * L::LDX + kh * KH + 16 * g + lr16], g0[g]);
                        if ((g & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                    }
                }
                const float gu1 = D1[(t + lq) * L::LD + cb * 16 + lr16];
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    g1[j] = mfma4(gu1, A0s[(t + lq) * L::LD + (kh + 2 * j) * 16 + lr16], g1[j]);
                if ((w >> 2) < MP / 16)
                    g2 = mfma4(GPs[(t + lq) * L::LDP + (w >> 2) * 16 + lr16], A1s[(t + lq) * L::LD + (w & 3) * 16 + lr16],
                               g2);
            }
            if (ltid < H) {
                float s = 0.f;
                for (int row = 0; row < BT; ++row) s += D1[row * L::LD + ltid];
                b1acc += s;
            } else if (ltid < H + MP) {
                float s = 0.f;
                for (int row = 0; row < BT; ++row) s += GPs[row * L::LDP + ltid - H];
                b2acc += s;
            }
        }
        __syncthreads();
    }

    const int64_t blk = blockIdx.x;
    if constexpr (GRAD) {
        // this workgroup's slab in the flat, parameter-chunk-major layout wpart[f / 64][S][64]
        // (k_gather_flat): flat parameter f in the reference order W0, b0, W1, b1, W2, b2
        // (gaussian_mlp.py:61-64); padded columns / rows are not stored
        const int nobs = o.n, mact = o.m;
        const int fb0 = H * nobs, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + mact * H;
        float* wp = o.wpart + blk * 64;
        const int64_t cs = (int64_t)gridDim.x * 64;
        auto put = [&](int f, float v) {
            MJRL_SLAB_CHECK(blk * 64 + (int64_t)(f >> 6) * cs + (f & 63), o.wcap);
            wp[(int64_t)(f >> 6) * cs + (f & 63)] = v;
        };
#pragma unroll
        for (int g = 0; g < KG; ++g)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = cb * 16 + 4 * q + rr;
                const int k = kh * KH + 16 * g + r16;
                if (k < nobs) put(n * nobs + k, g0[g][rr]);
                else if (k == nobs) put(fb0 + n, g0[g][rr]);   // the bias column: b0
            }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = cb * 16 + 4 * q + rr;
                const int k = (kh + 2 * j) * 16 + r16;
                put(fW1 + n * H + k, g1[j][rr]);
            }
        if ((w >> 2) < MP / 16) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int n = (w >> 2) * 16 + 4 * q + rr;
                const int k = (w & 3) * 16 + r16;
                if (n < mact) put(fW2 + n * H + k, g2[rr]);
            }
        }
        if (tid < H)
            put(fb1 + tid, b1acc);
        else if (tid < H + mact)
            put(fb2 + (tid - H), b2acc);
    }
    if (MODE != FVP) {
        static_assert(L::total >= 2 * KT, "row_pass_final scratch");
        __syncthreads();
        row_pass_final<MODE, MP, KT>(racc0, racc1, reinterpret_cast<double*>(smem), a.rpart, blk, tid);
    }
}

}  // namespace
