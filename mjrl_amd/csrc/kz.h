// kz.h — the Fisher-vector product of the MLP(64,64) policy on split-f16 rows as a
// three-role software pipeline (included by policy.hip after kx.h, whose helpers it
// uses).  NPG.HVP, mjrl/algos/npg_cg.py:55-74, in the Gauss-Newton form of
// DESIGN.md §2; products in the split-f16 form of common.h (hi*hi + hi*lo + lo*hi
// on v_mfma_f32_16x16x32_f16, f32 accumulate), the same scaling as k_kx.
//
// Why: k_kx runs every phase of a 32-row tile on all 8 waves with a barrier
// between phases, so the 64-wide middle layers (four short dependent phases, ~58 %
// of its tile) leave the first-layer MFMAs and the HBM stream idle.  Here one
// 768-thread workgroup per CU holds three kinds of waves, one of each per SIMD:
//   waves 0-3  (P1)    the first layer du0 = dW0 xhat of the NEXT tile: wave w owns
//                      hidden blocks {2(w&1), 2(w&1)+1} over observation half w>>1
//                      (its dW0 slice in registers, 8 KG VGPRs); it reads the tile's
//                      split rows straight from global memory (L2: touched one
//                      period ahead) and writes the two half partials to D0 / D0B;
//   waves 4-7  (P6)    the gW0 sums of the PREVIOUS tile: wave 4+c owns hidden block
//                      c over all NP features (accumulators in registers, 8 KG
//                      VGPRs), reading the tile's rows from the x image with
//                      transposed LDS reads, and then refills the image with the
//                      current tile (L2 hits) for the next period;
//   waves 8-11 (chain) the 64-wide layers of the CURRENT tile: P2 (layer 1
//                      tangent), P3 (output layer), P4 (gu1) + gW2 sums, P5 (gu0) +
//                      gW1 sums, the weight images in LDS, the cached activations
//                      a0 / a1 read from global one period ahead (rows for the MFMA
//                      operands, written once into row-major images for the
//                      weight-gradient sums' transposed reads).
// A period is four barrier intervals I1..I4; in period k the chain works on tile
// t_k, P6 on t_{k-1} (I1) and the x image for t_k (I2-I4), P1 on t_{k+1} (I2-I4).
// Every exchange buffer is written and read in fixed intervals, so one copy of
// each suffices (LDS 160.4 KB); each role runs its own loop with the same four
// barriers per period, so the register allocator sees one role's live values at a
// time (P1: dW0 slice, P6: gW0 accumulators, chain: prefetched activations).
// Reductions are in fixed order; slabs in the flat layout of k_kx (k_gather_flat).
#pragma once

#ifdef MJRL_KX_PROF
// interval profile (debug builds): wave 0 of each role in workgroup 0 adds, per
// interval I1..I4, the s_memtime cycles from the interval's start to its barrier
// (work) and to the barrier's release (total); read with mjrl_debug_kz_prof
constexpr int KZ_NPROF = 3 * 8 + 4;   // [role][interval][work, total], then periods, prologue per role
__device__ unsigned long long g_kz_prof[KZ_NPROF];
#define KZ_PROF_DECL unsigned long long kza_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, kzt_ = __builtin_amdgcn_s_memtime()
#define KZ_BAR(i)                                                      \
    do {                                                               \
        __builtin_amdgcn_sched_barrier(0);                             \
        kza_[2 * (i)] += __builtin_amdgcn_s_memtime() - kzt_;          \
        __syncthreads();                                               \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();    \
        kza_[2 * (i) + 1] += n_ - kzt_;                                \
        kzt_ = n_;                                                     \
        __builtin_amdgcn_sched_barrier(0);                             \
    } while (0)
#define KZ_PROF_START() kzt_ = __builtin_amdgcn_s_memtime()
#define KZ_PROF_END(role, nper)                                                        \
    do {                                                                               \
        if (blockIdx.x == 0 && (threadIdx.x & 255) == 0) {                             \
            for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_kz_prof[(role) * 8 + i_], kza_[i_]); \
            if ((role) == 0) atomicAdd(&g_kz_prof[24], (unsigned long long)(nper));    \
        }                                                                              \
    } while (0)
#else
#define KZ_PROF_DECL
// a period's barrier; no instruction is scheduled across it (each interval keeps its work)
#define KZ_BAR(i)                          \
    do {                                   \
        __builtin_amdgcn_sched_barrier(0); \
        __syncthreads();                   \
        __builtin_amdgcn_sched_barrier(0); \
    } while (0)
#define KZ_PROF_START() \
    do {                \
    } while (0)
#define KZ_PROF_END(role, nper) \
    do {                        \
    } while (0)
#endif

namespace {

constexpr int ZT = 768;   // 12 waves

template <int MP, int KG>
struct ZLayout {
    static constexpr int H = 64, BT = 32;
    static constexpr int NP = 32 * KG, KH = NP / 2, KS = KH / 32;
    static constexpr int RBYTES = NP * 2;            // one f16 row of the x image (hi or lo)
    static constexpr int LD = H + 4, LDT = BT + 4, LDG = 32 + 4;
    static constexpr int WIMG = 64 * 128, WIMG2 = 32 * 128;
    static constexpr int AIMG = 32 * 128;            // row-major [32 rows][64] f16 activation image (hi or lo)
    static constexpr int oXH = 0;
    static constexpr int oXL = oXH + BT * RBYTES;
    static constexpr int oS1 = oXL + BT * RBYTES;    // W1c (column-scaled) hi, lo
    static constexpr int oS2 = oS1 + 2 * WIMG;       // dW1r (row-scaled)
    static constexpr int oS3 = oS2 + 2 * WIMG;       // W2c
    static constexpr int oS4 = oS3 + 2 * WIMG2;      // dW2r
    static constexpr int oSC = oS4 + 2 * WIMG2;      // inverse scales s1[64] s2[64] s3[64] s4[32]
    static constexpr int oU = oSC + (64 + 64 + 64 + 32) * 4;   // Us[2][BT]: row scales of the split rows
    static constexpr int oD0 = oU + 2 * BT * 4;      // f32 [BT][LD]: first-layer partial, observation half 0
    static constexpr int oD0B = oD0 + BT * LD * 4;   // half 1
    static constexpr int oR1 = oD0B + BT * LD * 4;   // D1 [BT][LD] (I1 -> I2) | G1T [H][LDT] (I3 -> I4)
    static constexpr int R1SZ = (BT * LD > H * LDT ? BT * LD : H * LDT) * 4;
    static constexpr int oG1 = oR1 + R1SZ;           // G1 [BT][LD] (I3 -> I4)
    static constexpr int oR3 = oG1 + BT * LD * 4;    // GPf [BT][LDG] + GPT [32][LDT] (I2 -> I3) | G0T [H][LDT] (I4 -> I1)
    static constexpr int R3SZ = ((BT * LDG + 32 * LDT) > H * LDT ? (BT * LDG + 32 * LDT) : H * LDT) * 4;
    static constexpr int oA0 = oR3 + R3SZ;           // a0 image hi, lo (row-major, woff layout)
    static constexpr int oA1 = oA0 + 2 * AIMG;       // a1 image
    static constexpr int bytes = oA1 + 2 * AIMG;
    static_assert(bytes <= 160 * 1024, "LDS");
    static_assert(NP % 128 == 0 && KS >= 1, "chunk swizzle of the x image");
    static_assert(MP == 16 || MP == 32, "output layer: one k32 step");
    static_assert(KS % 2 == 0 || KS == 1 || KS == 3, "P1 parts");
};

// A operand of an activation row (A[row][k]: lane (r16 = row, q) k = 32 s + 8 q ..) from
// f32 cached activations in global memory: rows past T read row `rclamp`
__device__ __forceinline__ float8v act_row(const float* a, int64_t row, int s, int q) {
    return load8(a + row * 64 + 32 * s + 8 * q);
}

template <int MP, int KG, int ROLES = 7>   // ROLES: a bit per role (register-pressure probes only)
__global__ void __launch_bounds__(ZT, 1) k_kz(RowArgs a, FOut o) {
#pragma clang fp contract(fast)
    using L = ZLayout<MP, KG>;
    constexpr int H = 64, BT = L::BT, NP = L::NP, KH = L::KH, KS = L::KS;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sb = reinterpret_cast<char*>(smem);
    char* XHb = sb + L::oXH;
    char* XLb = sb + L::oXL;
    char* S1 = sb + L::oS1;
    char* S2 = sb + L::oS2;
    char* S3 = sb + L::oS3;
    char* S4 = sb + L::oS4;
    float* sc1 = reinterpret_cast<float*>(sb + L::oSC);
    float* sc2 = sc1 + 64;
    float* sc3 = sc2 + 64;
    float* sc4v = sc3 + 64;
    float* Us = reinterpret_cast<float*>(sb + L::oU);
    float* D0 = reinterpret_cast<float*>(sb + L::oD0);
    float* D0B = reinterpret_cast<float*>(sb + L::oD0B);
    float* D1 = reinterpret_cast<float*>(sb + L::oR1);
    float* G1T = D1;
    float* G1 = reinterpret_cast<float*>(sb + L::oG1);
    float* GPf = reinterpret_cast<float*>(sb + L::oR3);
    float* GPT = GPf + BT * L::LDG;
    float* G0T = GPf;
    char* A0i = sb + L::oA0;
    char* A1i = sb + L::oA1;

    if (a.done && *a.done) return;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;
    const int64_t G = gridDim.x;
    // tiles of this workgroup: t_k = blockIdx.x + k G, k < N
    const int N = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int k) -> int64_t { return (int64_t)blockIdx.x + (int64_t)k * G; };
    const float* P = a.P;
    const float* V = a.V;
    const Packed pk(H, H, NP, MP);
    const char* xsb = reinterpret_cast<const char*>(a.xs);
    // a row of tile t (clamped into the batch: rows past T read a valid row, whose
    // contributions are masked to zero at the output layer, gp)
    auto crow = [&](int64_t t, int row) -> int64_t {
        const int64_t g = t * BT + row;
        return g < T ? g : (T > 0 ? T - 1 : 0);
    };

    // ---- preamble: weight images (waves 0-7), as k_kx's FVP preamble ----
    {
        float w1v[8], w3v[4];
        float8v rv1 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, rv2 = rv1;
        float* red1 = G1;           // [8][64] column-max partials (G1 is free until the first P4)
        float* red3 = G1 + 512;
        if (w < 8) {
            wload(P + pk.W1, H, w1v, tid);
            wload(P + pk.W2, MP, w3v, tid);
            rv1 = wload_rows<64>(V + pk.W1, H, tid);
            rv2 = wload_rows<32>(V + pk.W2, MP, tid);
            wrows_store<64>(rv1, S2, L::WIMG, sc2, tid);
            wrows_store<32>(rv2, S4, L::WIMG2, sc4v, tid);
            wscale<true>(w1v, sc1, red1, tid);
            wscale<true>(w3v, sc3, red3, tid);
        }
        __syncthreads();
        if (w < 8) {
            wscale_cols(sc1, red1, tid);
            wscale_cols(sc3, red3, tid);
        }
        __syncthreads();
        if (w < 8) {
            wstore<true>(w1v, S1, L::WIMG, sc1, tid);
            wstore<true>(w3v, S3, L::WIMG2, sc3, tid);
        }
    }
    // (images and scales are published by the prologue's barrier below)

    const int64_t blk = blockIdx.x;
    const int64_t S = gridDim.x;
    auto put = [&](int f, float v) {
        MJRL_SLAB_CHECK((((int64_t)(f >> 6)) * S + blk) * 64 + (f & 63), o.wcap);
        o.wpart[(((int64_t)(f >> 6)) * S + blk) * 64 + (f & 63)] = v;
    };
    const int n = o.n;
    const int fb0 = H * n, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + o.m * H;

    if (w < 4) {
        if constexpr (!(ROLES & 1)) return;
        // ================= P1: the first layer of the next tile =================
        const int hh = w & 1, kh = w >> 1;
        half8 wh[2][KS], wl[2][KS];
        float wsc[2];
#pragma unroll
        for (int j2 = 0; j2 < 2; ++j2) {
            float8v v[KS];
            float mx = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int k0 = kh * KH + 32 * s + 8 * q;
                v[s] = load8(V + pk.W0 + ((2 * hh + j2) * 16 + r16) * NP + k0) * load8(a.xc + k0);
                mx = fmaxf(mx, absmax8(v[s]));
            }
            const float sc = pow2_scale(max_over_groups(mx), wsc[j2]);
#pragma unroll
            for (int s = 0; s < KS; ++s) split8(v[s], sc, wh[j2][s], wl[j2][s]);
        }
        // (sc1 is final since the preamble's second barrier; D0 / D0B are free until the
        // chain's first P2, after the prologue barrier)
        float wsc1[2];
#pragma unroll
        for (int j2 = 0; j2 < 2; ++j2) wsc1[j2] = wsc[j2] * sc1[(2 * hh + j2) * 16 + r16];
        // the k-steps of a tile in three parts, each part's loads issued one
        // interval ahead of its MFMAs
        constexpr int NPART = KS % 3 == 0 ? 3 : (KS % 2 == 0 ? 2 : 1);
        constexpr int SPP = KS / NPART;   // k-steps per part
        half8 xh[2][SPP], xl[2][SPP];
        floatx4 acc[2][2];
        float touch[2] = {0.f, 0.f};
        int opq = 0;   // an opaque zero per period: offsets recomputed, not hoisted into live registers
        auto xload = [&](int64_t t, int part) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const char* src = xsb + crow(t, i * 16 + r16 + opq) * (4 * NP);
#pragma unroll
                for (int u = 0; u < SPP; ++u) {
                    const int k0 = kh * KH + 32 * (part * SPP + u) + 8 * q;
                    xh[i][u] = *reinterpret_cast<const half8*>(src + 2 * k0);
                    xl[i][u] = *reinterpret_cast<const half8*>(src + 2 * NP + 2 * k0);
                }
            }
        };
        auto part_mfma = [&](int part) {
#pragma unroll
            for (int u = 0; u < SPP; ++u)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j2 = 0; j2 < 2; ++j2)
                        acc[i][j2] = mfma_x3(xh[i][u], xl[i][u], wh[j2][part * SPP + u], wl[j2][part * SPP + u],
                                             acc[i][j2]);
            // the part's products stay in its interval
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2) asm volatile("" : "+v"(acc[i][j2]));
        };
        // the partials carry the W1c column scale (folded into wsc1) but not the row
        // scale xu of the split rows: the chain multiplies by it (exact, a power of two)
        auto epilogue = [&](int64_t t, int buf) {
            float* dst = kh ? D0B : D0;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        dst[(i * 16 + 4 * q + rr) * L::LD + (2 * hh + j2) * 16 + r16] = acc[i][j2][rr] * wsc1[j2];
            if (w == 0 && lane < BT) Us[buf * BT + lane] = a.xu[crow(t, lane)];
        };
        auto zero_acc = [&]() {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2) acc[i][j2] = zero4();
        };
        // one L2 touch per 128-byte line of tile t's split rows (48 KB: 384 lines over
        // the four P1 waves), kept alive in registers until the next touch
        auto touch_tile = [&](int64_t t) {
            asm volatile("" ::"v"(touch[0]), "v"(touch[1]));
#pragma unroll
            for (int v2 = 0; v2 < 2; ++v2) {
                const int line = (w * 64 + lane) + 256 * v2;   // < 512 lines; 384 used at NP = 384
                constexpr int nl = BT * 4 * NP / 128, lpr = 4 * NP / 128;
                const int ln = line < nl ? line : 0;
                touch[v2] = *reinterpret_cast<const float*>(xsb + crow(t, ln / lpr) * (4 * NP) + (ln % lpr) * 128);
            }
        };
        // prologue: tile t_0 in one go
        if (N > 0) {
            zero_acc();
#pragma unroll
            for (int part = 0; part < NPART; ++part) {
                xload(tile_of(0), part);
                part_mfma(part);
            }
            epilogue(tile_of(0), 0);
            if (N > 1) touch_tile(tile_of(1));
        }
        __syncthreads();   // prologue barrier: images, scales, t_0's first-layer partials
        KZ_PROF_DECL;
        for (int k = 0; k <= N; ++k) {
            opq = 0;
            asm volatile("" : "+v"(opq));
            const bool act = k + 1 < N;
            const int64_t tn = tile_of(k + 1);
            // I1: the first part's loads of t_{k+1} (L2: touched a period ago), the touch of t_{k+2}
            if (act) {
                zero_acc();
                xload(tn, 0);
                if (k + 2 < N) touch_tile(tile_of(k + 2));
            }
            KZ_BAR(0);
            // I2 .. I4: MFMAs of part p while part p + 1 loads; the partial to D0 / D0B in I4
            // (the chain read the previous tile's partials in I1)
#pragma unroll
            for (int iv = 0; iv < 3; ++iv) {
                if (act) {
                    if (iv < NPART) part_mfma(iv);
                    if (iv + 1 < NPART) xload(tn, iv + 1);
                    if (iv == 2) epilogue(tn, (k + 1) & 1);
                }
                KZ_BAR(iv + 1);
            }
        }
        KZ_PROF_END(0, N + 1);
        asm volatile("" ::"v"(touch[0]), "v"(touch[1]));
    } else if (w < 8) {
        if constexpr (!(ROLES & 2)) return;
        // ================= P6: the gW0 sums of the previous tile =================
        const int cb = w - 4;
        const int p6 = tid - 256;   // 0..255
        floatx4 g0[2 * KG];
#pragma unroll
        for (int g = 0; g < 2 * KG; ++g) g0[g] = zero4();
        // transposed-read offsets of group g: rows 8q + tq (+ 4 h), chunk tp/2 + 2g, half tp & 1
        const int g0row = 8 * q + (r16 >> 2);
        const int g0A = 16 * ((r16 & 3) >> 1), g0B = 16 * chunk_swz(g0row), g0C = g0row * L::RBYTES + 8 * (r16 & 1);
        // groups of the gW0 sums in I1 (the rest in I2): whole 16-chunk swizzle blocks,
        // about two thirds, so the image's first chunks can be refilled from I2 on
        constexpr int NGR = 2 * KG;
        constexpr int NG1 = NGR >= 16 ? (NGR * 2 / 3) / 8 * 8 : NGR;
        // refill of the x image with tile t: thread p6 owns row p6 >> 3, pieces (p6 & 7) + 8 u;
        // stage s = pieces u = 2 s, 2 s + 1 (chunks 16 s .. 16 s + 15) of both halves,
        // loaded in I(s + 1) and stored in I(s + 2), once the sums have read them
        constexpr int UPH = NP / 64;
        constexpr int NST = UPH / 2;
        static_assert(UPH % 2 == 0 && NST <= 3, "image refill stages");
        floatx4 xr[4];
        auto st_load = [&](int64_t t, int st) {
            const int row = p6 >> 3, c8 = p6 & 7;
            const char* src = xsb + crow(t, row) * (4 * NP);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int uu = 0; uu < 2; ++uu)
                    xr[2 * h + uu] = *reinterpret_cast<const floatx4*>(src + h * (2 * NP) + 16 * (c8 + 8 * (2 * st + uu)));
        };
        auto st_store = [&](int st, int opq) {
            const int row = p6 >> 3, c8 = (p6 & 7) + opq;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int uu = 0; uu < 2; ++uu)
                    *reinterpret_cast<floatx4*>((h ? XLb : XHb) + row * L::RBYTES +
                                                16 * ((c8 + 8 * (2 * st + uu)) ^ chunk_swz(row))) = xr[2 * h + uu];
        };
        __syncthreads();   // prologue barrier
        KZ_PROF_DECL;
        for (int k = 0; k <= N; ++k) {
            int opq = 0;   // opaque zero: offsets recomputed per use (not live registers)
            asm volatile("" : "+v"(opq));
            const int lr16 = r16 + opq, lq = q + opq;
            const bool act = k < N;
            // I1: gW0 += gu0^T x of tile t_{k-1}: its G0T operand (the previous period's P5)
            // into registers first (R3 is rewritten in I2), then the first NG1 groups
            half8 gh, gl;
            float s4[4];
            auto groups = [&](int g0_, int g1_) {
#pragma unroll
                for (int g = 0; g < NGR; ++g) {
                    if (g < g0_ || g >= g1_) continue;
                    short4v th[2], tl[2];
                    const int off = (((g0A + opq) + 32 * g) ^ g0B) + g0C;
#pragma unroll
                    for (int hq = 0; hq < 2; ++hq) {
                        th[hq] = ds_read_tr16(XHb + off + hq * 4 * L::RBYTES);
                        tl[hq] = ds_read_tr16(XLb + off + hq * 4 * L::RBYTES);
                    }
                    const floatx4 t = mfma_x3(gh, gl, cat_tr(th[0], th[1]), cat_tr(tl[0], tl[1]), zero4());
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) g0[g][rr] += t[rr] * s4[rr];
                    // the update stays in its interval (sunk past a barrier it would hold the products live)
                    asm volatile("" : "+v"(g0[g]));
                    if (g & 1) __builtin_amdgcn_sched_barrier(0);
                }
            };
            if (k >= 1) {
                gdyn(G0T, L::LDT, cb, lq, lr16, gh, gl, s4);
                groups(0, NG1);
            }
            if (act) st_load(tile_of(k), 0);
            KZ_BAR(0);
            // I2: the remaining groups; refill stage 0 stored, stage 1 loaded
            if (k >= 1) groups(NG1, NGR);
            if (act) {
                st_store(0, opq);
                if (NST > 1) st_load(tile_of(k), 1);
            }
            KZ_BAR(1);
            // I3: refill stage 1 stored, stage 2 loaded
            if (act) {
                if (NST > 1) st_store(1, opq);
                if (NST > 2) st_load(tile_of(k), 2);
            }
            KZ_BAR(2);
            // I4: refill stage 2 stored
            if (act) {
                if (NST > 2) st_store(2, opq);
            }
            KZ_BAR(3);
        }
        KZ_PROF_END(1, 0);

        // slabs: gW0 (b0 rides in the bias column n), the column scale applied (exact)
#pragma unroll
        for (int g = 0; g < 2 * KG; ++g) {
            const int kk = 16 * g + r16;
            const float xck = a.xc[kk];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int hid = cb * 16 + 4 * q + rr;
                if (kk < n)
                    put(hid * n + kk, g0[g][rr] * xck);
                else if (kk == n)
                    put(fb0 + hid, g0[g][rr] * xck);
            }
        }
    } else {
        if constexpr (!(ROLES & 4)) return;
        // ================= the chain: layers 1 and 2 of the current tile =================
        const int c = w - 8, rb = c & 1, hp = c >> 1;
        float bias1[2];
#pragma unroll
        for (int j2 = 0; j2 < 2; ++j2) bias1[j2] = V[pk.b1 + (2 * hp + j2) * 16 + r16];
        const int col3 = hp * 16 + r16;
        const bool p3 = hp < MP / 16;   // output-layer block of this wave (MP = 16: waves hp = 0)
        const float bias3 = p3 ? V[pk.b2 + col3] : 0.f;
        const float os3 = a.out_scale ? (col3 < m ? a.out_scale[col3] : 1.f) : 1.f;
        const float sg3 = expf(P[pk.ls + (p3 ? col3 : 0)]);
        const float wq3 = os3 * os3 * (2.f / (2.f * sg3 * sg3 + 1e-8f));
        floatx4 g2[2] = {zero4(), zero4()};   // gW2 block row hp, column blocks 2 rb + kk
        floatx4 g1[4] = {zero4(), zero4(), zero4(), zero4()};   // gW1 block row c
        float b1acc = 0.f, b2acc = 0.f;
        // cached activations of the tile: rows (A operands: a0 for P2 and the a0 image,
        // a1 for P3 and the a1 image) and output-layout values (rows rb 16 + 4 q + rr,
        // units (2 hp + j2) 16 + r16: pa1 for P2 / P4, pa0 for P5), each loaded in the
        // interval before its use from lines touched into L2 a period ahead
        float8v a0r[2], a1r[2];
        float pa0[2][4], pa1[2][4];
        float touch = 0.f;
        auto load_rows = [&](float8v (&ar)[2], const float* src, int64_t t, int lr16, int lq) {
            const int64_t row = crow(t, rb * 16 + lr16);
            ar[0] = act_row(src, row, 0, lq);
            ar[1] = act_row(src, row, 1, lq);
        };
        auto load_pa = [&](float (&pa)[2][4], const float* src, int64_t t, int lr16, int lq) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int64_t row = crow(t, rb * 16 + 4 * lq + rr);
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2) pa[j2][rr] = src[row * 64 + (2 * hp + j2) * 16 + lr16];
            }
        };
        // one dword per 128-byte line of tile t's a0 / a1 rows (2 x 64 lines over the chain's lanes)
        auto touch_act = [&](int64_t t) {
            asm volatile("" ::"v"(touch));
            const int idx = c * 64 + lane;
            const float* src = idx < 64 ? a.a0 : a.a1;
            const int ln = idx & 63;
            touch = (idx < 128 ? src : a.a0)[crow(t, ln >> 1) * 64 + (ln & 1) * 32];
        };
        // row-major activation images (woff layout: transposed reads by the weight-gradient sums)
        auto store_img = [&](char* img, const float8v (&ar)[2], int lr16, int lq) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                half8 h, l;
                split8(ar[s], AHR, h, l);
                const int off = woff(rb * 16 + lr16, 32 * s + 8 * lq);
                *reinterpret_cast<half8*>(img + off) = h;
                *reinterpret_cast<half8*>(img + L::AIMG + off) = l;
            }
        };
        if (N > 0) {
            load_rows(a0r, a.a0, tile_of(0), r16, q);
            load_pa(pa1, a.a1, tile_of(0), r16, q);
        }
        __syncthreads();   // prologue barrier
        KZ_PROF_DECL;
        for (int k = 0; k <= N; ++k) {
            const bool act = k < N;
            const int64_t t = tile_of(k);
            const int nrow = act ? (int)(T - t * BT < BT ? T - t * BT : BT) : 0;
            // lane indices through an opaque zero: the LDS offsets derived from them are
            // recomputed per period instead of held in registers across the loop
            int opq = 0;
            asm volatile("" : "+v"(opq));
            const int lr16 = r16 + opq, lq = q + opq;
            // ---- I1: P2, d1 = (1 - a1^2) (d0 W1^T + a0 dW1^T + db1), d0 = (D0 + D0B) xu (1 - a0^2) ----
            if (act) {
                if (k + 1 < N) touch_act(tile_of(k + 1));
                half8 ah[2], al[2], xh[2], xl[2];
                float8v dv[2];
                float mx = 0.f;
                const float us = Us[(k & 1) * BT + rb * 16 + lr16];   // the row's split-row scale (exact)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int o2 = (rb * 16 + lr16) * L::LD + 32 * s + 8 * lq;
                    dv[s] = (load8(D0 + o2) + load8(D0B + o2)) * us * (1.f - a0r[s] * a0r[s]);
                    mx = fmaxf(mx, absmax8(dv[s]));
                    split8(a0r[s], AHR, xh[s], xl[s]);
                }
                float rinv;
                const float sc = pow2_scale(max_over_groups(mx), rinv);
                float ri[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
#pragma unroll
                for (int s = 0; s < 2; ++s) split8(dv[s], sc, ah[s], al[s]);
                if (hp == 0) store_img(A0i, a0r, lr16, lq);   // the a0 image (one writer per row block)
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2) {
                    const int j = (2 * hp + j2) * 16 + lr16;
                    floatx4 acc = zero4(), accb = zero4();
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        half8 bh, bl;
                        wrow(S1, L::WIMG, j, s, lq, bh, bl);
                        acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                        wrow(S2, L::WIMG, j, s, lq, bh, bl);
                        accb = mfma_x3(xh[s], xl[s], bh, bl, accb);
                    }
                    const float dsc = sc2[j] * AHR_INV;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const float v = acc[rr] * ri[rr] + accb[rr] * dsc + bias1[j2];
                        D1[(rb * 16 + 4 * lq + rr) * L::LD + j] = (1.f - pa1[j2][rr] * pa1[j2][rr]) * v;
                    }
                }
                load_rows(a1r, a.a1, t, lr16, lq);   // for I2 (L2: touched a period ago)
            }
            KZ_BAR(0);
            // ---- I2: P3, gp = w (d1 W2^T + a1 dW2^T + db2) (masked past T and m) ----
            if (act) {
                if (p3) {
                    half8 ah[2], al[2];
                    const float rinv = adyn<2>(D1, L::LD, rb, lq, lr16, sc3, ah, al);
                    float ri[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
                    const int c3 = hp * 16 + lr16;
                    floatx4 acc = zero4(), accb = zero4();
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        half8 bh, bl, xh, xl;
                        wrow(S3, L::WIMG2, c3, s, lq, bh, bl);
                        acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                        split8(a1r[s], AHR, xh, xl);
                        wrow(S4, L::WIMG2, c3, s, lq, bh, bl);
                        accb = mfma_x3(xh, xl, bh, bl, accb);
                    }
                    const float dsc = sc4v[c3] * AHR_INV;
                    float gv[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int row = rb * 16 + 4 * lq + rr;
                        const float v = acc[rr] * ri[rr] + accb[rr] * dsc + bias3;
                        gv[rr] = (col3 < m && row < nrow) ? wq3 * v : 0.f;
                        GPf[row * L::LDG + c3] = gv[rr];
                    }
                    *reinterpret_cast<float4*>(GPT + c3 * L::LDT + rb * 16 + 4 * lq) =
                        make_float4(gv[0], gv[1], gv[2], gv[3]);
                }
                if (MP == 16 && !p3) {   // the padded k16..31 of P4's operand (R3 held G0T since I4)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) GPf[(rb * 16 + 4 * lq + rr) * L::LDG + 16 + lr16] = 0.f;
                }
                if (hp == 0) store_img(A1i, a1r, lr16, lq);
            }
            KZ_BAR(1);
            // ---- I3: P4, gu1 = (1 - a1^2) (gp W2); the gW2 / gb2 sums ----
            if (act) {
                {
                    half8 ah[1], al[1];
                    const float rinv = adyn<1>(GPf, L::LDG, rb, lq, lr16, nullptr, ah, al);
                    float ri[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
#pragma unroll
                    for (int j2 = 0; j2 < 2; ++j2) {
                        const int hb = 2 * hp + j2, hcol = hb * 16 + lr16;
                        half8 bh, bl;
                        wcol(S3, L::WIMG2, hb, 0, lq, lr16, bh, bl);
                        const floatx4 acc = mfma_x3(ah[0], al[0], bh, bl, zero4());
                        const float csc = sc3[hcol];
                        float gv[4];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int row = rb * 16 + 4 * lq + rr;
                            gv[rr] = (1.f - pa1[j2][rr] * pa1[j2][rr]) * (acc[rr] * ri[rr] * csc);
                            G1[row * L::LD + hcol] = gv[rr];
                        }
                        *reinterpret_cast<float4*>(G1T + hcol * L::LDT + rb * 16 + 4 * lq) =
                            make_float4(gv[0], gv[1], gv[2], gv[3]);
                    }
                }
                if (p3) {   // gW2[hp][2 rb + kk] += gp^T a1, gb2 on the rb = 0 waves
                    half8 gh, gl;
                    const float8v v = load8(GPT + (hp * 16 + lr16) * L::LDT + 8 * lq);
                    float inv;
                    const float sc = pow2_scale(max_over_groups(absmax8(v)), inv);
                    split8(v, sc, gh, gl);
                    float s4[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) s4[rr] = __shfl(inv * AHR_INV, 4 * lq + rr, 64);
                    if (rb == 0) b2acc += sum_over_groups(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
#pragma unroll
                    for (int kk = 0; kk < 2; ++kk) {
                        half8 bh, bl;
                        wcol(A1i, L::AIMG, 2 * rb + kk, 0, lq, lr16, bh, bl);
                        const floatx4 tt = mfma_x3(gh, gl, bh, bl, zero4());
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) g2[kk][rr] += tt[rr] * s4[rr];
                        asm volatile("" : "+v"(g2[kk]));
                    }
                }
                load_pa(pa0, a.a0, t, lr16, lq);   // for I4
            }
            KZ_BAR(2);
            // ---- I4: P5, gu0 = (1 - a0^2) (gu1 W1) xu (the row scale of the split rows);
            //      the gW1 / gb1 sums ----
            if (act) {
                {
                    half8 ah[2], al[2];
                    const float rinv = adyn<2>(G1, L::LD, rb, lq, lr16, nullptr, ah, al);
                    float ri[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
                    const float* us = Us + (k & 1) * BT;
#pragma unroll
                    for (int j2 = 0; j2 < 2; ++j2) {
                        const int hb = 2 * hp + j2, hcol = hb * 16 + lr16;
                        floatx4 acc = zero4();
#pragma unroll
                        for (int s = 0; s < 2; ++s) {
                            half8 bh, bl;
                            wcol(S1, L::WIMG, hb, s, lq, lr16, bh, bl);
                            acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                        }
                        const float csc = sc1[hcol];
                        float gv[4];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int row = rb * 16 + 4 * lq + rr;
                            gv[rr] = (1.f - pa0[j2][rr] * pa0[j2][rr]) * (acc[rr] * ri[rr] * csc) * us[row];
                        }
                        *reinterpret_cast<float4*>(G0T + hcol * L::LDT + rb * 16 + 4 * lq) =
                            make_float4(gv[0], gv[1], gv[2], gv[3]);
                    }
                }
                {   // gW1[c][kb] += gu1^T a0, gb1 (this wave's unit block c)
                    half8 gh, gl;
                    const float8v v = load8(G1T + (c * 16 + lr16) * L::LDT + 8 * lq);
                    float inv;
                    const float sc = pow2_scale(max_over_groups(absmax8(v)), inv);
                    split8(v, sc, gh, gl);
                    float s4[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) s4[rr] = __shfl(inv * AHR_INV, 4 * lq + rr, 64);
                    b1acc += sum_over_groups(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
#pragma unroll
                    for (int kb = 0; kb < 4; ++kb) {
                        half8 bh, bl;
                        wcol(A0i, L::AIMG, kb, 0, lq, lr16, bh, bl);
                        const floatx4 tt = mfma_x3(gh, gl, bh, bl, zero4());
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) g1[kb][rr] += tt[rr] * s4[rr];
                        asm volatile("" : "+v"(g1[kb]));
                    }
                }
                if (k + 1 < N) {   // the next tile's I1 operands (L2: touched in this period's I1)
                    load_rows(a0r, a.a0, tile_of(k + 1), lr16, lq);
                    load_pa(pa1, a.a1, tile_of(k + 1), lr16, lq);
                }
            }
            KZ_BAR(3);
        }
        KZ_PROF_END(2, 0);
        asm volatile("" ::"v"(touch));
        // slabs: gW2 (block hp, feature blocks 2 rb + kk), gb2
        if (p3) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int j = hp * 16 + 4 * q + rr;
                    if (j < o.m) put(fW2 + j * H + (2 * rb + kk) * 16 + r16, g2[kk][rr]);
                }
        }
        if (p3 && rb == 0 && q == 0 && col3 < o.m) put(fb2 + col3, b2acc);
        // gW1 (unit block c), gb1
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) put(fW1 + (c * 16 + 4 * q + rr) * H + kb * 16 + r16, g1[kb][rr]);
        if (q == 0) put(fb1 + c * 16 + r16, b1acc);
    }
}

}  // namespace
