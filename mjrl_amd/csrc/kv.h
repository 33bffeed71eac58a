// kv.h — the pipelined Fisher-vector-product kernel for the MLP(64,64) policy on
// split-f16 rows (the FVP of npg_cg.py:55-74 over gaussian_mlp.py:100-110,
// 176-182), included by policy.hip after kx.h (it reuses kx.h's image helpers).
//
// Why a second FVP kernel.  k_kx<FVP> runs 8 waves (two per SIMD) through one
// 32-row tile at a time: every phase of the 64-wide middle chain is a dependent
// LDS -> scale -> MFMA -> LDS chain behind a barrier, both waves of a SIMD sit in
// the same chain, and the tile takes ~16k cycles for ~3.5k cycles of MFMA issue
// (DESIGN.md §4).  Its first-layer state (the dW0 slice and the gW0 accumulator,
// 96 + 96 VGPRs per wave over 8 waves) fills the 256-register budget of two waves
// per SIMD, so a second tile in flight did not fit.
//
// k_kv runs FOUR waves, one per SIMD, with the whole 512-entry register file per
// wave.  Wave w owns hidden block w (16 units) of EVERY layer over the full
// observation width: its dW0 rows (96 VGPRs of split B fragments) and its gW0
// rows (96 accumulators) live in registers for the launch, so the first layer
// needs no cross-wave fold.  The xhat tiles are double-buffered in LDS and two
// tiles are in flight: the first layer of tile k+1 (72 MFMAs per wave) is issued
// in the same barrier intervals as the middle chain of tile k, so the chain's
// LDS / shuffle latency runs under matrix work:
//
//   I1  publish xhat(k+1) (register prefetch -> LDS);  P2(k)  layer-1 tangent
//   I2  P3(k) output layer + gW2 sums             ||  P1(k+1) k-steps 0 .. KG/2
//   I3  P4(k) gu1 + gW1 sums                      ||  P1(k+1) k-steps KG/2 .. KG
//   I4  P5(k) gu0, P6(k) gW0 sums (xhat(k))       ||  P1(k+1) epilogue, a0/a1 images(k+1)
//
// The split-f16 arithmetic is k_kx's (common.h "fp16x3"): every operand is scaled
// by a power of two (xhat rows by xu / xc, weights per row or column per launch,
// dynamic operands per row or per (tile, unit)) and carried as hi + lo f16; a
// product is hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_f16.  The middle
// weights W1 / W2 are LDS images scaled per column (their forward products fold
// the column scale into the dynamic left operand, their backward products apply
// it per output lane); the tangent's dW1 / dW2 rows are register fragments scaled
// per row.  Weight-gradient sums over the rows of a tile contract the MFMA K over
// the "interleaved" row order of a 16 x 16 output block (lane group q holds rows
// 4q..4q+3 and 16+4q..16+4q+3), so the backward signals go from their producing
// MFMA's output registers straight into the next MFMA's A operand; the activation
// images store rows in that order (vslot).  Every sum is in a fixed order with no
// float atomics; the per-workgroup slabs use k_kx's flat layout, so
// k_gather_flat folds them unchanged.
#pragma once

namespace {

constexpr int VT = 256;   // threads per k_kv workgroup: 4 waves, one per SIMD

template <int MP, int KG>
struct VLayout {
    static constexpr int H = 64, BT = 32;
    static constexpr int NP = 32 * KG;
    static constexpr int NFB = NP / 16;              // feature blocks of the gW0 sums
    static constexpr int RBYTES = NP * 2;            // one f16 row of an xhat image (in HBM)
    static constexpr int GBYTES = BT * 256;          // one 16-chunk group of an LDS image
    static constexpr int XIMG = BT * RBYTES;         // one hi (or lo) image of a tile
    static constexpr int LD = H + 4;                 // f32 [row][LD] exchange buffers
    static constexpr int LDG = 32 + 4;               // g [row][LDG] (MP padded to 32)
    static constexpr int WIMG = 64 * 128;            // W1 image (hi or lo), bytes
    static constexpr int WIMG2 = 32 * 128;           // W2 image (32 rows)
    static constexpr int oX = 0;                     // 2 tile buffers x (hi, lo)
    static constexpr int oU = oX + 4 * XIMG;         // 2 x [64] f32 row scales (one LDS-DMA wave: 64 lanes)
    static constexpr int oW1 = oU + 2 * 64 * 4;      // W1 image, column-scaled: hi, lo
    static constexpr int oW2 = oW1 + 2 * WIMG;       // W2 image, column-scaled: hi, lo
    static constexpr int oSC = oW2 + 2 * WIMG2;      // inverse column scales s1[64], s2[64]
    static constexpr int oDA0 = oSC + 128 * 4;       // f32 [BT][LD] da0 (P1 -> P2)
    static constexpr int oDA1 = oDA0 + BT * LD * 4;  // f32 [BT][LD] da1 (P2 -> P3), then gu1 (P4 -> P5)
    static constexpr int oGP = oDA1 + BT * LD * 4;   // f32 [BT][LDG] g (P3 -> P4)
    static constexpr int oA0 = oGP + BT * LDG * 4;   // a0 image hi, lo ([unit][row slot])
    static constexpr int oA1 = oA0 + 2 * AIMG_BYTES; // a1 image hi, lo
    static constexpr int bytes = oA1 + 2 * AIMG_BYTES;
    static_assert(bytes <= 160 * 1024, "LDS");
    static_assert(NP == 384, "xhat staging: 24 LDS-DMA pieces of 1 KB per image, 12 per wave");
    static_assert(MP == 16 || MP == 32, "output layer: one k32 step");
    static_assert(2 * 4 * 64 <= BT * LD, "preamble column maxima alias DA0");
    static_assert((MP / 16) * 4 * 4 * 64 <= BT * LD * 2, "gW2 fold aliases DA0 / DA1");
};

// xhat images, group-major: [NP / 128 groups][32 rows][16 chunks of 16 bytes]; chunk
// c of row r sits in group c >> 4 at position (c & 15) ^ vswz(r) (row bits 0-2 ->
// chunk bits 1-3).  Rows are 256 bytes apart (a multiple of the 64 banks, as the
// 768-byte rows of a row-major image), so the banking is the row-major image's; one
// LDS-DMA wave instruction (1 KB) fills four rows of one group.  Conflict-free for the first layer's b128 row reads (rows r16,
// chunks 4s + q) and for the gW0 sums' transposed reads (rows 4q + tq and
// 16 + 4q + tq: bit 4 of the row does not enter, so the second set is the first
// plus 16 rows).
__device__ __forceinline__ int vswz(int row) {
    return ((row & 1) << 1) | (((row >> 1) & 1) << 2) | (((row >> 2) & 1) << 3);
}

// activation images: tile row 16i + 4g + e (g < 4, e < 4) in slot 8g + 4i + e, so
// slots 8q..8q+7 hold the interleaved rows of lane group q (one b128 read)
__device__ __forceinline__ int vslot(int row) { return ((row >> 2) & 3) * 8 + (row >> 4) * 4 + (row & 3); }

// A operand of out = A W^T from an activation image (rows rb*16 + r, features 32s + 8q..)
__device__ __forceinline__ void arow_v(const char* img, int rb, int s, int q, int r, half8& h, half8& l) {
    const int tq = r >> 2, tp = r & 3;
    const int o0 = aoff(32 * s + 8 * q + tq, 8 * tp + 4 * rb);
    const int o1 = aoff(32 * s + 8 * q + 4 + tq, 8 * tp + 4 * rb);
    h = cat_tr(ds_read_tr16(img + o0), ds_read_tr16(img + o1));
    l = cat_tr(ds_read_tr16(img + AIMG_BYTES + o0), ds_read_tr16(img + AIMG_BYTES + o1));
}

__device__ __forceinline__ void astore4_v(char* img, int f, int row0, const float (&v)[4]) {
    astore4(img, f, vslot(row0), v);
}
__device__ __forceinline__ void aval4_v(const char* img, int f, int row0, float (&v)[4]) {
    aval4(img, f, vslot(row0), v);
}

typedef _Float16 half4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx4 mfma16_x3(const half4v& ah, const half4v& al, const half4v& bh, const half4v& bl,
                                             floatx4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, c, 0, 0, 0);
}

// f32 [rows][64] (row stride 64) -> registers of the preamble: thread (w, lane) holds
// column lane of rows w + 4k (rows >= nrows read as zero)
template <int IR>
__device__ __forceinline__ void vload(const float* __restrict__ W, int nrows, float (&v)[IR], int tid) {
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int k = 0; k < IR; ++k) v[k] = w + 4 * k < nrows ? W[(w + 4 * k) * 64 + lane] : 0.f;
}

// a B-operand fragment pair of out = A W^T (n = row j of W, k = 32s + 8q..), scaled per
// row j (max over the row's 64 entries, shared by the lane groups); returns the inverse
template <int KS>
__device__ __forceinline__ float wrow_reg(const float* __restrict__ Wj, int q, half8 (&h)[KS], half8 (&l)[KS]) {
    float8v v[KS];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        v[s] = load8(Wj + 32 * s + 8 * q);
        mx = fmaxf(mx, absmax8(v[s]));
    }
    float inv;
    const float sc = pow2_scale(max_over_groups(mx), inv);
#pragma unroll
    for (int s = 0; s < KS; ++s) split8(v[s], sc, h[s], l[s]);
    return inv;
}

// Running power-of-two scale of a weight-gradient sum that the MFMA accumulates
// across tiles (the gW1 / gW2 sums: the accumulator stays in AGPRs, no per-tile
// rescale on the VALU).
// S (per lane = per A-operand row of the sum, 0 until the row's first nonzero tile)
// maps the row's running max into [2^12, 2^13); a tile whose max mx would pass 2^15
// raises it (S shrinks by a power of two and the accumulator rows are multiplied by
// the exact ratio: wave-uniform branch, taken a few times per launch).  Element error
// of the split operand: 2^-23 |y| + 2^-38 M, M the row's running max.
constexpr float RUN_LIM = 32768.f;
template <int HR>   // the power of two s with M s in [2^(HR-1), 2^HR)
__device__ __forceinline__ float pow2_at(float M) {
    int E;
    frexpf(M, &E);   // M in [2^(E-1), 2^E)
    E = E < -100 ? -100 : E;
    return ldexpf(1.f, HR - E);
}
template <int NB>
__device__ __forceinline__ void run_rescale(float& S, float mx, floatx4 (&acc)[NB], int q) {
    const bool need = mx > 0.f && mx < 3.0e38f && (S == 0.f || !(mx * S < RUN_LIM));
    if (__any(need)) {
        float r = 1.f;
        if (need) {
            const float Sn = pow2_at<13>(mx);
            r = S > 0.f ? Sn * __builtin_amdgcn_rcpf(S) : 0.f;   // exact: powers of two
            S = Sn;
        }
        float r4[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) r4[rr] = __shfl(r, 4 * q + rr, 64);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            // the scaled block re-enters the accumulator through a zero-operand MFMA
            // (D = 0 * 0 + C): every value that the accumulator chain carries is an
            // MFMA result, so the chain stays in AGPRs (a VALU definition would pull
            // all of it into VGPRs)
            floatx4 t = acc[b];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) t[rr] *= r4[rr];
            acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(0.f, 0.f, t, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}
// the inverse of a running scale for output row 4q + rr of a block (0 for an unset row)
__device__ __forceinline__ void run_inv4(float S, int q, float (&o)[4]) {
    const float iv = S > 0.f ? __builtin_amdgcn_rcpf(S) : 0.f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) o[rr] = __shfl(iv, 4 * q + rr, 64);
}

// LDS-DMA in inline asm (global_load_lds_dwordx4 / _dword, m0 = the wave-uniform LDS
// destination, lane l writes dst + l * size).  Issued through asm so that the
// compiler, which does not see these writes, does not drain them (vmcnt(0)) before
// every LDS read that follows: the waits are explicit (kernel, I2 -> I3).  Unknown
// vector-memory operations only make the compiler's own counted waits conservative.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// the saddr form: address = sbase (wave-uniform SGPR pair) + voff (per-lane 32-bit)
__device__ __forceinline__ void dma16s(const void* sbase, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void* gsrc, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

template <int MP, int KG>
__global__ void __launch_bounds__(VT, 1) k_kv(RowArgs a, FOut o) {
#pragma clang fp contract(fast)
    using L = VLayout<MP, KG>;
    constexpr int H = 64, BT = L::BT, NP = L::NP, NFB = L::NFB;
    constexpr int NCB3 = MP / 16;        // output-layer column blocks
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sb = reinterpret_cast<char*>(smem);
    if (a.done && *a.done) return;
#ifdef MJRL_KX_PROF
    // phase profile (debug builds): g_kx_prof[0..11] = the stamps below, 15 preamble +
    // prologue, 16 tail, 17 launches, 12 past-headroom gW0 tiles (wave 0, workgroup 0)
    unsigned long long kx_acc_[KX_NPROF] = {0};
    unsigned long long kx_last_ = __builtin_amdgcn_s_memtime();
    const unsigned long long kx_t0_ = kx_last_;
#endif

    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int cb = w;                                 // hidden block of this wave
    const int hcol = cb * 16 + r16;                   // the unit of this lane's output column
    const bool p3 = w < 2 * NCB3;                     // output-layer waves
    const int rb3 = w / NCB3, cbo3 = w % NCB3, col3 = cbo3 * 16 + r16;
    const int m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;
    const int64_t G = gridDim.x;
    const float* P = a.P;
    const float* V = a.V;
    const Packed pk(H, H, NP, MP);

    char* W1i = sb + L::oW1;
    char* W2i = sb + L::oW2;
    float* sc1 = reinterpret_cast<float*>(sb + L::oSC);   // inverse column scales of W1i
    float* sc2 = sc1 + 64;                                // ... of W2i
    float* DA0 = reinterpret_cast<float*>(sb + L::oDA0);
    float* DA1 = reinterpret_cast<float*>(sb + L::oDA1);  // da1, then gu1
    float* GP = reinterpret_cast<float*>(sb + L::oGP);
    char* A0i = sb + L::oA0;
    char* A1i = sb + L::oA1;
    auto XB = [&](int b) { return sb + L::oX + b * 2 * L::XIMG; };   // hi image; lo at + XIMG
    auto US = [&](int b) { return reinterpret_cast<float*>(sb + L::oU) + b * 64; };

    // ---- xhat tiles by LDS-DMA (global_load_lds_dwordx4): DMA piece jj (0..23) of an
    // image fills group jj >> 3, rows 4 (jj & 7) .. + 3; lane l the row 4 (jj & 7) +
    // (l >> 4), position l & 15, read from the row's chunk 16 (jj >> 3) + ((l & 15) ^
    // vswz(row)): the swizzle goes on the source address.  vswz depends on the row's
    // bits 0-2 = (l >> 4, jj & 1), so two per-lane source offsets serve every piece
    // (the saddr form: wave-uniform base + per-lane offset).  Wave w fills image w >> 1,
    // pieces 12 (w & 1) .. + 11.  No registers hold the tile; the DMA of tile k+1 is in
    // flight across I1 and I2.
    const int ximg = w >> 1, jj0 = 12 * (w & 1);
    unsigned xoff[2];
#pragma unroll
    for (int par = 0; par < 2; ++par)
        xoff[par] = (lane >> 4) * (4 * NP) + 16 * ((lane & 15) ^ vswz(4 * par + (lane >> 4)));
    auto xdma = [&](int64_t t_, int b_, int u0, int u1) __attribute__((always_inline)) {
        const int64_t rb_ = t_ * BT;
        const int nr = (int)(T - rb_ < BT ? T - rb_ : BT);
        if (w == 0 && u0 == 0) {   // row scales first: rows past T (and lanes 32..63) read row T - 1
            const int64_t ri = rb_ + lane < T ? rb_ + lane : T - 1;
            dma4(a.xu + ri, lds_addr(US(b_)));
        }
        const char* src = reinterpret_cast<const char*>(a.xs) + rb_ * (4 * NP) + ximg * (2 * NP);
        const unsigned dst = lds_addr(XB(b_) + ximg * L::XIMG);
        if (nr == BT) {   // wave-uniform: every tile but the batch's last
#pragma unroll
            for (int u = 0; u < 12; ++u) {
                if (u < u0 || u >= u1) continue;
                const int jj = jj0 + u, g = jj >> 3, rq = jj & 7;
                dma16s(src + 4 * rq * (4 * NP) + 256 * g, xoff[rq & 1], dst + 1024 * jj);
            }
        } else {   // the last tile: rows past T read the tile's row 0 (finite; masked)
#pragma unroll
            for (int u = 0; u < 12; ++u) {
                if (u < u0 || u >= u1) continue;
                const int jj = jj0 + u, g = jj >> 3, rq = jj & 7, row = 4 * rq + (lane >> 4);
                const int off = row < nr ? 4 * rq * (4 * NP) + (int)xoff[rq & 1] : 16 * (lane & 15);
                dma16(src + 256 * g + off, dst + 1024 * jj);
            }
        }
    };
    // cached activations of this wave's units at (rows 16i + 4q + rr, unit hcol); rows
    // past T read the tile's row 0 (finite; their output-layer weights are masked)
    float pn0[2][4], pn1[2][4];   // next tile
    auto aload = [&](int64_t t_) __attribute__((always_inline)) {
        const int64_t rb_ = t_ * BT;
        const int nr = (int)(T - rb_ < BT ? T - rb_ : BT);
        const float* b0p = a.a0 + rb_ * H + hcol;
        const float* b1p = a.a1 + rb_ * H + hcol;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = i * 16 + 4 * q + rr;
                const int o = (row < nr ? row : 0) * H;
                pn0[i][rr] = b0p[o];
                pn1[i][rr] = b1p[o];
            }
    };
    xdma(blockIdx.x, 0, 0, 12);
    aload(blockIdx.x);

    // ---- launch preamble: W1 / W2 images (column-scaled), register fragments ----
    float w1v[16], w2v[8];
    vload(P + pk.W1, H, w1v, tid);
    vload(P + pk.W2, MP, w2v, tid);   // 32 image rows; rows >= MP zero
    // this wave's dW0 rows (units hcol) over all NP features, times the rows' column
    // scales xc (powers of two: exact), split at one power-of-two scale per wave
    half8 wh[KG], wl[KG];
    float wsc;
    {
        float8v v[KG];
        float mx = 0.f;
#pragma unroll
        for (int s = 0; s < KG; ++s) {
            const int k0 = 32 * s + 8 * q;
            v[s] = load8(V + pk.W0 + hcol * NP + k0) * load8(a.xc + k0);
            mx = fmaxf(mx, absmax8(v[s]));
        }
        const float sc = pow2_scale(max_over_groups(mx), wsc);
#pragma unroll
        for (int s = 0; s < KG; ++s) split8(v[s], sc, wh[s], wl[s]);
    }
    // dW1 rows hcol (P2: n = j) and dW2 rows col3 (P3), scaled per row
    half8 d1h[2], d1l[2], d2h[2], d2l[2];
    const float isd1 = wrow_reg<2>(V + pk.W1 + hcol * H, q, d1h, d1l) * AHR_INV;
    float isd2 = 0.f;
    if (p3) isd2 = wrow_reg<2>(V + pk.W2 + col3 * H, q, d2h, d2l) * AHR_INV;
    const float db1 = V[pk.b1 + hcol];
    const float db2 = p3 ? V[pk.b2 + col3] : 0.f;
    float wq3 = 0.f;
    if (p3) {
        const float os3 = a.out_scale ? (col3 < m ? a.out_scale[col3] : 1.f) : 1.f;
        const float sg = expf(P[pk.ls + col3]);
        wq3 = os3 * os3 * (2.f / (2.f * sg * sg + 1e-8f));
    }
    {
        // column maxima of W1 / W2 through LDS (DA0 is free until the first P1 epilogue)
        float m1 = 0.f, m2 = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) m1 = fmaxf(m1, fabsf(w1v[k]));
#pragma unroll
        for (int k = 0; k < 8; ++k) m2 = fmaxf(m2, fabsf(w2v[k]));
        DA0[w * 64 + lane] = m1;
        DA0[256 + w * 64 + lane] = m2;
        if (MP == 16)
            for (int i = tid; i < BT * 16; i += VT) GP[(i >> 4) * L::LDG + 16 + (i & 15)] = 0.f;   // P4's zero K pad
        __syncthreads();
        if (tid < 128) {
            const float* red = DA0 + (tid >> 6) * 256;
            const float mx = fmaxf(fmaxf(red[lane], red[64 + lane]), fmaxf(red[128 + lane], red[192 + lane]));
            float iv;
            pow2_scale(mx, iv);
            sc1[tid] = iv;   // tid < 64: sc1[lane]; else sc2[lane]
        }
        __syncthreads();
        const float s1 = __builtin_amdgcn_rcpf(sc1[lane]), s2 = __builtin_amdgcn_rcpf(sc2[lane]);   // exact
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int j = w + 4 * k, off = woff(j, lane);
            const float y = w1v[k] * s1;
            const _Float16 h = (_Float16)y;
            *reinterpret_cast<_Float16*>(W1i + off) = h;
            *reinterpret_cast<_Float16*>(W1i + L::WIMG + off) = (_Float16)(y - (float)h);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = w + 4 * k, off = woff(j, lane);
            const float y = w2v[k] * s2;
            const _Float16 h = (_Float16)y;
            *reinterpret_cast<_Float16*>(W2i + off) = h;
            *reinterpret_cast<_Float16*>(W2i + L::WIMG2 + off) = (_Float16)(y - (float)h);
        }
    }
    // lane constants of the column scales: P1 folds W1's column scale of its unit into
    // da0, P2 folds W2's into da1; P4 / P5 apply them to their outputs
    const float f1 = sc1[hcol], f2 = sc2[hcol];
    const float fw = wsc * f1;

    // per-lane LDS offsets.  P1 row reads: row i*16 + r16, chunk 4s + q = group s >> 2,
    // position (4 (s & 3) + q) ^ vswz(r16) = 4 ((s & 3) ^ k1) + (q ^ (vswz & 3)).  P6
    // transposed reads: rows 4q + tq (+16), chunk 2 fb + (tp >> 1) = group fb >> 3,
    // position 2 ((fb & 7) ^ k6) + (tp >> 1).  Two registers each instead of 4 + 8.
    const int sw1 = vswz(r16), k1 = sw1 >> 2;
    const int p1b = r16 * 256 + 16 * (q ^ (sw1 & 3));
    const int prow = 4 * q + (r16 >> 2), k6 = vswz(prow) >> 1;
    const int p6b = prow * 256 + 16 * ((r16 >> 1) & 1) + 8 * (r16 & 1);
    auto p1off = [&](int s_) { return p1b + 64 * ((s_ & 3) ^ k1) + L::GBYTES * (s_ >> 2); };
    auto p6off = [&](int fb_) { return p6b + 32 * ((fb_ & 7) ^ k6) + L::GBYTES * (fb_ >> 3); };

    floatx4 acc1[2];
    auto p1 = [&](int b, int s0, int s1) __attribute__((always_inline)) {
        const char* xh = XB(b);
#pragma unroll
        for (int s = 0; s < KG; ++s) {
            if (s < s0 || s >= s1) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int off = p1off(s) + i * 16 * 256;   // rows i*16 + r16: same swizzle
                const half8 xh8 = *reinterpret_cast<const half8*>(xh + off);
                const half8 xl8 = *reinterpret_cast<const half8*>(xh + L::XIMG + off);
                acc1[i] = mfma_x3(xh8, xl8, wh[s], wl[s], acc1[i]);
            }
        }
    };
    // da0 = (1 - a0^2) dz0, dz0 = P1 * xu * wsc; times W1's column scale (fold for P2)
    auto p1_epi = [&](int b) __attribute__((always_inline)) {
        const float* us = US(b);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float4 u4 = *reinterpret_cast<const float4*>(us + i * 16 + 4 * q);
            const float uu[4] = {u4.x, u4.y, u4.z, u4.w};
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const float av = pn0[i][rr];
                DA0[(i * 16 + 4 * q + rr) * L::LD + hcol] = (1.f - av * av) * (acc1[i][rr] * uu[rr] * fw);
            }
        }
    };
    // the a0 / a1 images of the next tile and its activations as the current ones
    auto next_images = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            astore4_v(A0i, hcol, i * 16 + 4 * q, pn0[i]);
            astore4_v(A1i, hcol, i * 16 + 4 * q, pn1[i]);
        }
    };

    floatx4 g0[NFB];
#pragma unroll
    for (int fb = 0; fb < NFB; ++fb) g0[fb] = zero4();
    floatx4 g1[4], g2[4];
#pragma unroll
    for (int hb = 0; hb < 4; ++hb) {
        g1[hb] = zero4();
        g2[hb] = zero4();
    }
    float b1acc = 0.f, b2acc = 0.f;
    // scales of the weight-gradient sums' left operands (per lane = per A row): gW0 is
    // anchored at the unit's first nonzero tile (max -> [2^9, 2^10)); a tile that
    // reaches 2^15 at that scale runs its gW0 sums on exact-f32 MFMA instead.  gW1 /
    // gW2 keep running scales (run_rescale).
    float S0 = 0.f, S1 = 0.f, S2 = 0.f;
    bool ovf = false;   // this wave's slab entries hold gW0 sums of past-headroom tiles

    // ---- prologue: tile blockIdx.x through P1, its images, the next tile's loads ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of xhat(t0)
    __syncthreads();   // images, scales, xhat(t0)
    acc1[0] = zero4();
    acc1[1] = zero4();
    p1(0, 0, KG);
    p1_epi(0);
    next_images();
    __syncthreads();
#ifdef MJRL_KX_PROF
    kx_last_ = __builtin_amdgcn_s_memtime();
    kx_acc_[15] = kx_last_ - kx_t0_;
    kx_acc_[17] = 1;
#endif

    int b = 0;
    for (int64_t k = blockIdx.x; k < ntiles; k += G, b ^= 1) {
        const int64_t kn = k + G;
        const bool nx = kn < ntiles;
        const int64_t row_base = k * BT;
        const int nrow = (int)(T - row_base < BT ? T - row_base : BT);

        // ===== I1: the DMA of xhat(k+1) into the free buffer; P2(k): dz1 = da0 W1^T +
        // a0 dW1^T + db1, da1 = (1 - a1^2) dz1 (times W2's column scale, P3's fold) =====
        // half of the DMA of xhat(k+1) now, half between P2's row blocks (an LDS-DMA
        // piece costs the issuing wave ~150 cycles; spread, it runs in P2's LDS waits)
        if (nx) xdma(kn, b ^ 1, 0, 6);
        KX_STAMP(11);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i == 1 && nx) xdma(kn, b ^ 1, 6, 12);
            half8 ah[2], al[2];
            const float rinv = adyn<2>(DA0, L::LD, i, q, r16, nullptr, ah, al);
            floatx4 acc = zero4(), accb = zero4();
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                half8 bh, bl, xh, xl;
                wrow(W1i, L::WIMG, hcol, s, q, bh, bl);
                acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                arow_v(A0i, i, s, q, r16, xh, xl);
                accb = mfma_x3(xh, xl, d1h[s], d1l[s], accb);
            }
            float a4[4];   // a1 of this tile at (rows 16i + 4q + rr, unit hcol), from the image
            aval4_v(A1i, hcol, i * 16 + 4 * q, a4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const float ri = __shfl(rinv, 4 * q + rr, 64);
                const float v = acc[rr] * ri + accb[rr] * isd1 + db1;
                const float av = a4[rr];
                DA1[(i * 16 + 4 * q + rr) * L::LD + hcol] = (1.f - av * av) * v * f2;
            }
        }
        KX_STAMP(0);
        // the DMA stays in flight across this barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        KX_STAMP(1);

        // ===== I2: P3(k): g = wq (da1 W2^T + a1 dW2^T + db2), masked; the gW2 sums of
        // its 16 rows (K = 16, the output block's own layout) =====
        if (p3) {
            float g3[4];
            {
                half8 ah[2], al[2];
                const float rinv = adyn<2>(DA1, L::LD, rb3, q, r16, nullptr, ah, al);
                floatx4 acc = zero4(), accb = zero4();
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    half8 bh, bl, xh, xl;
                    wrow(W2i, L::WIMG2, col3, s, q, bh, bl);
                    acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                    arow_v(A1i, rb3, s, q, r16, xh, xl);
                    accb = mfma_x3(xh, xl, d2h[s], d2l[s], accb);
                }
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = rb3 * 16 + 4 * q + rr;
                    const float ri = __shfl(rinv, 4 * q + rr, 64);
                    const float v = acc[rr] * ri + accb[rr] * isd2 + db2;
                    g3[rr] = (col3 < m && row < nrow) ? wq3 * v : 0.f;
                    GP[row * L::LDG + col3] = g3[rr];
                }
            }
            b2acc += sum_over_groups((g3[0] + g3[1]) + (g3[2] + g3[3]));
            // gW2[jo][h] += sum over this row block of g[row][jo] a1[row][h] (K = 16 rows)
            run_rescale(S2, max_over_groups(fmaxf(fmaxf(fabsf(g3[0]), fabsf(g3[1])), fmaxf(fabsf(g3[2]), fabsf(g3[3])))),
                        g2, q);
            const float4 y = make_float4(g3[0] * S2, g3[1] * S2, g3[2] * S2, g3[3] * S2);
            half4v gh, gl;
            gh[0] = (_Float16)y.x; gh[1] = (_Float16)y.y; gh[2] = (_Float16)y.z; gh[3] = (_Float16)y.w;
            gl[0] = (_Float16)(y.x - (float)gh[0]);
            gl[1] = (_Float16)(y.y - (float)gh[1]);
            gl[2] = (_Float16)(y.z - (float)gh[2]);
            gl[3] = (_Float16)(y.w - (float)gh[3]);
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) {
                const int off = aoff(hb * 16 + r16, 8 * q + 4 * rb3);
                const half4v bh = *reinterpret_cast<const half4v*>(A1i + off);
                const half4v bl = *reinterpret_cast<const half4v*>(A1i + AIMG_BYTES + off);
                g2[hb] = mfma16_x3(gh, gl, bh, bl, g2[hb]);
            }
        }
        // the next tile's activations (consumed in I4); their wait is the drain below.
        // Loaded here rather than in I4: the compiler waits for every outstanding load
        // before an asm statement with a memory clobber (the DMA issue of I1)
        if (nx) aload(kn);
        KX_STAMP(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of xhat(k+1)
        __syncthreads();   // P1(k+1) reads xhat(k+1) from I3 on
        KX_STAMP(3);

        // ===== I3: P4(k): gu1 = (1 - a1^2) (g W2) (W2's column scale on the lane's unit);
        // the gW1 sums from gu1's output registers; P1(k+1) first half =====
        // P1(k+1) first half: no branch around it (past the last tile it reads a stale
        // buffer; its results are never used), so it shares P4's basic block and the
        // scheduler can issue its MFMAs into P4's LDS / shuffle latency
        acc1[0] = zero4();
        acc1[1] = zero4();
        p1(b ^ 1, 0, KG / 2);
        {
            float gu[2][4];
            half8 bh, bl;
            wcol(W2i, L::WIMG2, cb, 0, q, r16, bh, bl);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                half8 ah[1], al[1];
                const float rinv = adyn<1>(GP, L::LDG, i, q, r16, nullptr, ah, al);
                const floatx4 acc = mfma_x3(ah[0], al[0], bh, bl, zero4());
                float a4[4];
                aval4_v(A1i, hcol, i * 16 + 4 * q, a4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const float ri = __shfl(rinv, 4 * q + rr, 64);
                    const float av = a4[rr];
                    gu[i][rr] = (1.f - av * av) * (acc[rr] * ri * f2);
                    DA1[(i * 16 + 4 * q + rr) * L::LD + hcol] = gu[i][rr];
                }
            }
            KX_STAMP(4);
            // gW1[j][h] += sum_rows gu1[row][j] a0[row][h]: A = gu1^T (m = j = hcol, K =
            // the interleaved rows of lane group q), B = the a0 image (slots 8q..8q+7)
            const float8v v = {gu[0][0], gu[0][1], gu[0][2], gu[0][3], gu[1][0], gu[1][1], gu[1][2], gu[1][3]};
            b1acc += sum_over_groups(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
            run_rescale(S1, max_over_groups(absmax8(v)), g1, q);
            half8 gh, gl;
            split8(v, S1, gh, gl);
#pragma unroll
            for (int hb = 0; hb < 4; ++hb) {
                half8 ch, cl;
                acol(A0i, hb * 16 + r16, q, ch, cl);
                g1[hb] = mfma_x3(gh, gl, ch, cl, g1[hb]);
            }
        }
        KX_STAMP(5);
        __syncthreads();
        KX_STAMP(6);

        // ===== I4: P5(k): gu0 = (1 - a0^2) (gu1 W1) xu (W1's column scale on the lane's
        // unit; xu folds the rows' scale into the gW0 sums); P6(k): gW0 += gu0^T xhat;
        // P1(k+1) second half and epilogue, the a0 / a1 images of k+1, loads of k+2 =====
        p1(b ^ 1, KG / 2, KG);   // P1(k+1) second half, beside P5 (no branch around it either)
        {
            float8v v;
            {
                const float* us = US(b);
                half8 bh[2], bl[2];
#pragma unroll
                for (int s = 0; s < 2; ++s) wcol(W1i, L::WIMG, cb, s, q, r16, bh[s], bl[s]);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    half8 ah[2], al[2];
                    const float rinv = adyn<2>(DA1, L::LD, i, q, r16, nullptr, ah, al);
                    floatx4 acc = zero4();
#pragma unroll
                    for (int s = 0; s < 2; ++s) acc = mfma_x3(ah[s], al[s], bh[s], bl[s], acc);
                    const float4 u4 = *reinterpret_cast<const float4*>(us + i * 16 + 4 * q);
                    const float uu[4] = {u4.x, u4.y, u4.z, u4.w};
                    float a4[4];
                    aval4_v(A0i, hcol, i * 16 + 4 * q, a4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const float ri = __shfl(rinv, 4 * q + rr, 64);
                        const float av = a4[rr];
                        v[4 * i + rr] = (1.f - av * av) * (acc[rr] * ri * f1) * uu[rr];
                    }
                }
            }
            KX_STAMP(7);
            const float mx0 = max_over_groups(absmax8(v));
            if (S0 == 0.f && mx0 > 0.f && mx0 < 3.0e38f) S0 = pow2_at<10>(mx0);
            const char* xh = XB(b);
            const bool tovf = __any(!(mx0 * S0 < RUN_LIM));   // wave-uniform
            if (tovf) {
                // a tile past the anchor's headroom (or non-finite): its gW0 sums at a
                // per-tile scale (k_kx's), added in f32 to this workgroup's own slab
                // entries in global memory (the final write adds the accumulator to
                // them).  The accumulator chain below still runs, on a zero operand: the
                // accumulator registers see MFMAs only, on one straight path (a VALU
                // access or a branch around them pulls the 96-register chain out of the
                // AGPRs).  A runtime loop over the feature blocks: nothing in it is
                // loop-invariant enough to be hoisted out of the tile loop.
                float inv;
                const float sc = pow2_scale(mx0, inv);
                half8 gh, gl;
                split8(v, sc, gh, gl);
                float s4[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) s4[rr] = __shfl(inv, 4 * q + rr, 64);
                float* wp = o.wpart + (int64_t)blockIdx.x * 64;
                const int64_t S64 = (int64_t)gridDim.x * 64;
#pragma unroll 1
                for (int fb = 0; fb < NFB; ++fb) {
                    const int off = p6off(fb);
                    const half8 th = cat_tr(ds_read_tr16(xh + off), ds_read_tr16(xh + off + 16 * 256));
                    const half8 tl = cat_tr(ds_read_tr16(xh + L::XIMG + off), ds_read_tr16(xh + L::XIMG + off + 16 * 256));
                    const floatx4 t = mfma_x3(gh, gl, th, tl, zero4());
                    const int kf = fb * 16 + r16;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int hid = cb * 16 + 4 * q + rr;
                        const int f = kf < o.n ? hid * o.n + kf : H * o.n + hid;
                        if (kf <= o.n) {
                            float* dst = wp + (f >> 6) * S64 + (f & 63);
                            const float c = t[rr] * s4[rr];
                            *dst = ovf ? *dst + c : c;
                        }
                    }
                }
                ovf = true;
#ifdef MJRL_KX_PROF
                kx_acc_[12] += 1;
#endif
            }
            {
                half8 gh, gl;
                split8(v, tovf ? 0.f : S0, gh, gl);
#pragma unroll
                for (int fb = 0; fb < NFB; ++fb) {
                    const int off = p6off(fb);
                    const half8 th = cat_tr(ds_read_tr16(xh + off), ds_read_tr16(xh + off + 16 * 256));
                    const half8 tl = cat_tr(ds_read_tr16(xh + L::XIMG + off), ds_read_tr16(xh + L::XIMG + off + 16 * 256));
                    g0[fb] = mfma_x3(gh, gl, th, tl, g0[fb]);
                    if (fb & 1) __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        KX_STAMP(8);
        p1_epi(b ^ 1);   // past the last tile: stale values into buffers nothing reads again
        KX_STAMP(19);
        next_images();
        KX_STAMP(20);
        KX_STAMP(9);
        __syncthreads();
        KX_STAMP(10);
    }

    // ---- slabs: k_kx's flat, parameter-chunk-major layout wpart[f / 64][S][64] ----
    const int n = o.n, mm = o.m;
    const int64_t S = gridDim.x, blk = blockIdx.x;
    auto put = [&](int f, float v) { o.wpart[(((int64_t)(f >> 6)) * S + blk) * 64 + (f & 63)] = v; };
    const int fb0 = H * n, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + mm * H;
    float i0[4], i1[4], i2[4];   // inverse scales of the output rows 4q + rr
    run_inv4(S0, q, i0);
    run_inv4(S1, q, i1);
    run_inv4(S2, q, i2);
    // gW2 / gb2: the two row-block waves of an output column block fold through LDS
    float* red = DA0;                  // [NCB3][4 hb][4 rr][64 lanes] (DA0 + DA1)
    float* redb = GP;                  // [NCB3][64]
    if (p3 && rb3 == 1) {
#pragma unroll
        for (int hb = 0; hb < 4; ++hb)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) red[((cbo3 * 4 + hb) * 4 + rr) * 64 + lane] = g2[hb][rr] * i2[rr] * AHR_INV;
        redb[cbo3 * 64 + lane] = b2acc;
    }
    __syncthreads();
#pragma unroll
    for (int fb = 0; fb < NFB; ++fb) {
        const int kf = fb * 16 + r16;
        const float xck = a.xc[kf];   // the rows' column scale (exact)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int hid = cb * 16 + 4 * q + rr;
            const int f = kf < n ? hid * n + kf : fb0 + hid;   // b0 rides in the bias column
            if (kf <= n) {
                float g = g0[fb][rr] * i0[rr];
                if (ovf) g += o.wpart[(((int64_t)(f >> 6)) * S + blk) * 64 + (f & 63)];
                put(f, g * xck);
            }
        }
    }
#pragma unroll
    for (int hb = 0; hb < 4; ++hb)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
            put(fW1 + (cb * 16 + 4 * q + rr) * H + hb * 16 + r16, g1[hb][rr] * i1[rr] * AHR_INV);
    if (q == 0) put(fb1 + hcol, b1acc);
    if (p3 && rb3 == 0) {
#pragma unroll
        for (int hb = 0; hb < 4; ++hb)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int jo = cbo3 * 16 + 4 * q + rr;
                if (jo < mm)
                    put(fW2 + jo * H + hb * 16 + r16,
                        g2[hb][rr] * i2[rr] * AHR_INV + red[((cbo3 * 4 + hb) * 4 + rr) * 64 + lane]);
            }
        if (q == 0 && col3 < mm) put(fb2 + col3, b2acc + redb[cbo3 * 64 + lane]);
    }
#ifdef MJRL_KX_PROF
    kx_acc_[16] = __builtin_amdgcn_s_memtime() - kx_last_;
    if (blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < KX_NPROF; ++i) g_kx_prof[i] += kx_acc_[i];
#endif
}

}  // namespace
