// kx.h — the K-split persistent FWD / FVP / EVAL kernel for the MLP(64,64) policy
// with EVERY product on split-f16 MFMA (common.h "fp16x3": hi*hi + hi*lo + lo*hi
// on v_mfma_f32_16x16x32_f16, f32 accumulate), included by policy.hip.
//
// Same tile walk as k_ks<.., SX = true> (ks.h): one 512-thread workgroup per CU,
// 32-row tiles, the first layer K-split over the 8 waves with the W0 / dW0 slice
// and the gW0 accumulator in registers, the xhat tile as swizzled hi / lo images.
// The 64-wide layers, which k_ks keeps on exact-f32 MFMA, run here as split
// products too:
//   weights  — split once per launch into LDS images (hi, lo), each scaled by a
//              power of two per row or per column; one image serves a layer's
//              forward product (row reads) and its backward product (transposed
//              reads, ds_read_b64_tr_b16) when it is column-scaled, the column
//              scale being folded into the dynamic left operand;
//   cached activations a0 / a1 (|a| <= 1) — split at the fixed scale 2^14
//              (common.h AHR) into [feature][row] images read both ways;
//   dynamic operands (tangents, upstream gradients) — scaled by a power of two
//              per row (over the K of the product, max over the 4 lane groups)
//              or, for the weight-gradient sums, per (tile, unit) column, split
//              in registers, and unscaled on the f32 accumulator.
// Phases per tile (barriers between them): publish, first layer + fold,
// P2 (layer 1), P3 (output layer), P4 (gu1), P5 (gu0), weight-gradient sums.
#pragma once


namespace {

constexpr int AIMG_BYTES = 64 * 64;   // one [64 feature][32 row] f16 activation image

template <int MP, int KG>
struct XLayout {
    static constexpr int H = 64, BT = 32;
    static constexpr int NP = 32 * KG, KH = NP / 2;
    static constexpr int RBYTES = NP * 2;          // one f16 row of the xhat hi / lo image
    static constexpr int LD = H + 4;               // f32 [row][LD] buffers
    static constexpr int LDT = BT + 4;             // f32 transposed [unit][LDT] buffers
    static constexpr int LDG = 32 + 4;             // GPf [row][LDG] (MP padded to 32)
    static constexpr int WIMG = 64 * 128;          // one 64-row weight image (hi or lo), bytes
    static constexpr int WIMG2 = 32 * 128;         // one 32-row (output layer) weight image
    static constexpr int AIMG = AIMG_BYTES;
    // byte offsets
    static constexpr int oXH = 0;
    static constexpr int oXL = oXH + BT * RBYTES;
    static constexpr int oS1 = oXL + BT * RBYTES;  // W1c (FVP / FWD) | W1r (EVAL): hi, lo
    static constexpr int oS2 = oS1 + 2 * WIMG;     // dW1r (FVP) | W1r (FWD)
    static constexpr int oS3 = oS2 + 2 * WIMG;     // W2c (FVP / FWD) | W2r (EVAL)
    static constexpr int oS4 = oS3 + 2 * WIMG2;    // dW2r (FVP) | W2r (FWD)
    static constexpr int oSC = oS4 + 2 * WIMG2;    // f32 inverse scales: s1[64] s2[64] s3[64] s4[32]
    static constexpr int oU = oSC + (64 + 64 + 64 + 32) * 4;
    static constexpr int oD0 = oU + BT * 4;        // f32 [BT][LD]: D0 (P1 -> P2), then G1 (P4 -> P5)
    static constexpr int oD1 = oD0 + BT * LD * 4;  // f32 [BT][LD]: D1 (P2 -> P3), then G0T [H][LDT] (P5 -> P6)
    static constexpr int D1SZ = (BT * LD > H * LDT ? BT * LD : H * LDT) * 4;
    static constexpr int oGP = oD1 + D1SZ;         // f32 [BT][LDG]
    static constexpr int oGPT = oGP + BT * LDG * 4;  // f32 [32][LDT] (units x rows)
    static constexpr int oG1T = oGPT + 32 * LDT * 4; // f32 [H][LDT]
    static constexpr int oA0 = oG1T + H * LDT * 4;   // a0 image hi, lo
    static constexpr int oA1 = oA0 + 2 * AIMG;       // a1 image hi, lo
    static constexpr int oD0B = oA1 + 2 * AIMG;      // FVP: f32 [BT][LD] partial of observation half 1
    static constexpr int bytes = oD0B + BT * LD * 4;
    static_assert(bytes <= 160 * 1024, "LDS");
    static_assert(bytes >= 2 * KT * 8, "row_pass_final scratch");
    static constexpr int XPER = BT * NP / 4 / KT;
    static_assert(NP % 128 == 0, "chunk swizzle of the xhat images");
    static_assert(MP == 16 || MP == 32, "output layer: one k32 step");
};

// 128-byte-row f16 images (weights [row][64]) and 64-byte-row images
// (activations [feature][32 rows]): XOR swizzles of the 16-byte chunks under which
// the b128 row reads and the transposed reads of each image are bank-conflict
// free (tools/swizzle_search.py).
__device__ __forceinline__ int swz128(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int woff(int row, int col) { return row * 128 + 16 * ((col >> 3) ^ swz128(row)) + 2 * (col & 7); }
__device__ __forceinline__ int aoff(int f, int row) { return f * 64 + 16 * ((row >> 3) ^ (((f >> 3) & 1) << 1)) + 2 * (row & 7); }

// max over the 16 lanes of a DPP row (lanes 16 r .. 16 r + 15), in every lane of
// the row: quad_perm [1, 0, 3, 2], quad_perm [2, 3, 0, 1], row_half_mirror,
// row_mirror (VALU only, where __shfl_xor is an LDS-queue ds_bpermute per step)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    return fmaxf(v, dpp_f<0x140>(v));
}

__device__ __forceinline__ half8 cat_tr(const short4v& a, const short4v& b) {
    return __builtin_bit_cast(half8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// B operand of out = A W^T from a weight image: lane (j = jb*16 + r, k = 32 s + 8 q ..)
__device__ __forceinline__ void wrow(const char* img, int imgbytes, int j, int s, int q, half8& h, half8& l) {
    const int off = woff(j, 32 * s + 8 * q);
    h = *reinterpret_cast<const half8*>(img + off);
    l = *reinterpret_cast<const half8*>(img + imgbytes + off);
}
// B operand of out = A W from a weight image (B[k = j][n = h] = W[j][h]): transposed reads
__device__ __forceinline__ void wcol(const char* img, int imgbytes, int hb, int s, int q, int r, half8& h, half8& l) {
    const int tq = r >> 2, tp = r & 3;
    const int o0 = woff(32 * s + 8 * q + tq, hb * 16 + 4 * tp);
    const int o1 = woff(32 * s + 8 * q + 4 + tq, hb * 16 + 4 * tp);
    h = cat_tr(ds_read_tr16(img + o0), ds_read_tr16(img + o1));
    l = cat_tr(ds_read_tr16(img + imgbytes + o0), ds_read_tr16(img + imgbytes + o1));
}
// A operand of out = A W^T from an activation image [feature][row] (rows rb*16 + r)
__device__ __forceinline__ void arow(const char* img, int rb, int s, int q, int r, half8& h, half8& l) {
    const int tq = r >> 2, tp = r & 3;
    const int o0 = aoff(32 * s + 8 * q + tq, rb * 16 + 4 * tp);
    const int o1 = aoff(32 * s + 8 * q + 4 + tq, rb * 16 + 4 * tp);
    h = cat_tr(ds_read_tr16(img + o0), ds_read_tr16(img + o1));
    l = cat_tr(ds_read_tr16(img + AIMG_BYTES + o0), ds_read_tr16(img + AIMG_BYTES + o1));
}
// B operand of a weight-gradient sum (B[k = row][n = feature]) from an activation image
__device__ __forceinline__ void acol(const char* img, int f, int q, half8& h, half8& l) {
    const int off = aoff(f, 8 * q);
    h = *reinterpret_cast<const half8*>(img + off);
    l = *reinterpret_cast<const half8*>(img + AIMG_BYTES + off);
}
// Activation images hold a * AHR (common.h: the 2^14 headroom of every split
// block); aval4 returns a itself, MFMA consumers fold AHR_INV into their scales.
// a at (feature f, rows row0 .. row0 + 3), row0 % 4 == 0: one 8-byte read each of hi and lo
__device__ __forceinline__ void aval4(const char* img, int f, int row0, float (&v)[4]) {
    typedef unsigned uint2v __attribute__((ext_vector_type(2)));
    const int off = aoff(f, row0);
    const uint2v h = *reinterpret_cast<const uint2v*>(img + off);
    const uint2v l = *reinterpret_cast<const uint2v*>(img + AIMG_BYTES + off);
    v[0] = mix_add_lo(h[0], l[0]) * AHR_INV;
    v[1] = mix_add_hi(h[0], l[0]) * AHR_INV;
    v[2] = mix_add_lo(h[1], l[1]) * AHR_INV;
    v[3] = mix_add_hi(h[1], l[1]) * AHR_INV;
}
// store 4 consecutive rows (row0..row0+3, row0 % 4 == 0) of feature f into an activation image
__device__ __forceinline__ void astore4(char* img, int f, int row0, const float (&a)[4]) {
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
    typedef unsigned uint2v __attribute__((ext_vector_type(2)));
    typedef float float4v __attribute__((ext_vector_type(4)));
    const float v[4] = {a[0] * AHR, a[1] * AHR, a[2] * AHR, a[3] * AHR};
    const float4v x = {v[0], v[1], v[2], v[3]};
    const half4 h = __builtin_convertvector(x, half4);
    const uint2v hb = __builtin_bit_cast(uint2v, h);
    const uint2v lb = {mix_lo2(hb[0], v[0], v[1]), mix_lo2(hb[1], v[2], v[3])};
    const int off = aoff(f, row0);
    *reinterpret_cast<uint2v*>(img + off) = hb;
    *reinterpret_cast<uint2v*>(img + AIMG_BYTES + off) = lb;
}

// Dynamic left operand from an f32 [row][ld] buffer: rows rb*16 + r, K = 32*KS
// columns, optionally times fold[k] (a column scale of the right operand);
// scaled per row (power of two over the row's K), split.  Returns the row's
// inverse scale (same in all four lane groups).
template <int KS>
__device__ __forceinline__ float adyn(const float* buf, int ld, int rb, int q, int r, const float* fold,
                                      half8 (&h)[KS], half8 (&l)[KS]) {
    float8v v[KS];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        v[s] = load8(buf + (rb * 16 + r) * ld + 32 * s + 8 * q);
        if (fold) v[s] *= load8(fold + 32 * s + 8 * q);
        mx = fmaxf(mx, absmax8(v[s]));
    }
    float inv;
    const float sc = pow2_scale(max_over_groups(mx), inv);
#pragma unroll
    for (int s = 0; s < KS; ++s) split8(v[s], sc, h[s], l[s]);
    return inv;
}

// Dynamic left operand of a weight-gradient sum from a transposed f32 [unit][LDT]
// buffer: unit u = ub*16 + r, rows 8q..8q+7; scaled per (tile, unit); returns in
// sc4[rr] the inverse scale of output row (unit) 4q + rr of the block.
__device__ __forceinline__ void gdyn(const float* bufT, int ldt, int ub, int q, int r, half8& h, half8& l,
                                     float (&sc4)[4]) {
    const float8v v = load8(bufT + (ub * 16 + r) * ldt + 8 * q);
    float inv;
    const float s = pow2_scale(max_over_groups(absmax8(v)), inv);
    split8(v, s, h, l);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) sc4[rr] = __shfl(inv, 4 * q + rr, 64);
}

// Split a [rows][64] f32 weight matrix (global, row-major, row stride 64) into an
// LDS image pair scaled per row (COLS = false) or per column (COLS = true);
// inverse scales to inv[].  Three steps, so that a launch issues the loads of all
// its images before it waits on any: wload (thread = column lane, rows w + 8k;
// rows >= nrows read as zero), wscale (row maxima by wave shuffles, column maxima
// through red[8][64] in LDS) and wstore.  IR = image rows / 8.
template <int IR>
__device__ __forceinline__ void wload(const float* __restrict__ W, int nrows, float (&v)[IR], int tid) {
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int k = 0; k < IR; ++k) {
        const int j = w + 8 * k;
        v[k] = j < nrows ? W[j * 64 + lane] : 0.f;
    }
}

template <bool COLS, int IR>
__device__ __forceinline__ void wscale(const float (&v)[IR], float* inv, float* red, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    if (COLS) {
        float mx = 0.f;
#pragma unroll
        for (int k = 0; k < IR; ++k) mx = fmaxf(mx, fabsf(v[k]));
        red[w * 64 + lane] = mx;
    } else {
#pragma unroll
        for (int k = 0; k < IR; ++k) {
            float mx = fabsf(v[k]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
            float iv;
            pow2_scale(mx, iv);
            if (lane == 0) inv[w + 8 * k] = iv;
        }
    }
}

// COLS images: the column maxima in red[] -> inv[] (wave 0, after a barrier)
__device__ __forceinline__ void wscale_cols(float* inv, const float* red, int tid) {
    if (tid < 64) {
        float mx = 0.f;
#pragma unroll
        for (int i = 0; i < KT / 64; ++i) mx = fmaxf(mx, red[i * 64 + tid]);
        float iv;
        pow2_scale(mx, iv);
        inv[tid] = iv;
    }
}

// Row-scaled images, one 16-byte chunk per thread: thread t owns image row t >> 3
// and its columns 8 (t & 7) .. + 7, so a row's maximum is a 3-step shuffle over 8
// neighbouring lanes (the per-column lane mapping of wload needed a 6-step wave
// reduction per row, 12 rows per wave in one serial chain: most of the launch
// preamble), and each thread stores one swizzled 16-byte hi / lo chunk.  Rows >=
// nrows (and threads past the image) read as zero.  NR = image rows (64 or 32).
template <int NR>
__device__ __forceinline__ float8v wload_rows(const float* __restrict__ W, int nrows, int tid) {
    const int j = tid >> 3;
    float8v v = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (j < NR && j < nrows) v = load8(W + j * 64 + 8 * (tid & 7));
    return v;
}
// split row j's chunk into the image at the row's power-of-two scale; its inverse
// to inv[j] (lane 0 of the row's 8)
template <int NR>
__device__ __forceinline__ void wrows_store(const float8v& v, char* img, int imgbytes, float* inv, int tid) {
    float mx = absmax8(v);
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    const int j = tid >> 3;
    if (j < NR) {
        float iv;
        const float sc = pow2_scale(mx, iv);
        half8 h, l;
        split8(v, sc, h, l);   // the bits of wstore's v / inv -> (hi, f16(y - hi)): sc = 1 / iv exactly
        const int off = j * 128 + 16 * ((tid & 7) ^ swz128(j));
        *reinterpret_cast<half8*>(img + off) = h;
        *reinterpret_cast<half8*>(img + imgbytes + off) = l;
        if ((tid & 7) == 0) inv[j] = iv;
    }
}

template <bool COLS, int IR>
__device__ __forceinline__ void wstore(const float (&v)[IR], char* img, int imgbytes, const float* inv, int tid) {
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int k = 0; k < IR; ++k) {
        const int j = w + 8 * k;
        const float y = v[k] * __builtin_amdgcn_rcpf(inv[COLS ? lane : j]);   // exact: inv is a power of two
        const _Float16 h = (_Float16)y;
        const int off = woff(j, lane);
        *reinterpret_cast<_Float16*>(img + off) = h;
        *reinterpret_cast<_Float16*>(img + imgbytes + off) = (_Float16)(y - (float)h);
    }
}

#ifdef MJRL_KX_ABL_NOCHAIN
constexpr bool KX_ABL_NOCHAIN = true;    // timing ablation only: the FVP's P2-P5 skipped (barriers kept)
#else
constexpr bool KX_ABL_NOCHAIN = false;
#endif
#ifdef MJRL_KX_ABL_NOCOLS
constexpr bool KX_ABL_NOCOLS = true;     // timing ablation only: the FVP preamble's column scales not computed
#else
constexpr bool KX_ABL_NOCOLS = false;
#endif

// PACK (FWD only): the batch assembly (k_pack_split_q, a5) fused into the forward
// pass: the tile's f32 observation rows are loaded instead of split rows and split
// in the publish, with the pack's own f32 operations (bit-identical rows), which
// also writes them to a.xs_w / a.xu_w for the FVP and EVAL passes.  The identity
// input normalisation only (the policy's default; the division of a given
// in_shift / in_scale spilled 115 registers here, so those batches keep the
// separate pack); n_obs % 4 == 0 and 16-byte-aligned rows (mjrl_vpg_accumulate_pack
// checks).
template <int MP, int KG, int MODE, bool PACK = false>
__global__ void __launch_bounds__(KT, 1) k_kx(RowArgs a, FOut o) {
    // multiply-add chains in this kernel contract to FMA (the reference-order
    // elementwise code lives in other kernels; -ffp-contract=off is the file default)
#pragma clang fp contract(fast)
    using L = XLayout<MP, KG>;
    constexpr int H = 64, BT = L::BT, NP = L::NP, KH = L::KH;
    constexpr bool GRAD = MODE != EVAL;
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
    float* D0 = reinterpret_cast<float*>(sb + L::oD0);    // D0 (FVP: half-0 partial), then G1
    float* D0B = reinterpret_cast<float*>(sb + L::oD0B);  // FVP: half-1 partial
    float* D1 = reinterpret_cast<float*>(sb + L::oD1);    // D1, then G0T
    float* GPf = reinterpret_cast<float*>(sb + L::oGP);
    float* GPT = reinterpret_cast<float*>(sb + L::oGPT);
    float* G1T = reinterpret_cast<float*>(sb + L::oG1T);
    char* A0i = sb + L::oA0;
    char* A1i = sb + L::oA1;

#ifdef MJRL_KX_PROF
    const unsigned long long kx_t0_ = __builtin_amdgcn_s_memtime();
    unsigned long long kx_pre_[6];
#endif
    // the wave index in an SGPR (readfirstlane): cb / kh and every address term and
    // branch condition derived from them are scalar, not per-lane VALU work and
    // exec-mask branches
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int cb = w & 3, kh = w >> 2;
    const int m = a.m;
    const int64_t T = a.T;
    const int64_t ntiles = (T + BT - 1) / BT;
    const float* P = a.P;
    const Packed pk(H, H, NP, MP);
    const float* W0src = (MODE == FVP ? a.V : P) + pk.W0;


    // ---- launch preamble: weight images, this wave's W0 / dW0 slice to registers ----
    // every global load of the preamble is issued before the first wait
    constexpr int KS = KH / 32;   // k32 steps per observation half
    static_assert(KT == 512 && MP <= 32, "preamble layout: 8 waves, output-layer images of 32 rows");
    // column-scaled images (FVP / FWD: W1c, W2c) with the per-column lane mapping;
    // row-scaled images (FVP: dW1r / dW2r, FWD: W1r / W2r, EVAL: W1r / W2r) one
    // 16-byte chunk per thread (wload_rows)
    float w1v[8], w3v[4];
    float8v rv1, rv2;
    if (MODE == EVAL) {
        rv1 = wload_rows<64>(P + pk.W1, H, tid);
        rv2 = wload_rows<32>(P + pk.W2, MP, tid);
    } else {
        wload(P + pk.W1, H, w1v, tid);
        wload(P + pk.W2, MP, w3v, tid);
        const float* src = MODE == FVP ? a.V : P;   // FVP: dW1r / dW2r;  FWD: W1r / W2r
        rv1 = wload_rows<64>(src + pk.W1, H, tid);
        rv2 = wload_rows<32>(src + pk.W2, MP, tid);
    }
    const float* BV = MODE == FVP ? a.V : P;
    const float bias1 = BV[pk.b1 + cb * 16 + r16];
    const int cbo3 = w & (MP / 16 - 1), rb3 = w / (MP / 16);   // P3: waves < 2 * MP/16
    const int col3 = cbo3 * 16 + r16;
    const float bias3 = BV[pk.b2 + col3];
    const float os3 = a.out_scale ? (col3 < m ? a.out_scale[col3] : 1.f) : 1.f;
    const float osh3 = a.out_shift ? (col3 < m ? a.out_shift[col3] : 0.f) : 0.f;
    float wq3 = 0.f;
    if (MODE == FVP) {
        const float sg = expf(P[pk.ls + col3]);
        wq3 = os3 * os3 * (2.f / (2.f * sg * sg + 1e-8f));
    }
    const float sls = MODE == FVP ? 0.f : ls_sum(P + pk.ls, m);
    RowConst rconst{};
    if constexpr (MODE != FVP) rconst = row_const<MODE, MP>(a, P + pk.ls, tid);
    KX_PRE(0);
    half8 wh[KS], wl[KS];
    float wsc;
    {
        // W0 xc: the split rows carry xhat / (xc xu) (common.h col_scale), so the slice
        // takes the column scales (exact: powers of two)
        float8v v[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k0 = kh * KH + 32 * s + 8 * q;
            v[s] = load8(W0src + (cb * 16 + r16) * NP + k0) * load8(a.xc + k0);
        }
        float mx = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) mx = fmaxf(mx, absmax8(v[s]));
        const float sc = pow2_scale(max_over_groups(mx), wsc);
#pragma unroll
        for (int s = 0; s < KS; ++s) split8(v[s], sc, wh[s], wl[s]);
    }
    KX_PRE(1);
    {
        float* red1 = D0;          // [8][64] column-max partials (D0 / D0B are free until P1)
        float* red3 = D0 + 512;
        // the row-scaled images first: their scales need no barrier
        if (MODE == EVAL) {
            wrows_store<64>(rv1, S1, L::WIMG, sc1, tid);
            wrows_store<32>(rv2, S3, L::WIMG2, sc3, tid);
        } else {
            wrows_store<64>(rv1, S2, L::WIMG, sc2, tid);
            wrows_store<32>(rv2, S4, L::WIMG2, sc4v, tid);
            if (!(KX_ABL_NOCOLS && MODE == FVP)) {
                wscale<true>(w1v, sc1, red1, tid);
                wscale<true>(w3v, sc3, red3, tid);
            }
        }
        KX_PRE(2);
        if (MODE != EVAL && !(KX_ABL_NOCOLS && MODE == FVP)) {
            __syncthreads();
            wscale_cols(sc1, red1, tid);
            wscale_cols(sc3, red3, tid);
            __syncthreads();
        }
        KX_PRE(3);
        if (MODE != EVAL) {
            wstore<true>(w1v, S1, L::WIMG, sc1, tid);
            wstore<true>(w3v, S3, L::WIMG2, sc3, tid);
        }
    }
    KX_PRE(4);
    // PACK: 1 / xc of every column (exact: powers of two) in LDS (the D0B region,
    // FVP-only), read by the tile publish
    float* picx = D0B;
    if constexpr (PACK) {
        static_assert(MODE == FWD, "the fused pack is the forward pass's");
        static_assert(NP * 4 <= L::BT * L::LD * 4, "pack table in the D0B region");
        for (int k = tid; k < NP; k += KT) picx[k] = 1.f / a.xc[k];
    }
    // a converged CG loop (cg_solve.py:19-20): checked once the preamble's loads have
    // been consumed (image stores, W0 slice split), so the flag's load overlaps them
    // FVP: a converged CG loop (cg_solve.py:19-20); EVAL: a TRPO trial the device line
    // search no longer needs (mjrl_policy_eval_if)
    if ((MODE == FVP || MODE == EVAL) && a.done && *a.done) return;

    floatx4 g0[KG];
#pragma unroll
    for (int g = 0; g < KG; ++g) g0[g] = zero4();
    floatx4 g1[2] = {zero4(), zero4()};   // gW1 blocks (jb = cb, kb = kh + 2j)
    floatx4 g2 = zero4();                 // gW2 block (jb = w >> 2 < MP/16, kb = w & 3)
    float b1acc = 0.f, b2acc = 0.f;
    double racc0 = 0.0, racc1 = 0.0;


    float touch[2] = {0.f, 0.f};
    // the xhat tile is software-pipelined through registers: tile t+1's pieces are
    // loaded at the start of tile t's weight-gradient phase and stored to the
    // images at the top of the next iteration (16 threads per row, piece c = tid %
    // 16 + 16 u: u < NP/128 hi chunks, the rest lo chunks)
    float4 xn[L::XPER];
    float un = 1.f;
    // pieces u0 .. u1 - 1 (callers split the loads over two phases so the vector
    // memory issue of the 48 KB tile does not stall one phase).  The vector-memory
    // counter is in order, so a load under a branch makes the compiler's wait for
    // any EARLIER load conservative (vmcnt(0)-like): the loads whose values are
    // waited for inside a tile (the FVP's cached activations, EVAL's row-pass
    // inputs, the L2 touch) are unconditional from clamped addresses, and the
    // conditional xhat loads of the next tile come before them (EVAL) or after
    // their last use (FWD / FVP: P4 / P5); a rejected variant with unconditional
    // xhat loads made the compiler copy them between registers right after issue,
    // waiting on HBM there.
    auto xload = [&](int64_t t_, int tid_, int u0 = 0, int u1 = L::XPER) {
        const int64_t rb_ = t_ * BT;
        const int row = tid_ >> 4, c16 = tid_ & 15;
        const bool ok = t_ < ntiles && rb_ + row < T;
        if constexpr (PACK) {
            // the f32 row's columns 8 ch .. 8 ch + 7 of the thread's chunks ch = c16 + 16 c
            // (c < UH): pieces 2c, 2c + 1 (columns >= n_obs read as zero; n_obs % 4 == 0)
            const float* src = a.obs32 + (ok ? (rb_ + row) * (int64_t)a.n_obs : 0);
#pragma unroll
            for (int u = 0; u < L::XPER; ++u)
                if (u >= u0 && u < u1) {
                    const int col = 8 * (c16 + 16 * (u >> 1)) + 4 * (u & 1);
                    xn[u] = ok && col < a.n_obs ? *reinterpret_cast<const float4*>(src + col)
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            return;
        }
        const char* src = reinterpret_cast<const char*>(a.xs) + (ok ? (rb_ + row) * (4 * NP) : 0);
#pragma unroll
        for (int u = 0; u < L::XPER; ++u)
            if (u >= u0 && u < u1)
                xn[u] = ok ? *reinterpret_cast<const float4*>(src + 16 * (c16 + 16 * u)) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (u0 == 0) {
            // rows past T take row 0's scale (finite; their xhat and gradient rows are
            // zero), without a select whose wait the compiler would hoist
            const bool uok = tid_ < BT && t_ < ntiles && rb_ + tid_ < T;
            un = a.xu[uok ? rb_ + tid_ : 0];
        }
    };
    xload(blockIdx.x, tid);
    __syncthreads();   // images and scales ready
#ifdef MJRL_KX_PROF
    unsigned long long kx_acc_[KX_NPROF] = {0};
    unsigned long long kx_last_ = __builtin_amdgcn_s_memtime();
    kx_acc_[15] = kx_last_ - kx_t0_;
    kx_acc_[17] = 1;
    kx_acc_[18] = kx_pre_[0] - kx_t0_;
    for (int i = 1; i < 5; ++i) kx_acc_[18 + i] = kx_pre_[i] - kx_pre_[i - 1];
    kx_acc_[23] = kx_last_ - kx_pre_[4];
#endif

    // FVP: P1's partials carry the W1c column scale of their unit (both powers of two:
    // exact), so P2 folds them without it
    const float wsc1 = MODE == FVP ? wsc * sc1[cb * 16 + r16] : wsc;
    // P1's xhat-image offsets (row r16, chunk kh*KH/8 + 4s + q, swizzled): tile-invariant,
    // kept in KS registers instead of being recomputed per tile
#ifndef MJRL_KX_OFFREG
    // computed per use from three per-lane values (2 VALU each: add, xor-add) instead of
    // KS + KG live offsets: the FVP's register file then has no spills, whose scratch
    // reloads waited in order (vmcnt) on the next tile's HBM prefetch loads
    const int p1A = 16 * (kh * (KH / 8) + q), p1B = 16 * chunk_swz(r16), p1C = r16 * L::RBYTES;
    auto p1off_at = [&](int s, int opq_) { return (((p1A + opq_) + 64 * s) ^ p1B) + p1C; };
#else
    int p1off[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) p1off[s] = r16 * L::RBYTES + 16 * ((kh * (KH / 8) + 4 * s + q) ^ chunk_swz(r16));
    auto p1off_at = [&](int s, int) { return p1off[s]; };
#endif
    // and the transposed-read offsets of the gW0 sums (group g: rows 8q + tq, chunk
    // kh*KH/8 + tp/2 + 2g, half tp & 1), kept in registers (FWD / FVP)
    auto gw0_off = [&](int r_, int q_, int g) {
        const int tq = r_ >> 2, tp = r_ & 3, row = 8 * q_ + tq;
        return row * L::RBYTES + 16 * (((kh * KH) / 8 + (tp >> 1) + 2 * g) ^ chunk_swz(row)) + 8 * (tp & 1);
    };
#ifndef MJRL_KX_OFFREG
    // gw0_off(r16, q, g) = ((g0A + 32 g) ^ g0B) + g0C (the chunk term 16 ((kh KH/8 + tp/2 +
    // 2g) ^ swz) with the row's swizzle bits 1-3 and the half / row terms added after)
    const int g0row = 8 * q + (r16 >> 2);
    const int g0A = 16 * ((kh * KH) / 8 + ((r16 & 3) >> 1)), g0B = 16 * chunk_swz(g0row),
              g0C = g0row * L::RBYTES + 8 * (r16 & 1);
    auto g0off_at = [&](int g, int opq_) { return (((g0A + opq_) + 32 * g) ^ g0B) + g0C; };
#else
    int g0off[MODE != EVAL ? KG : 1];
    if constexpr (MODE != EVAL) {
#pragma unroll
        for (int g = 0; g < KG; ++g) g0off[g] = gw0_off(r16, q, g);
    }
    auto g0off_at = [&](int g, int) { return g0off[g]; };
#endif
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        KX_STAMP(9);   // loop top (the wait on the previous tile's last barrier)
        // per-lane indices through an opaque zero: recomputed per tile rather than
        // hoisted into live registers (see ks.h)
        // (FVP keeps its lane indices r16 / q in registers at the cost of 8 spilled
        // VGPRs: 220 fewer VALU per tile, FVP 896 -> 867 us in rocprofv3; FWD
        // spills 19 that way and is 5 % slower, so it recomputes them; EVAL has the
        // registers to keep all three; profiles/r02s/ab_lane_index.txt)
        int opq = 0;
        if constexpr (MODE != EVAL) asm volatile("" : "+v"(opq));
        constexpr int OPQ_LANE = MODE == FWD ? 1 : 0;
        const int ltid = tid + opq, lr16 = r16 + OPQ_LANE * opq, lq = q + OPQ_LANE * opq;
        const int64_t row_base = tile * BT;
        const int nrow = (int)(T - row_base < BT ? T - row_base : BT);

        // ---- publish: xhat tile -> images, row scales; FVP: cached activations ----
        asm volatile("" ::"v"(touch[0]), "v"(touch[1]));
        if constexpr (PACK) {
            // the pack (k_pack_split_q) of this thread's 24 columns of its row: the bias
            // column 1 -> / xc; the row's power-of-two scale over its 16 lanes; hi / lo to
            // the images and to the split rows in HBM
#pragma clang fp contract(off)
            constexpr int UH = NP / 128;
            const int row = ltid >> 4, c16 = ltid & 15;
            const bool ok = row < nrow;
            float8v v[UH];
            float mx = 0.f;
#pragma unroll
            for (int c = 0; c < UH; ++c) {
                const int c0 = 8 * (c16 + 16 * c);
                v[c] = float8v{xn[2 * c].x, xn[2 * c].y, xn[2 * c].z, xn[2 * c].w,
                               xn[2 * c + 1].x, xn[2 * c + 1].y, xn[2 * c + 1].z, xn[2 * c + 1].w};
                const float8v ic = load8(picx + c0);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if (c0 + e == a.n_obs && ok) v[c][e] = 1.f;   // bias column (rows past T stay zero)
                    v[c][e] *= ic[e];
                }
                mx = fmaxf(mx, absmax8(v[c]));
            }
            mx = row16_max(mx);
            float inv;
            const float sc = pow2_scale(mx, inv);
            char* dst = XHb + row * L::RBYTES + 16 * (c16 ^ chunk_swz(row));
            _Float16* gdst = a.xs_w + (row_base + row) * (2 * (int64_t)NP);
#pragma unroll
            for (int c = 0; c < UH; ++c) {
                half8 h, l;
                split8(v[c], sc, h, l);
                *reinterpret_cast<half8*>(dst + 256 * c) = h;
                *reinterpret_cast<half8*>(dst + BT * L::RBYTES + 256 * c) = l;
                if (ok) {
                    const int c0 = 8 * (c16 + 16 * c);
                    *reinterpret_cast<half8*>(gdst + c0) = h;
                    *reinterpret_cast<half8*>(gdst + NP + c0) = l;
                }
            }
            if (c16 == 0) {
                Us[row] = inv;
                if (ok) a.xu_w[row_base + row] = inv;
            }
        } else {
            const int row = ltid >> 4, c16 = ltid & 15;
            char* dst = XHb + row * L::RBYTES + 16 * (c16 ^ chunk_swz(row));
#pragma unroll
            for (int u = 0; u < L::XPER; ++u) {
                constexpr int UH = NP / 128;
                *reinterpret_cast<float4*>(dst + (u / UH) * (BT * L::RBYTES) + 256 * (u % UH)) = xn[u];
            }
            if (ltid < BT) Us[ltid] = un;
        }
        // EVAL has no weight-gradient phase: the next tile's xhat loads go right
        // after the publish, before this tile's unconditional row-pass loads
        if (MODE == EVAL) xload(tile + gridDim.x, ltid);
        float pa0[4], pa1[4];   // FVP: cached a0 / a1 at (rows kh*16 + 4q + rr, unit cb*16 + r)
        if (MODE == FVP) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = kh * 16 + 4 * lq + rr;
                // rows past T read row 0 of the tile instead of zero: finite values whose
                // output-layer weights are masked to zero (gp), so they add nothing, and
                // no select pulls the wait for these L2 loads to the top of P1
                const int64_t gi = (row_base + (row < nrow ? row : 0)) * H + cb * 16 + lr16;
                pa0[rr] = a.a0[gi];
                pa1[rr] = a.a1[gi];
            }
        }
        __syncthreads();
        KX_STAMP(0);
        // EVAL: this tile's row-pass inputs into registers now (L2 hits since the
        // previous tile's touch below), consumed after P3
        RowPre<BT, MP, KT> rpre;
        if constexpr (MODE == EVAL) row_pre_load<MODE, BT, MP, KT>(a, row_base, ltid, rpre);
        // pull the next tile's other per-row inputs into L2: one dword per 128-byte
        // line (FVP the a0 / a1 caches; FWD / EVAL actions, advantages and the old
        // means / log-likelihoods), kept alive in 2 VGPRs until the next publish
        {
            const int64_t nt = tile + gridDim.x;
            if (nt < ntiles) {
                const int64_t nb = nt * BT;
                const int nr = (int)(T - nb < BT ? T - nb : BT);
                const int mline = (BT * m * 4 + 127) / 128;   // lines of a [BT][m] f32 slab
                const int idx = ltid;
                const float* p = nullptr;
                if (MODE == FVP) {
                    if (idx < 4 * BT && (idx & 63) / 2 < nr)
                        p = (idx < 2 * BT ? a.a0 : a.a1) + (nb + (idx & 63) / 2) * H + (idx & 1) * 32;
                } else {
                    const int ne = nr * m;
                    if (idx < mline) {
                        if (32 * idx < ne) p = a.act + nb * m + 32 * idx;
                    } else if (MODE == EVAL && idx < 2 * mline) {
                        if (32 * (idx - mline) < ne) p = a.mu0 + nb * m + 32 * (idx - mline);
                    } else if (idx == 2 * mline) {
                        p = (MODE == FWD ? a.adv_vpg : a.adv) + nb;
                    } else if (MODE == EVAL && idx == 2 * mline + 1) {
                        p = a.ll0 + nb;
                    }
                }
                touch[0] = *(p ? p : reinterpret_cast<const float*>(a.xs));   // unconditional (see xload)
            } else {
                touch[0] = *reinterpret_cast<const float*>(a.xs);
            }
        }

        // ---- P1: first layer, partial over this wave's observation half ----
        floatx4 acc1[2] = {zero4(), zero4()};
#ifdef MJRL_KX_ABL_NOP1
        if (MODE != FVP)   // timing ablation only: the FVP's first-layer products skipped
#endif
        {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int off = p1off_at(s, opq) + i * 16 * L::RBYTES;   // row i*16 + r16: same swizzle
                    const half8 xh = *reinterpret_cast<const half8*>(XHb + off);
                    const half8 xl = *reinterpret_cast<const half8*>(XLb + off);
                    acc1[i] = mfma_x3(xh, xl, wh[s], wl[s], acc1[i]);
                }
                if (s % 3 == 2) __builtin_amdgcn_sched_barrier(0);   // groups of 3 k-steps: FVP 875 -> 865 us (pairs before)
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc1[i][rr] *= Us[i * 16 + 4 * lq + rr] * wsc1;
        }
        if (MODE == FVP) {
            // FVP: both observation-half partials go to LDS whole (kh = 0 -> D0, kh = 1 ->
            // D0B) and P2 folds them while it loads its operand: no fold phase.  The
            // cached activations of this wave's rows go into the a0 / a1 images.
            float* dst = kh ? D0B : D0;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) dst[(i * 16 + 4 * lq + rr) * L::LD + cb * 16 + lr16] = acc1[i][rr];
            astore4(A0i, cb * 16 + lr16, kh * 16 + 4 * lq, pa0);
            astore4(A1i, cb * 16 + lr16, kh * 16 + 4 * lq, pa1);
            __syncthreads();
            KX_STAMP(1);
            KX_STAMP(2);
        } else {
            // fold the observation halves: wave (cb, kh) hands its partial of row block
            // 1 - kh to its partner and finishes row block kh
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                D0[((1 - kh) * 16 + 4 * lq + rr) * L::LD + cb * 16 + lr16] = kh ? acc1[0][rr] : acc1[1][rr];
            __syncthreads();
            KX_STAMP(1);
            {
                const int col = cb * 16 + lr16;
                float av[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int row = kh * 16 + 4 * lq + rr;
                    av[rr] = tanhf((kh ? acc1[1][rr] : acc1[0][rr]) + D0[row * L::LD + col]);
                    if (MODE == FWD && row < nrow) a.a0[(row_base + row) * H + col] = av[rr];
                }
                astore4(A0i, col, kh * 16 + 4 * lq, av);
            }
            __syncthreads();
            KX_STAMP(2);
        }

        // ---- P2: layer 1, wave -> (rb = kh, cb) ----
        if (!(KX_ABL_NOCHAIN && MODE == FVP)) {
            const int j = cb * 16 + lr16;
            floatx4 acc = zero4();
            float rinv = 1.f;
            if (MODE == FVP) {
                // d0 = (partial_kh0 + partial_kh1) (1 - a0^2), times the W1c column scale,
                // scaled per row and split: d0 W1^T;  + a0 dW1^T (dW1r), a0 from the image
                half8 xh[2], xl[2], ah[2], al[2];
                float8v dv[2];
                float mx = 0.f;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    arow(A0i, kh, s, lq, lr16, xh[s], xl[s]);
                    const int o = (kh * 16 + lr16) * L::LD + 32 * s + 8 * lq;
                    const float8v av = hilo8(xh[s], xl[s]) * AHR_INV;
                    dv[s] = (load8(D0 + o) + load8(D0B + o)) * (1.f - av * av);   // W1c column scale folded in P1
                    mx = fmaxf(mx, absmax8(dv[s]));
                }
                const float sc = pow2_scale(max_over_groups(mx), rinv);
                float ri[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
                floatx4 accb = zero4();
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    split8(dv[s], sc, ah[s], al[s]);
                    half8 bh, bl;
                    wrow(S1, L::WIMG, j, s, lq, bh, bl);
                    acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                    wrow(S2, L::WIMG, j, s, lq, bh, bl);
                    accb = mfma_x3(xh[s], xl[s], bh, bl, accb);
                }
                const float dsc = sc2[j] * AHR_INV;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc[rr] = acc[rr] * ri[rr] + accb[rr] * dsc;
            } else {
                // a0 W1^T (W1r: FWD slot 2, EVAL slot 1)
                const char* img = MODE == FWD ? S2 : S1;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    half8 bh, bl, xh, xl;
                    arow(A0i, kh, s, lq, lr16, xh, xl);
                    wrow(img, L::WIMG, j, s, lq, bh, bl);
                    acc = mfma_x3(xh, xl, bh, bl, acc);
                }
                const float rsc = (MODE == FWD ? sc2 : sc1)[j] * AHR_INV;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc[rr] *= rsc;
            }
            float av[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = kh * 16 + 4 * lq + rr;
                const float v = acc[rr] + bias1;
                if (MODE == FVP) {
                    D1[row * L::LD + j] = (1.f - pa1[rr] * pa1[rr]) * v;
                } else {
                    av[rr] = tanhf(v);
                    if (MODE == FWD && row < nrow) a.a1[(row_base + row) * H + j] = av[rr];
                }
            }
            if (MODE != FVP) astore4(A1i, j, kh * 16 + 4 * lq, av);
        }
        __syncthreads();
        KX_STAMP(3);

        // ---- P3: output layer [32 x MP], waves < 2 * MP/16 -> (rb3, cbo3) ----
        if (w < 2 * (MP / 16) && !(KX_ABL_NOCHAIN && MODE == FVP)) {
            floatx4 acc = zero4();
            if (MODE == FVP) {
                // D1 W2^T (W2c, folded) + a1 dW2^T (dW2r)
                half8 ah[2], al[2];
                const float rinv = adyn<2>(D1, L::LD, rb3, lq, lr16, sc3, ah, al);
                float ri[4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
                floatx4 accb = zero4();
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    half8 bh, bl, xh, xl;
                    wrow(S3, L::WIMG2, col3, s, lq, bh, bl);
                    acc = mfma_x3(ah[s], al[s], bh, bl, acc);
                    arow(A1i, rb3, s, lq, lr16, xh, xl);
                    wrow(S4, L::WIMG2, col3, s, lq, bh, bl);
                    accb = mfma_x3(xh, xl, bh, bl, accb);
                }
                const float dsc = sc4v[col3] * AHR_INV;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc[rr] = acc[rr] * ri[rr] + accb[rr] * dsc;
            } else {
                const char* img = MODE == FWD ? S4 : S3;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    half8 bh, bl, xh, xl;
                    arow(A1i, rb3, s, lq, lr16, xh, xl);
                    wrow(img, L::WIMG2, col3, s, lq, bh, bl);
                    acc = mfma_x3(xh, xl, bh, bl, acc);
                }
                const float rsc = (MODE == FWD ? sc4v : sc3)[col3] * AHR_INV;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc[rr] *= rsc;
            }
            float gv[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = rb3 * 16 + 4 * lq + rr;
                const float v = acc[rr] + bias3;
                if (MODE == FVP)
                    gv[rr] = (col3 < m && row < nrow) ? wq3 * v : 0.f;
                else
                    gv[rr] = col3 < m ? v * os3 + osh3 : 0.f;
                GPf[row * L::LDG + col3] = gv[rr];
            }
            if (MODE == FVP)
                *reinterpret_cast<float4*>(GPT + col3 * L::LDT + rb3 * 16 + 4 * lq) =
                    make_float4(gv[0], gv[1], gv[2], gv[3]);
        }
        if (MP == 16) {   // the padded k16..31 of the P4 operand
            for (int i = ltid; i < BT * 16; i += KT) GPf[(i >> 4) * L::LDG + 16 + (i & 15)] = 0.f;
        }
        __syncthreads();
        KX_STAMP(4);

        if (MODE == EVAL) {
            // per-row pass: LR and KL, its inputs loaded at the top of the tile
            row_pass<MODE, BT, MP, KT, false, true>(a, P + pk.ls, sls, row_base, GPf, L::LDG, racc0, racc1, ltid,
                                                    &rpre, &rconst);
            __syncthreads();
            KX_STAMP(5);
            continue;
        }
        if (MODE != FVP) {
            // per-row pass: FWD log-lik / caches / VPG upstream
            row_pass<MODE, BT, MP, KT, false>(a, P + pk.ls, sls, row_base, GPf, L::LDG, racc0, racc1, ltid,
                                              nullptr, &rconst);
            __syncthreads();
        KX_STAMP(5);
            if (MODE == EVAL) continue;
            for (int i = ltid; i < BT * MP; i += KT) {   // GPT for the gW2 sums
                const int row = i / MP, jj = i % MP;
                GPT[jj * L::LDT + row] = GPf[row * L::LDG + jj];
            }
        }
        if (MODE == EVAL) continue;

        xload(tile + gridDim.x, ltid, 0, L::XPER / 2);   // first half of the next tile's xhat
        // ---- P4: gu1 = (1 - a1^2) (gp W2), wave -> (rb = kh, cb) ----
        if (!(KX_ABL_NOCHAIN && MODE == FVP)) {
            const int hcol = cb * 16 + lr16;
            half8 ah[1], al[1];
            const float rinv = adyn<1>(GPf, L::LDG, kh, lq, lr16, nullptr, ah, al);
            float ri[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
            half8 bh, bl;
            wcol(S3, L::WIMG2, cb, 0, lq, lr16, bh, bl);
            const floatx4 acc = mfma_x3(ah[0], al[0], bh, bl, zero4());
            const float csc = sc3[hcol];
            float gv[4], a4[4];
            if (MODE != FVP) aval4(A1i, hcol, kh * 16 + 4 * lq, a4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = kh * 16 + 4 * lq + rr;
                const float av = MODE == FVP ? pa1[rr] : a4[rr];
                gv[rr] = (1.f - av * av) * (acc[rr] * ri[rr] * csc);
                D0[row * L::LD + hcol] = gv[rr];   // G1
            }
            *reinterpret_cast<float4*>(G1T + hcol * L::LDT + kh * 16 + 4 * lq) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        }
        // the gW2 sums (gW2[jb = w >> 2][kb = w & 3] += gp^T a1; gb2 = row sums of gp on
        // waves kb = 0): FVP runs them beside P4, off P5's chain (GPT is complete since
        // P3); FWD in P5 (its GPT is transposed right before P4, without a barrier)
        auto gw2_sum = [&]() __attribute__((always_inline)) {
            half8 gh, gl;
            float s4[4];
            if ((w >> 2) < MP / 16) {
                const float8v v = load8(GPT + ((w >> 2) * 16 + lr16) * L::LDT + 8 * lq);
                float inv;
                const float sc = pow2_scale(max_over_groups(absmax8(v)), inv);
                split8(v, sc, gh, gl);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) s4[rr] = __shfl(inv * AHR_INV, 4 * lq + rr, 64);
                if ((w & 3) == 0) {
                    b2acc += sum_over_groups(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
                }
                half8 bh, bl;
                acol(A1i, (w & 3) * 16 + lr16, lq, bh, bl);
                const floatx4 t = mfma_x3(gh, gl, bh, bl, zero4());
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) g2[rr] += t[rr] * s4[rr];
            }
        };
        if (MODE == FVP && !KX_ABL_NOCHAIN) gw2_sum();
        __syncthreads();
        KX_STAMP(6);
        // ---- P5: gu0 = (1 - a0^2) (gu1 W1), times the xhat row scale; beside it the
        // gW1 / gW2 sums (their operands are complete since P4) and the next tile's
        // xhat loads (consumed at the next publish) ----
        xload(tile + gridDim.x, ltid, L::XPER / 2, L::XPER);
        auto p5_gu0 = [&]() __attribute__((always_inline)) {
            const int hcol = cb * 16 + lr16;
            half8 ah[2], al[2];
            const float rinv = adyn<2>(D0, L::LD, kh, lq, lr16, nullptr, ah, al);
            float ri[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) ri[rr] = __shfl(rinv, 4 * lq + rr, 64);
            floatx4 acc = zero4();
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                half8 bh, bl;
                wcol(S1, L::WIMG, cb, s, lq, lr16, bh, bl);
                acc = mfma_x3(ah[s], al[s], bh, bl, acc);
            }
            const float csc = sc1[hcol];
            float gv[4], a4[4];
            aval4(A0i, hcol, kh * 16 + 4 * lq, a4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int row = kh * 16 + 4 * lq + rr;
                const float av = a4[rr];
                gv[rr] = (1.f - av * av) * (acc[rr] * ri[rr] * csc) * Us[row];
            }
            *reinterpret_cast<float4*>(D1 + hcol * L::LDT + kh * 16 + 4 * lq) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        };
        auto p5_gw = [&]() __attribute__((always_inline)) {
            half8 gh, gl;
            float s4[4];
            // gW1[jb = cb][kb = kh + 2jj] += gu1^T a0;  gb1 = row sums of gu1 (waves kh = 0)
            {
                const float8v v = load8(G1T + (cb * 16 + lr16) * L::LDT + 8 * lq);
                float inv;
                const float sc = pow2_scale(max_over_groups(absmax8(v)), inv);
                split8(v, sc, gh, gl);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) s4[rr] = __shfl(inv * AHR_INV, 4 * lq + rr, 64);
                if (kh == 0) {
                    b1acc += sum_over_groups(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
                }
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                half8 bh, bl;
                acol(A0i, (kh + 2 * jj) * 16 + lr16, lq, bh, bl);
                const floatx4 t = mfma_x3(gh, gl, bh, bl, zero4());
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) g1[jj][rr] += t[rr] * s4[rr];
            }
        };
        // (running the two halves in opposite orders on the two waves of a SIMD,
        // kh = 0 / 1, measured 0.5 %: the phase is issue-bound, not latency-bound)
        if (!(KX_ABL_NOCHAIN && MODE == FVP)) {
            p5_gu0();
            p5_gw();
        }
        if (MODE != FVP) gw2_sum();
        __syncthreads();
        KX_STAMP(7);

        // ---- P6: the gW0 sums ----
        KX_STAMP(10);
#ifdef MJRL_KX_ABL_NOP6
        if (false)   // timing ablation only (the two-kernel decomposition): results are wrong
#endif
        {
            // gW0 (xhat transposed reads)
            half8 gh, gl;
            float s4[4];
            gdyn(D1, L::LDT, cb, lq, lr16, gh, gl, s4);   // G0T
            KX_STAMP(11);
#pragma unroll
            for (int g = 0; g < KG; ++g) {
                short4v th[2], tl[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // rows 8q + 4h + tq: the chunk swizzle ignores row bit 2, so h = 1 is
                    // the h = 0 offset plus four rows
                    const int off = g0off_at(g, opq) + h * 4 * L::RBYTES;
                    th[h] = ds_read_tr16(XHb + off);
                    tl[h] = ds_read_tr16(XLb + off);
                }
                const floatx4 t = mfma_x3(gh, gl, cat_tr(th[0], th[1]), cat_tr(tl[0], tl[1]), zero4());
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) g0[g][rr] += t[rr] * s4[rr];
                if (g & 1) __builtin_amdgcn_sched_barrier(0);
            }
            KX_STAMP(12);
        }
        KX_STAMP(14);
        __syncthreads();
        KX_STAMP(8);
    }

    // slabs in the flat, parameter-chunk-major layout wpart[f / 64][S][64] (f = the
    // reference's flat parameter index, S = gridDim.x): k_gather_flat then reads
    // every chunk as one contiguous run.  The values are staged in LDS in flat
    // parameter order first (the tile loop's buffers are free) and leave in 16-byte
    // stores, each chunk's 256 bytes from 16 lanes: ~15 wide stores per thread
    // instead of ~60 scattered 4-byte ones (the scattered tail took 15.8k cycles per
    // FVP launch, profiles/r04f/kx_phase_profile_125k.txt)
    const int64_t blk = blockIdx.x;
    if constexpr (GRAD) {
        const int n = o.n, mm = o.m;
        const int64_t S = gridDim.x;
        float* slab = smem;   // [d_mu] in flat parameter order
        static_assert(H * NP + H + H * H + H + MP * H + MP <= L::bytes / 4, "slab staging in LDS");
        auto put = [&](int f, float v) { slab[f] = v; };
        const int fb0 = H * n, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + mm * H;
#pragma unroll
        for (int g = 0; g < KG; ++g) {
            const int k = kh * KH + 16 * g + r16;
            const float xck = a.xc[k];   // the rows' column scale (exact)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int hid = cb * 16 + 4 * q + rr;
                if (k < n)
                    put(hid * n + k, g0[g][rr] * xck);
                else if (k == n)
                    put(fb0 + hid, g0[g][rr] * xck);   // b0 rides in the bias column
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) put(fW1 + (cb * 16 + 4 * q + rr) * H + (kh + 2 * j) * 16 + r16, g1[j][rr]);
        if ((w >> 2) < MP / 16) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int j = (w >> 2) * 16 + 4 * q + rr;
                if (j < mm) put(fW2 + j * H + (w & 3) * 16 + r16, g2[rr]);
            }
        }
        if (kh == 0 && q == 0) put(fb1 + cb * 16 + r16, b1acc);
        if ((w >> 2) < MP / 16 && (w & 3) == 0 && q == 0 && (w >> 2) * 16 + r16 < mm)
            put(fb2 + (w >> 2) * 16 + r16, b2acc);
        __syncthreads();
        const int dmu = fb2 + mm;
        for (int f0 = 4 * tid; f0 < dmu; f0 += 4 * KT) {
            const int64_t gi = (((int64_t)(f0 >> 6)) * S + blk) * 64 + (f0 & 63);   // f0 % 4 == 0: one chunk
            if (f0 + 3 < dmu) {
                MJRL_SLAB_CHECK(gi + 3, o.wcap);
                *reinterpret_cast<float4*>(o.wpart + gi) = *reinterpret_cast<const float4*>(slab + f0);
            } else {
                for (int e = 0; f0 + e < dmu; ++e) {
                    MJRL_SLAB_CHECK(gi + e, o.wcap);
                    o.wpart[gi + e] = slab[f0 + e];
                }
            }
        }
    }
    if (MODE != FVP) {
        __syncthreads();
        row_pass_final<MODE, MP, KT>(racc0, racc1, reinterpret_cast<double*>(smem), a.rpart, blk, tid);
    }
#ifdef MJRL_KX_PROF
    kx_acc_[16] = __builtin_amdgcn_s_memtime() - kx_last_;
    if (blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < KX_NPROF; ++i) g_kx_prof[i] += kx_acc_[i];
#endif
}

}  // namespace
