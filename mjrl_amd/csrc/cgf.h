// cgf.h — the whole conjugate-gradient solve of a small batch in ONE launch
// (included by policy.hip after fused.h and the gathers).  mjrl/utils/cg_solve.py:3-22
// with the FVP of mjrl/algos/npg_cg.py:55-74.
//
// For the k_fused shapes (hidden <= 64, small observations: Swimmer) every CG
// iteration was three latency-bound launches — the FVP (one 64-row tile per
// workgroup at 12.5k rows), the slab gather with the z step, and the iteration's
// tail — ~33 us, mostly launch gaps and single-tile latency.  Here the k_fused
// workgroups stay resident for all iterations and meet at grid barriers:
//   FVP       fused_body: this workgroup's tiles -> its slab (flat layout)
//   barrier
//   gather    64-parameter chunks ch = blockIdx.x + k G: the S slabs folded in
//             k_gather_flat's order (16 slice ranges, fixed-order fp64), then the
//             z step and the chunk's p.z partial (cgz_epilogue)
//   barrier
//   tail      every workgroup folds the p.z partials and the new r.r over all of
//             d in k_cgm_xrp_f's order (a 1024-thread fold emulated by 512
//             threads), then updates x, r, p (and packed p) of its own elements
//   barrier
// so the results are bit-identical to the three-launch loop.  The grid must be
// co-resident (one 110 KB workgroup per CU; the host checks the occupancy before
// choosing this path); a barrier that waits ~0.1 s anyway gives up and sets an
// error word the host checks, so a non-resident grid ends with an error instead of
// a hang.  Barrier counter and error word: cg[10], cg[11] (zeroed by mjrl_cg_init).
#pragma once

namespace {

struct CgfArgs {
    CgZ cz;              // p, z, cg, ls, inv_T, damping, ls0
    float* x;
    float* r0;
    float* r1;           // r alternates r0 -> r1 -> r0 ... (k_cgm_xrp_f's ping-pong)
    float* packed_p;
    int32_t* done;
    float tol;
    int iters, d, d_mu, nch;
    mjrl_shape s;
};

// grid barrier: release this workgroup's writes, count in, spin (agent-scope loads,
// s_sleep between polls), acquire the others' writes
__device__ __forceinline__ void cgf_barrier(unsigned* ctr, unsigned target, unsigned* err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        atomicAdd(ctr, 1u);
        if (!__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            unsigned spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins == (1u << 20)) {   // ~0.1 s: the grid is not co-resident
                    atomicOr(err, 1u);
                    break;
                }
            }
        }
        __threadfence();
    }
    __syncthreads();
}

// block_sum<1024> of k_cgm_xrp_f with 512 threads: q0 is virtual thread tid's
// partial, q1 virtual thread tid + 512's; the same wave trees and the same in-order
// sum of the 16 wave partials
__device__ __forceinline__ double cgf_fold1024(double q0, double q1, double* red) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    q0 = wave_sum(q0);
    q1 = wave_sum(q1);
    __syncthreads();
    if (l == 0) {
        red[w] = q0;
        red[w + 8] = q1;
    }
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i];
    return s;
}

template <int H0, int H1, int MP, int NCH>
__global__ void __launch_bounds__(FT, 1) k_cg_fused(RowArgs a, FOut o, CgfArgs c) {
    static_assert(FT == 512 && GATHER_WAVES == 16, "the gather / tail folds emulate 1024-thread blocks");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float* cg = c.cz.cg;
    unsigned* ctr = reinterpret_cast<unsigned*>(cg) + 10;
    unsigned* err = reinterpret_cast<unsigned*>(cg) + 11;
    const unsigned G = gridDim.x;
    const int S = (int)G;   // one slab per workgroup
    const double* pzp = reinterpret_cast<const double*>(cg + CG_PZ_PARTS);
    const PackMap pm(c.s);
    unsigned target = 0;
    float rdotr = cg[0];   // k_cgm_init's (previous launch)
    float pz = 0.f, v = 0.f, mu = 0.f, rr = rdotr;
    int k = 0;
    while (k < c.iters) {
        // ---- FVP: this workgroup's slab ----
        fused_body<H0, H1, MP, NCH, FVP>(a, o);
        target += G;
        cgf_barrier(ctr, target, err);
        // ---- gather + z: k_gather_flat's fold, 16 slice ranges on 8 waves ----
        {
            double* part = reinterpret_cast<double*>(smem);   // [16][64]
            const int per = (S + GATHER_WAVES - 1) / GATHER_WAVES;
            for (int ch = blockIdx.x; ch < c.nch; ch += G) {
                const int f = ch * 64 + lane;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int vw = w + 8 * h;
                    double acc = 0.0;
                    if (f < c.d_mu) {
                        const int s0 = vw * per, s1 = min(S, s0 + per);
                        const float* p = o.wpart + (int64_t)ch * S * 64 + lane;
                        for (int sb = s0; sb < s1; sb += GATHER_PER) {
                            float vv[GATHER_PER];
#pragma unroll
                            for (int j = 0; j < GATHER_PER; ++j) vv[j] = sb + j < s1 ? p[(int64_t)(sb + j) * 64] : 0.f;
#pragma unroll
                            for (int j = 0; j < GATHER_PER; ++j) acc += (double)vv[j];
                        }
                    }
                    part[vw * 64 + lane] = acc;
                }
                __syncthreads();
                if (w == 0) {
                    float gs = 0.f;
                    if (f < c.d) {
                        double t = part[lane];
#pragma unroll
                        for (int j = 1; j < GATHER_WAVES; ++j) t += part[j * 64 + lane];
                        gs = (float)t;
                    }
                    cgz_epilogue(c.cz, f, c.d, gs, ch);
                }
                __syncthreads();
            }
        }
        target += G;
        cgf_barrier(ctr, target, err);
        // ---- the iteration's tail: k_cgm_xrp_f's folds in every workgroup ----
        {
            double* red = reinterpret_cast<double*>(smem);
            const float* r_in = (k & 1) ? c.r1 : c.r0;
            float* r_out = (k & 1) ? c.r0 : c.r1;
            const float* z = c.cz.z;
            float* p = const_cast<float*>(c.cz.p);
            double q0 = 0.0, q1 = 0.0;
            for (int i = tid; i < c.nch; i += 1024) q0 += pzp[i];
            for (int i = tid + 512; i < c.nch; i += 1024) q1 += pzp[i];
            pz = (float)cgf_fold1024(q0, q1, red);
            v = rdotr / pz;   // v = rdotr / p.z
            double a0 = 0.0, a1 = 0.0;
#pragma unroll 8
            for (int f = tid; f < c.d; f += 1024) {
                const float rf = __fsub_rn(r_in[f], __fmul_rn(v, z[f]));
                a0 += (double)rf * (double)rf;
            }
#pragma unroll 8
            for (int f = tid + 512; f < c.d; f += 1024) {
                const float rf = __fsub_rn(r_in[f], __fmul_rn(v, z[f]));
                a1 += (double)rf * (double)rf;
            }
            rr = (float)cgf_fold1024(a0, a1, red);
            mu = rr / rdotr;
            for (int f = blockIdx.x * FT + tid; f < c.d; f += (int)G * FT) {
                const float pf = p[f];
                c.x[f] = __fadd_rn(c.x[f], __fmul_rn(v, pf));
                const float rf = __fsub_rn(r_in[f], __fmul_rn(v, z[f]));
                r_out[f] = rf;
                if (!(rr < c.tol)) {   // converged: p is not used again
                    const float pn = __fadd_rn(rf, __fmul_rn(mu, pf));
                    p[f] = pn;
                    pack_one(pm, f, pn, c.packed_p, false, 0.f);
                }
            }
        }
        rdotr = rr;
        ++k;
        if (rr < c.tol) break;   // cg_solve.py:19-20 (every workgroup computed the same rr)
        target += G;
        cgf_barrier(ctr, target, err);
    }
    if (blockIdx.x == 0 && tid == 0) {
        cg[4] = pz;
        cg[2] = v;
        cg[3] = mu;
        cg[0] = rr;
        cg[1] += (float)k;
        if (rr < c.tol) *c.done = 1;
    }
}

}  // namespace
