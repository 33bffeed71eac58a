// cg.hip — parameter packing, conjugate gradient and the natural-gradient step,
// all on device so the CG loop never synchronises with the host.
//
// Reference: mjrl/utils/cg_solve.py:3-22, mjrl/algos/npg_cg.py:128-144,
// mjrl/algos/trpo.py:100-108, mjrl/policies/gaussian_mlp.py:66-88.
// The d-length vector work is tiny (d <= ~1e5): one 1024-thread workgroup,
// fp64 accumulation of the dot products, fp32 scalar arithmetic in the
// reference's order (numpy fp32 arrays).
#include <math.h>

#include "common.h"

using namespace mjrl;

namespace {

constexpr int CG_THREADS = 1024;
constexpr int CG_U = 8;   // elements per thread per chunk of a pass


__global__ void __launch_bounds__(256) k_pack(mjrl_shape s, const float* __restrict__ theta, float* __restrict__ packed,
                                              int clamp, float min_ls) {
    const PackMap pm(s);
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < s.d) pack_one(pm, f, theta[f], packed, clamp != 0, min_ls);
}

__device__ __forceinline__ double block_sum1024(double v, double* red) { return block_sum<CG_THREADS>(v, red); }

// cg_solve.py:4-7: x = 0, r = b, p = r, rdotr = r.r
__global__ void __launch_bounds__(CG_THREADS) k_cg_init(mjrl_shape s, const float* __restrict__ b, float* __restrict__ x,
                                                        float* __restrict__ r, float* __restrict__ p,
                                                        float* __restrict__ packed_p, float* __restrict__ cg,
                                                        int32_t* __restrict__ done) {
    __shared__ double red[CG_THREADS / 64];
    const PackMap pm(s);
    double acc = 0.0;
#pragma unroll 8
    for (int f = threadIdx.x; f < s.d; f += CG_THREADS) {
        const float v = b[f];
        x[f] = 0.f;
        r[f] = v;
        p[f] = v;
        pack_one(pm, f, v, packed_p, false, 0.f);
        acc += (double)v * (double)v;
    }
    const double rr = block_sum1024(acc, red);
    if (threadIdx.x == 0) {
        cg[0] = (float)rr;   // rdotr
        cg[1] = 0.f;         // iterations run
        *reinterpret_cast<unsigned*>(cg + 8) = 0u;   // k_cgm_* ticket
        *done = 0;
    }
}

// One CG iteration (cg_solve.py:10-20) given the raw FVP sums for direction p:
// z = F p + damping p with F p = gsum / T on the mean block and c(sigma) p on the
// log-std block (closed form of the double-backprop HVP).
__global__ void __launch_bounds__(CG_THREADS) k_cg_step(mjrl_shape s, const float* __restrict__ gsum, double inv_T,
                                                        float damping, const float* __restrict__ packed_theta,
                                                        float* __restrict__ x, float* __restrict__ r,
                                                        float* __restrict__ p, float* __restrict__ z,
                                                        float* __restrict__ packed_p, float* __restrict__ cg,
                                                        int32_t* __restrict__ done, float tol) {
    __shared__ double red[CG_THREADS / 64];
    if (*done) return;
    const PackMap pm(s);
    const int ls0 = s.d - s.m, d = s.d, tid = threadIdx.x;
    constexpr int CH = CG_THREADS * CG_U;
    // each pass walks d in chunks of CG_U elements per thread, all loads of a
    // chunk issued before use (the single workgroup is latency-bound otherwise)
    double acc = 0.0;
    for (int f0 = 0; f0 < d; f0 += CH) {
        float pf[CG_U], gv[CG_U];
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            pf[u] = f < d ? p[f] : 0.f;
            gv[u] = f < ls0 ? gsum[f] : (f < d ? packed_theta[pm.pk.ls + (f - ls0)] : 0.f);
        }
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            if (f >= d) continue;
            float hv;
            if (f >= ls0) {
                const float sg = expf(gv[u]);
                const double uu = (double)sg * (double)sg;
                const double c = 4.0 * uu * (2.0 * uu - 1e-8) / ((2.0 * uu + 1e-8) * (2.0 * uu + 1e-8));
                hv = (float)(c * (double)pf[u]);
            } else {
                hv = (float)((double)gv[u] * inv_T);
            }
            const float zf = __fadd_rn(hv, __fmul_rn(damping, pf[u]));   // hvp_flat + regu_coef*vector
            z[f] = zf;
            acc += (double)pf[u] * (double)zf;
        }
    }
    const float pz = (float)block_sum1024(acc, red);
    const float rdotr = cg[0];
    const float v = rdotr / pz;
    acc = 0.0;
    for (int f0 = 0; f0 < d; f0 += CH) {
        float xv[CG_U], pv[CG_U], rv[CG_U], zv[CG_U];
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            const bool in = f < d;
            xv[u] = in ? x[f] : 0.f;
            pv[u] = in ? p[f] : 0.f;
            rv[u] = in ? r[f] : 0.f;
            zv[u] = in ? z[f] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            if (f >= d) continue;
            x[f] = __fadd_rn(xv[u], __fmul_rn(v, pv[u]));
            const float rf = __fsub_rn(rv[u], __fmul_rn(v, zv[u]));
            r[f] = rf;
            acc += (double)rf * (double)rf;
        }
    }
    const float rr = (float)block_sum1024(acc, red);
    const float mu = rr / rdotr;
    for (int f0 = 0; f0 < d; f0 += CH) {
        float pv[CG_U], rv[CG_U];
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            pv[u] = f < d ? p[f] : 0.f;
            rv[u] = f < d ? r[f] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < CG_U; ++u) {
            const int f = f0 + u * CG_THREADS + tid;
            if (f >= d) continue;
            const float pf = __fadd_rn(rv[u], __fmul_rn(mu, pv[u]));
            p[f] = pf;
            pack_one(pm, f, pf, packed_p, false, 0.f);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        cg[0] = rr;
        cg[1] += 1.f;
        cg[2] = v;
        cg[3] = mu;
        cg[4] = pz;
        if (rr < tol) *done = 1;   // cg_solve.py:19-20
    }
}

// ---------------------------------------------------------------------------
// The same iteration as k_cg_step over many workgroups (MJRL_CG_WG elements
// each), in three launches; each dot product is a fixed-order fp64 sum of
// per-workgroup partials folded by the LAST workgroup to arrive (atomic ticket,
// no spinning), so results do not depend on scheduling:
//   k_cgm_z : z = F p + damping p, pz            -> cg[4] = pz, cg[2] = v = rdotr / pz
//   k_cgm_xr: x += v p, r -= v z, rr             -> cg[0] = rr, cg[3] = mu, iters, done
//   k_cgm_p : p = r + mu p, packed p
// State beyond cg[0..7]: cg[8] = ticket (u32), cg[16..] = double partials.
// ---------------------------------------------------------------------------
constexpr int CGM_T = 256;                 // threads per workgroup
constexpr int CGM_U = 4;                   // elements per thread
constexpr int CGM_WG = CGM_T * CGM_U;      // elements per workgroup
constexpr int CGM_MAXWG = (CG_PZ_PARTS - 16) / 2;   // partials below the fused gather's region
constexpr int CG_PZ_MAX = (MJRL_CG_STATE - CG_PZ_PARTS) / 2;   // fused gather workgroups (64 parameters each)

// fixed-order fold of nwg per-workgroup partials by the last workgroup to finish
__device__ __forceinline__ bool cgm_last(double part, float* cg, int nwg, double* red, double& total) {
    double* parts = reinterpret_cast<double*>(cg + 16);
    const double b = block_sum<CGM_T>(part, red);
    __shared__ unsigned ticket;
    if (threadIdx.x == 0) {
        parts[blockIdx.x] = b;
        __threadfence();
        ticket = atomicAdd(reinterpret_cast<unsigned*>(cg + 8), 1u);
    }
    __syncthreads();
    if (ticket != (unsigned)(nwg - 1)) return false;
    __threadfence();
    if (threadIdx.x < 64) {
        // wave 0: lane l folds partials l, l + 64, ... in order (all loads in flight
        // together), then a fixed shuffle tree; the same order on every run
        double t = 0.0;
        for (int i = threadIdx.x; i < nwg; i += 64) t += parts[i];   // visible after the acquire fence above
        t = wave_sum(t);
        if (threadIdx.x == 0) {
            total = t;
            *reinterpret_cast<unsigned*>(cg + 8) = 0u;   // reset the ticket for the next launch
        }
    }
    return true;
}

__global__ void __launch_bounds__(CGM_T) k_cgm_z(mjrl_shape s, const float* __restrict__ gsum, double inv_T,
                                                 float damping, const float* __restrict__ packed_theta,
                                                 const float* __restrict__ p, float* __restrict__ z, float* cg,
                                                 const int32_t* __restrict__ done) {
    __shared__ double red[CGM_T / 64];
    if (*done) return;
    const Packed pk(s.h0, s.h1, s.np, s.mp);
    const int ls0 = s.d - s.m, d = s.d;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f >= d) continue;
        const float pf = p[f];
        float hv;
        if (f >= ls0) {
            const float sg = expf(packed_theta[pk.ls + (f - ls0)]);
            const double uu = (double)sg * (double)sg;
            const double c = 4.0 * uu * (2.0 * uu - 1e-8) / ((2.0 * uu + 1e-8) * (2.0 * uu + 1e-8));
            hv = (float)(c * (double)pf);
        } else {
            hv = (float)((double)gsum[f] * inv_T);
        }
        const float zf = __fadd_rn(hv, __fmul_rn(damping, pf));   // hvp_flat + regu_coef*vector
        z[f] = zf;
        acc += (double)pf * (double)zf;
    }
    double t;
    if (cgm_last(acc, cg, gridDim.x, red, t) && threadIdx.x == 0) {
        const float pz = (float)t;
        cg[4] = pz;
        cg[2] = cg[0] / pz;   // v = rdotr / p.z
    }
}

__global__ void __launch_bounds__(CGM_T) k_cgm_xr(int d, const float* __restrict__ p, const float* __restrict__ z,
                                                  float* __restrict__ x, float* __restrict__ r, float* cg,
                                                  int32_t* __restrict__ done, float tol) {
    __shared__ double red[CGM_T / 64];
    if (*done) return;
    const float v = cg[2];
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f >= d) continue;
        x[f] = __fadd_rn(x[f], __fmul_rn(v, p[f]));
        const float rf = __fsub_rn(r[f], __fmul_rn(v, z[f]));
        r[f] = rf;
        acc += (double)rf * (double)rf;
    }
    double t;
    if (cgm_last(acc, cg, gridDim.x, red, t) && threadIdx.x == 0) {
        const float rr = (float)t;
        const float rdotr = cg[0];
        cg[3] = rr / rdotr;   // mu
        cg[0] = rr;
        cg[1] += 1.f;
        if (rr < tol) *done = 1;   // cg_solve.py:19-20
    }
}

// The rest of a fused-gather CG iteration in ONE launch (cg_solve.py:11-20):
// every workgroup folds the gather's p.z partials, then computes the new
// r.r = sum_f (r_f - v z_f)^2 over ALL of d itself (the same f32 r_f the update
// stores, fp64 sums in the same fixed order in every workgroup), so it knows mu
// without waiting for the others and updates x, r and p of its own 1024-element
// chunk.  The new r goes to r_out (every workgroup reads all of r_in), the
// caller alternating the two buffers.  The last workgroup to take the ticket (all
// have read rdotr by then) records rdotr, mu, v, p.z, the iteration count and the
// residual_tol break.
constexpr int CGX_T = 1024;
template <int XRP_PRE>   // terms of the r.r fold per thread loaded up front (8: d <= 8192, 32: d <= 32768)
__global__ void __launch_bounds__(CGX_T) k_cgm_xrp_f(mjrl_shape s, float* __restrict__ p, const float* __restrict__ z,
                                                     float* __restrict__ x, const float* __restrict__ r,
                                                     float* __restrict__ r_out, float* __restrict__ packed_p, float* cg,
                                                     int32_t* __restrict__ done, float tol, int ng) {
    __shared__ double red[CGX_T / 64];
    __shared__ unsigned ticket;
    const int d = s.d;
    // every load that does not depend on v / mu is issued up front: this thread's own
    // element (p, x, r, z) and the first XRP_PRE terms of the r.r fold per thread
    const int f = blockIdx.x * CGX_T + threadIdx.x;
    const bool own = f < d;
    const float pf = own ? p[f] : 0.f, xf = own ? x[f] : 0.f, rfo = own ? r[f] : 0.f, zfo = own ? z[f] : 0.f;
    float rpre[XRP_PRE], zpre[XRP_PRE];
#pragma unroll
    for (int u = 0; u < XRP_PRE; ++u) {
        const int g = threadIdx.x + u * CGX_T;
        rpre[u] = g < d ? r[g] : 0.f;
        zpre[u] = g < d ? z[g] : 0.f;
    }
    const float rdotr = cg[0];
    const double* pzp = reinterpret_cast<const double*>(cg + CG_PZ_PARTS);
    double q = 0.0;
    for (int i = threadIdx.x; i < ng; i += CGX_T) q += pzp[i];
    const float pz = (float)block_sum<CGX_T>(q, red);
    const float v = rdotr / pz;   // v = rdotr / p.z
    double acc = 0.0;   // the fold of r.r in f order, as before: the prefetched terms first
#pragma unroll
    for (int u = 0; u < XRP_PRE; ++u)
        if (threadIdx.x + u * CGX_T < d) {
            const float rf = __fsub_rn(rpre[u], __fmul_rn(v, zpre[u]));
            acc += (double)rf * (double)rf;
        }
#pragma unroll 8
    for (int g = threadIdx.x + XRP_PRE * CGX_T; g < d; g += CGX_T) {
        const float rf = __fsub_rn(r[g], __fmul_rn(v, z[g]));
        acc += (double)rf * (double)rf;
    }
    const float rr = (float)block_sum<CGX_T>(acc, red);
    const float mu = rr / rdotr;
    // a converged CG loop (cg_solve.py:19-20): nothing is stored; checked after the
    // folds, so the flag's load overlaps the state's
    if (*done) return;
    if (own) {
        x[f] = __fadd_rn(xf, __fmul_rn(v, pf));
        const float rf = __fsub_rn(rfo, __fmul_rn(v, zfo));
        r_out[f] = rf;
        if (!(rr < tol)) {   // converged: p is not used again
            const float pn = __fadd_rn(rf, __fmul_rn(mu, pf));
            p[f] = pn;
            pack_one(PackMap(s), f, pn, packed_p, false, 0.f);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(reinterpret_cast<unsigned*>(cg + 8), 1u);
    __syncthreads();
    if (ticket == gridDim.x - 1 && threadIdx.x == 0) {
        cg[4] = pz;
        cg[2] = v;
        cg[3] = mu;
        cg[0] = rr;
        cg[1] += 1.f;
        if (rr < tol) *done = 1;   // cg_solve.py:19-20
        *reinterpret_cast<unsigned*>(cg + 8) = 0u;
    }
}

// The z step of a CG iteration from an all-reduced gradient sum (the sharded path):
// z = gsum inv_T + c(sigma) p_ls + damping p and one p.z partial per 64 parameters,
// exactly as the fused gather's epilogue writes them from its own fold
// (cgz_epilogue), so k_cgm_xrp_f finishes the iteration as in one process (with
// one rank the two schedules are bit-identical).
__global__ void __launch_bounds__(64) k_cg_zpart(int d, const float* __restrict__ gsum,
                                                 const int32_t* __restrict__ done, CgZ cz) {
    if (*done) return;
    const int f = blockIdx.x * 64 + threadIdx.x;
    cgz_epilogue(cz, f, d, f < d ? gsum[f] : 0.f);
}

// A whole CG iteration after an all-reduced gradient sum (the sharded path) in ONE
// launch: every workgroup forms z = gsum inv_T + c(sigma) p_ls + damping p on the
// fly for all of d, folds p.z and then the new r.r in the same fixed order as
// every other workgroup, and updates x, r (into r_out) and p of its own chunk;
// the last workgroup to take the ticket records the CG scalars.  z itself is
// never stored (cg_solve.py keeps it local too).
__device__ __forceinline__ float cg_z(const mjrl_shape& s, const float* __restrict__ gsum, double inv_T,
                                      float damping, const float* __restrict__ P_ls, const float* __restrict__ p,
                                      int f) {
    const float pf = p[f];
    float hv;
    const int ls0 = s.d - s.m;
    if (f >= ls0) {
        const float sg = expf(P_ls[f - ls0]);
        const double uu = (double)sg * (double)sg;
        const double c = 4.0 * uu * (2.0 * uu - 1e-8) / ((2.0 * uu + 1e-8) * (2.0 * uu + 1e-8));
        hv = (float)(c * (double)pf);
    } else {
        hv = (float)((double)gsum[f] * inv_T);
    }
    return __fadd_rn(hv, __fmul_rn(damping, pf));   // hvp_flat + regu_coef * vector
}

__global__ void __launch_bounds__(CGX_T) k_cgm_step1(mjrl_shape s, const float* __restrict__ gsum, double inv_T,
                                                     float damping, const float* __restrict__ packed_theta,
                                                     float* __restrict__ x, const float* __restrict__ r,
                                                     float* __restrict__ r_out, const float* __restrict__ p,
                                                     float* __restrict__ p_out, float* __restrict__ packed_p,
                                                     float* cg, int32_t* __restrict__ done, float tol) {
    __shared__ double red[CGX_T / 64];
    __shared__ unsigned ticket;
    if (*done) return;
    const int d = s.d;
    const float* P_ls = packed_theta + Packed(s.h0, s.h1, s.np, s.mp).ls;
    double acc = 0.0;
#pragma unroll 4
    for (int f = threadIdx.x; f < d; f += CGX_T) acc += (double)p[f] * (double)cg_z(s, gsum, inv_T, damping, P_ls, p, f);
    const float pz = (float)block_sum<CGX_T>(acc, red);
    const float rdotr = cg[0];
    const float v = rdotr / pz;   // v = rdotr / p.z
    acc = 0.0;
#pragma unroll 4
    for (int f = threadIdx.x; f < d; f += CGX_T) {
        const float rf = __fsub_rn(r[f], __fmul_rn(v, cg_z(s, gsum, inv_T, damping, P_ls, p, f)));
        acc += (double)rf * (double)rf;
    }
    const float rr = (float)block_sum<CGX_T>(acc, red);
    const float mu = rr / rdotr;
    const int f = blockIdx.x * CGX_T + threadIdx.x;
    if (f < d) {   // own chunk; r and p go to the other buffer of their pair (all workgroups read r / p)
        const float pf = p[f];
        const float rf = __fsub_rn(r[f], __fmul_rn(v, cg_z(s, gsum, inv_T, damping, P_ls, p, f)));
        x[f] = __fadd_rn(x[f], __fmul_rn(v, pf));
        r_out[f] = rf;
        const float pn = __fadd_rn(rf, __fmul_rn(mu, pf));
        p_out[f] = pn;
        pack_one(PackMap(s), f, pn, packed_p, false, 0.f);
    }
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(reinterpret_cast<unsigned*>(cg + 8), 1u);
    __syncthreads();
    if (ticket == gridDim.x - 1 && threadIdx.x == 0) {
        cg[4] = pz;
        cg[2] = v;
        cg[3] = mu;
        cg[0] = rr;
        cg[1] += 1.f;
        if (rr < tol) *done = 1;   // cg_solve.py:19-20
        *reinterpret_cast<unsigned*>(cg + 8) = 0u;
    }
}

__global__ void __launch_bounds__(CGM_T) k_cgm_p(mjrl_shape s, const float* __restrict__ r, float* __restrict__ p,
                                                 float* __restrict__ packed_p, const float* cg,
                                                 const int32_t* __restrict__ done) {
    if (*done) return;   // converged: p is not used again
    const PackMap pm(s);
    const float mu = cg[3];
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f >= s.d) continue;
        const float pf = __fadd_rn(r[f], __fmul_rn(mu, p[f]));
        p[f] = pf;
        pack_one(pm, f, pf, packed_p, false, 0.f);
    }
}

// cg_solve.py:4-7 over many workgroups: x = 0, r = p = b (and packed p), rdotr
// = b.b folded in fixed order by the last workgroup.
// b: the right-hand side, or (gsum != null) b = float(double(gsum) * scale) formed
// here and written to b (the VPG's mean from its sums, k_scale_vec's arithmetic:
// one launch fewer per update)
__global__ void __launch_bounds__(CGM_T) k_cgm_init(mjrl_shape s, float* __restrict__ b, float* __restrict__ x,
                                                    float* __restrict__ r, float* __restrict__ p,
                                                    float* __restrict__ packed_p, float* cg, int32_t* __restrict__ done,
                                                    const float* __restrict__ gsum, double scale) {
    __shared__ double red[CGM_T / 64];
    const PackMap pm(s);
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f >= s.d) continue;
        float v;
        if (gsum) {
            v = (float)((double)gsum[f] * scale);
            b[f] = v;
        } else {
            v = b[f];
        }
        x[f] = 0.f;
        r[f] = v;
        p[f] = v;
        pack_one(pm, f, v, packed_p, false, 0.f);
        acc += (double)v * (double)v;
    }
    const double blk = block_sum<CGM_T>(acc, red);
    double t;
    if (threadIdx.x < 64 &&
        last_wg_fold(blk, reinterpret_cast<double*>(cg + 16), reinterpret_cast<unsigned*>(cg + 8), gridDim.x, t) &&
        threadIdx.x == 0) {
        cg[0] = (float)t;   // rdotr
        cg[1] = 0.f;        // iterations run
        *done = 0;
    }
}

// Step size and parameter update (npg_cg.py:128-141), over many workgroups:
// k_npgm_dot folds g.x (fixed order, last workgroup) and sets alpha / delta;
// k_npgm_apply writes theta + alpha x (log-std clamp) and its packed copy.
// out[MJRL_STEP_OUT]: out[0..2] results, out[8] ticket, out + 16 double partials.
__global__ void __launch_bounds__(CGM_T) k_npgm_dot(int d, const float* __restrict__ g, const float* __restrict__ x,
                                                    int mode, float delta, float alpha_in, int const_lr,
                                                    float* out) {
    __shared__ double red[CGM_T / 64];
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f < d) acc += (double)g[f] * (double)x[f];
    }
    const double blk = block_sum<CGM_T>(acc, red);
    double t;
    if (threadIdx.x < 64 &&
        last_wg_fold(blk, reinterpret_cast<double*>(out + 16), reinterpret_cast<unsigned*>(out + 8), gridDim.x, t) &&
        threadIdx.x == 0) {
        const float gx = (float)t;
        float alpha, dl = delta;
        if (mode == 0) {
            alpha = sqrtf(fabsf(delta / __fadd_rn(gx, 1e-20f)));
        } else {
            alpha = alpha_in;
            if (const_lr) dl = __fmul_rn(alpha * alpha, gx);
        }
        out[0] = alpha;
        out[1] = gx;
        out[2] = dl;
    }
}

// theta_new = theta + alpha x over this workgroup's elements, the log-std clamp of
// set_param_values, the packed copy
__device__ __forceinline__ void apply_step(const mjrl_shape& s, const float* __restrict__ x,
                                           const float* __restrict__ theta, float min_ls, float alpha,
                                           float* __restrict__ theta_new, float* __restrict__ packed_new) {
    const PackMap pm(s);
#pragma unroll
    for (int u = 0; u < CGM_U; ++u) {
        const int f = blockIdx.x * CGM_WG + u * CGM_T + threadIdx.x;
        if (f >= s.d) continue;
        float v = __fadd_rn(theta[f], __fmul_rn(alpha, x[f]));
        int p1, p2;
        if (pm.map(f, p1, p2) >= 0) v = v < min_ls ? min_ls : v;   // set_param_values clamp
        theta_new[f] = v;
        packed_new[p1] = v;
        if (p2 >= 0) packed_new[p2] = v;
    }
}

__global__ void __launch_bounds__(CGM_T) k_npgm_apply(mjrl_shape s, const float* __restrict__ x,
                                                      const float* __restrict__ theta, float min_ls,
                                                      float* __restrict__ theta_new, float* __restrict__ packed_new,
                                                      const float* __restrict__ out) {
    apply_step(s, x, theta, min_ls, out[0], theta_new, packed_new);
}

// TRPO's backtracking (trpo.py:105-118) on the device, trial k >= 1 of a line search:
// trial k - 1's evaluation (its sums) is logged and tested (kl < kl_dist, kl =
// float(sums[1] / T) as the host forms it); a rejected trial sets alpha_k =
// float32(0.9) * alpha_{k-1} in f32 (numpy 2: `0.9 * np.float32`) and writes theta +
// alpha_k x for the next evaluation, an accepted one raises *skip, so the remaining
// speculative trials and evaluations of the launch sequence return at once, and
// out[0] = the accepted alpha.
// apply = 0: log and test only (the sequence's last launch).  State ls (floats):
// [1] accepted, [2] trials logged, [8 + t] alpha_t (t >= 1; alpha_0 is out[0] of the
// mode-0 step), [MJRL_LS_LOG + 3 t ..] trial t's (alpha, kl, surr).
__global__ void __launch_bounds__(CGM_T) k_trpo_trial(mjrl_shape s, const float* __restrict__ x,
                                                      const float* __restrict__ theta, float min_ls,
                                                      float* __restrict__ theta_new, float* __restrict__ packed_new,
                                                      float* out, const double* __restrict__ sums,
                                                      double inv_T, double kl_dist, int k, int apply, float* ls,
                                                      int32_t* skip) {
    if (k > 1 && *skip) return;   // trial 1 starts the search: the flag is its to set
    const float a_prev = k == 1 ? out[0] : ls[8 + (k - 1)];
    const float kl = (float)(sums[1] * inv_T), surr = (float)(sums[0] * inv_T);
    const bool acc = (double)kl < kl_dist;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        float* lg = ls + MJRL_LS_LOG + 3 * (k - 1);
        lg[0] = a_prev;
        lg[1] = kl;
        lg[2] = surr;
        ls[1] = acc ? 1.f : 0.f;
        ls[2] = (float)k;
        *skip = acc ? 1 : 0;
        // the accepted alpha is the step's result (out[0], as a host step leaves it);
        // trial 1 writes the value its other workgroups read, unchanged
        if (acc) out[0] = a_prev;
        if (!acc && apply) ls[8 + k] = __fmul_rn(0.9f, a_prev);
    }
    if (acc || !apply) return;
    apply_step(s, x, theta, min_ls, __fmul_rn(0.9f, a_prev), theta_new, packed_new);
}

// Step size and parameter update (npg_cg.py:128-141), one workgroup (d beyond the
// multi-workgroup partials).
__global__ void __launch_bounds__(CG_THREADS) k_npg_step(mjrl_shape s, const float* __restrict__ g,
                                                         const float* __restrict__ x,
                                                         const float* __restrict__ theta, int mode, float delta,
                                                         float alpha_in, int const_lr, float min_ls,
                                                         float* __restrict__ theta_new, float* __restrict__ packed_new,
                                                         float* __restrict__ out) {
    __shared__ double red[CG_THREADS / 64];
    const PackMap pm(s);
    double acc = 0.0;
#pragma unroll 8
    for (int f = threadIdx.x; f < s.d; f += CG_THREADS) acc += (double)g[f] * (double)x[f];
    const float gx = (float)block_sum1024(acc, red);
    float alpha, dl = delta;
    if (mode == 0) {
        alpha = sqrtf(fabsf(delta / __fadd_rn(gx, 1e-20f)));
    } else {
        alpha = alpha_in;
        if (const_lr) dl = __fmul_rn(alpha * alpha, gx);
    }
#pragma unroll 8
    for (int f = threadIdx.x; f < s.d; f += CG_THREADS) {
        float v = __fadd_rn(theta[f], __fmul_rn(alpha, x[f]));
        int p1, p2;
        if (pm.map(f, p1, p2) >= 0) v = v < min_ls ? min_ls : v;   // set_param_values clamp
        theta_new[f] = v;
        packed_new[p1] = v;
        if (p2 >= 0) packed_new[p2] = v;
    }
    if (threadIdx.x == 0) {
        out[0] = alpha;
        out[1] = gx;
        out[2] = dl;
    }
}

// Generic CG for an arbitrary operator (the f_Ax of cg_solve.py:3): init and
// the update given z = A p computed by the caller.
__global__ void __launch_bounds__(CG_THREADS) k_cg_init_vec(int d, const float* __restrict__ b, float* __restrict__ x,
                                                            float* __restrict__ r, float* __restrict__ p,
                                                            float* __restrict__ cg, int32_t* __restrict__ done) {
    __shared__ double red[CG_THREADS / 64];
    double acc = 0.0;
    for (int f = threadIdx.x; f < d; f += CG_THREADS) {
        const float v = b[f];
        x[f] = 0.f;
        r[f] = v;
        p[f] = v;
        acc += (double)v * (double)v;
    }
    const double rr = block_sum1024(acc, red);
    if (threadIdx.x == 0) {
        cg[0] = (float)rr;
        cg[1] = 0.f;
        *done = 0;
    }
}

__global__ void __launch_bounds__(CG_THREADS) k_cg_update(int d, const float* __restrict__ z, float* __restrict__ x,
                                                          float* __restrict__ r, float* __restrict__ p,
                                                          float* __restrict__ cg, int32_t* __restrict__ done,
                                                          float tol) {
    __shared__ double red[CG_THREADS / 64];
    if (*done) return;
    double acc = 0.0;
    for (int f = threadIdx.x; f < d; f += CG_THREADS) acc += (double)p[f] * (double)z[f];
    const float pz = (float)block_sum1024(acc, red);
    const float rdotr = cg[0];
    const float v = rdotr / pz;
    acc = 0.0;
    for (int f = threadIdx.x; f < d; f += CG_THREADS) {
        x[f] = __fadd_rn(x[f], __fmul_rn(v, p[f]));
        const float rf = __fsub_rn(r[f], __fmul_rn(v, z[f]));
        r[f] = rf;
        acc += (double)rf * (double)rf;
    }
    const float rr = (float)block_sum1024(acc, red);
    const float mu = rr / rdotr;
    for (int f = threadIdx.x; f < d; f += CG_THREADS) p[f] = __fadd_rn(r[f], __fmul_rn(mu, p[f]));
    __syncthreads();
    if (threadIdx.x == 0) {
        cg[0] = rr;
        cg[1] += 1.f;
        cg[2] = v;
        cg[3] = mu;
        cg[4] = pz;
        if (rr < tol) *done = 1;
    }
}

inline int err(hipError_t e) { return e == hipSuccess ? MJRL_OK : (int)e; }

}  // namespace

extern "C" {

int mjrl_pack_params(const mjrl_shape* s, const float* theta, float* packed, int32_t clamp_log_std,
                     float min_log_std, void* stream) {
    if (!s || !theta || !packed) return MJRL_EINVAL;
    hipLaunchKernelGGL(k_pack, dim3((s->d + 255) / 256), dim3(256), 0, (hipStream_t)stream, *s, theta, packed,
                       clamp_log_std, min_log_std);
    return err(hipGetLastError());
}

int mjrl_cg_init(const mjrl_shape* s, const float* b, float* x, float* r, float* p, float* packed_p, float* cg,
                 int32_t* done, void* stream) {
    if (!s || !b || !x || !r || !p || !packed_p || !cg || !done) return MJRL_EINVAL;
    const int nwg = (s->d + CGM_WG - 1) / CGM_WG;
    if (nwg <= CGM_MAXWG && nwg > 0) {
        hipLaunchKernelGGL(k_cgm_init, dim3(nwg), dim3(CGM_T), 0, (hipStream_t)stream, *s, const_cast<float*>(b), x, r,
                           p, packed_p, cg, done, (const float*)nullptr, 0.0);
        return err(hipGetLastError());
    }
    hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(CG_THREADS), 0, (hipStream_t)stream, *s, b, x, r, p, packed_p, cg,
                       done);
    return err(hipGetLastError());
}

int mjrl_cg_init_scaled(const mjrl_shape* s, const float* gsum, double scale, float* g, float* x, float* r, float* p,
                        float* packed_p, float* cg, int32_t* done, void* stream) {
    if (!s || !gsum || !g || !x || !r || !p || !packed_p || !cg || !done) return MJRL_EINVAL;
    const int nwg = (s->d + CGM_WG - 1) / CGM_WG;
    if (nwg <= CGM_MAXWG && nwg > 0) {
        hipLaunchKernelGGL(k_cgm_init, dim3(nwg), dim3(CGM_T), 0, (hipStream_t)stream, *s, g, x, r, p, packed_p, cg,
                           done, gsum, scale);
        return err(hipGetLastError());
    }
    // beyond the multi-workgroup partials: the two launches
    const int rc = mjrl_scale_vec(gsum, s->d, scale, g, stream);
    if (rc != MJRL_OK) return rc;
    return mjrl_cg_init(s, g, x, r, p, packed_p, cg, done, stream);
}

int mjrl_cg_step_xr_p(const mjrl_shape* s, float* x, const float* r, float* r_out, float* p, const float* z,
                      float* packed_p, float* cg, int32_t* done, float residual_tol, void* stream) {
    if (!s || !x || !r || !r_out || r_out == r || !p || !z || !packed_p || !cg || !done) return MJRL_EINVAL;
    const int ng = (s->d + 63) / 64;   // the fused gather's workgroups
    if (ng > CG_PZ_MAX) return MJRL_EINVAL;
    // every term of the r.r fold in flight at once up to d = 32768 (Humanoid: 29,410);
    // small d keeps 8, its masked loads past d would cost more than they hide
    if (s->d > 8 * CGX_T)
        hipLaunchKernelGGL(k_cgm_xrp_f<32>, dim3((s->d + CGX_T - 1) / CGX_T), dim3(CGX_T), 0, (hipStream_t)stream, *s,
                           p, z, x, r, r_out, packed_p, cg, done, residual_tol, ng);
    else
        hipLaunchKernelGGL(k_cgm_xrp_f<8>, dim3((s->d + CGX_T - 1) / CGX_T), dim3(CGX_T), 0, (hipStream_t)stream, *s,
                           p, z, x, r, r_out, packed_p, cg, done, residual_tol, ng);
    return err(hipGetLastError());
}

int mjrl_cg_z(const mjrl_shape* s, const float* gsum, double inv_T, float damping, const float* packed_theta,
              const float* p, float* z, float* cg, const int32_t* done, void* stream) {
    if (!s || !gsum || !packed_theta || !p || !z || !cg || !done) return MJRL_EINVAL;
    const int ng = (s->d + 63) / 64;
    if (ng > CG_PZ_MAX) return MJRL_EINVAL;
    const Packed pk(s->h0, s->h1, s->np, s->mp);
    CgZ cz{p, z, cg, packed_theta + pk.ls, inv_T, damping, s->d - s->m};
    hipLaunchKernelGGL(k_cg_zpart, dim3(ng), dim3(64), 0, (hipStream_t)stream, s->d, gsum, done, cz);
    return err(hipGetLastError());
}

int mjrl_cg_step(const mjrl_shape* s, const float* gsum, double inv_T, float damping, const float* packed_theta,
                 float* x, float* r, float* p, float* z, float* packed_p, float* cg, int32_t* done,
                 float residual_tol, void* stream) {
    if (!s || !gsum || !packed_theta || !x || !r || !p || !z || !packed_p || !cg || !done) return MJRL_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const int nwg = (s->d + CGM_WG - 1) / CGM_WG;
    if (nwg > CGM_MAXWG) {   // beyond the partials the state holds: the single-workgroup form
        hipLaunchKernelGGL(k_cg_step, dim3(1), dim3(CG_THREADS), 0, st, *s, gsum, inv_T, damping, packed_theta, x, r,
                           p, z, packed_p, cg, done, residual_tol);
        return err(hipGetLastError());
    }
    hipLaunchKernelGGL(k_cgm_z, dim3(nwg), dim3(CGM_T), 0, st, *s, gsum, inv_T, damping, packed_theta, p, z, cg, done);
    hipLaunchKernelGGL(k_cgm_xr, dim3(nwg), dim3(CGM_T), 0, st, s->d, p, z, x, r, cg, done, residual_tol);
    hipLaunchKernelGGL(k_cgm_p, dim3(nwg), dim3(CGM_T), 0, st, *s, r, p, packed_p, cg, done);
    return err(hipGetLastError());
}

int mjrl_cg_step1(const mjrl_shape* s, const float* gsum, double inv_T, float damping, const float* packed_theta,
                  float* x, const float* r, float* r_out, const float* p, float* p_out, float* packed_p, float* cg,
                  int32_t* done, float residual_tol, void* stream) {
    if (!s || !gsum || !packed_theta || !x || !r || !r_out || !p || !p_out || !packed_p || !cg || !done) return MJRL_EINVAL;
    if (r_out == r || p_out == p) return MJRL_EINVAL;
    hipLaunchKernelGGL(k_cgm_step1, dim3((s->d + CGX_T - 1) / CGX_T), dim3(CGX_T), 0, (hipStream_t)stream, *s, gsum,
                       inv_T, damping, packed_theta, x, r, r_out, p, p_out, packed_p, cg, done, residual_tol);
    return err(hipGetLastError());
}

int mjrl_cg_init_vec(int32_t d, const float* b, float* x, float* r, float* p, float* cg, int32_t* done,
                     void* stream) {
    if (d < 0 || !b || !x || !r || !p || !cg || !done) return MJRL_EINVAL;
    hipLaunchKernelGGL(k_cg_init_vec, dim3(1), dim3(CG_THREADS), 0, (hipStream_t)stream, d, b, x, r, p, cg, done);
    return err(hipGetLastError());
}

int mjrl_cg_update(int32_t d, const float* z, float* x, float* r, float* p, float* cg, int32_t* done,
                   float residual_tol, void* stream) {
    if (d < 0 || !z || !x || !r || !p || !cg || !done) return MJRL_EINVAL;
    hipLaunchKernelGGL(k_cg_update, dim3(1), dim3(CG_THREADS), 0, (hipStream_t)stream, d, z, x, r, p, cg, done,
                       residual_tol);
    return err(hipGetLastError());
}

int mjrl_trpo_trial(const mjrl_shape* s, const float* x, const float* theta, float min_log_std, float* theta_new,
                    float* packed_new, float* out, const double* sums, double inv_T, double kl_dist, int32_t k,
                    int32_t apply, float* ls, int32_t* skip, void* stream) {
    if (!s || !x || !theta || !theta_new || !packed_new || !out || !sums || !ls || !skip || k < 1 ||
        k + 8 >= MJRL_LS_LOG || MJRL_LS_LOG + 3 * k > MJRL_LS_STATE)
        return MJRL_EINVAL;
    const int nwg = (s->d + CGM_WG - 1) / CGM_WG;
    hipLaunchKernelGGL(k_trpo_trial, dim3(nwg > 0 ? nwg : 1), dim3(CGM_T), 0, (hipStream_t)stream, *s, x, theta,
                       min_log_std, theta_new, packed_new, out, sums, inv_T, kl_dist, (int)k, (int)apply, ls, skip);
    return err(hipGetLastError());
}

int mjrl_npg_step(const mjrl_shape* s, const float* g, const float* x, const float* theta, int32_t mode, float delta,
                  float alpha_in, int32_t const_lr, float min_log_std, float* theta_new, float* packed_new,
                  float* out, void* stream) {
    if (!s || !g || !x || !theta || !theta_new || !packed_new || !out) return MJRL_EINVAL;
    const int nwg = (s->d + CGM_WG - 1) / CGM_WG;
    hipStream_t st = (hipStream_t)stream;
    if (nwg <= (MJRL_STEP_OUT - 16) / 2 && nwg > 0) {
        hipLaunchKernelGGL(k_npgm_dot, dim3(nwg), dim3(CGM_T), 0, st, s->d, g, x, mode, delta, alpha_in, const_lr, out);
        hipLaunchKernelGGL(k_npgm_apply, dim3(nwg), dim3(CGM_T), 0, st, *s, x, theta, min_log_std, theta_new,
                           packed_new, (const float*)out);
        return err(hipGetLastError());
    }
    hipLaunchKernelGGL(k_npg_step, dim3(1), dim3(CG_THREADS), 0, st, *s, g, x, theta, mode, delta, alpha_in, const_lr,
                       min_log_std, theta_new, packed_new, out);
    return err(hipGetLastError());
}

}  // extern "C"
