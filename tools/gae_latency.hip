// Microbenchmark of the GAE scan's serial step on gfx950:
// the dependent fp64 multiply -> add (discount_sum's acc = x + c * acc, no FMA),
// alone and with what k_gae does around it per step.  One wave, lanes 0-2 active
// (k_gae's three chains), N steps, timed with HIP events over the launch.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/gae_latency.hip -o /tmp/gae_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int GU = 32;

template <int MODE>
__global__ void __launch_bounds__(64) k_chain(const double* __restrict__ in, double* __restrict__ out, int nb,
                                              double c) {
    __shared__ double src[2048];
    __shared__ double dst[2048];
    const int lane = threadIdx.x;
    for (int i = lane; i < 2048; i += 64) src[i] = in[i];
    __syncthreads();
    if (lane < (MODE == 8 ? 64 : 3)) {
        double acc = 0.0;
        double xv[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) xv[u] = src[u + lane];
        for (int j = 0; j < nb; ++j) {
            const int base = (j * GU) & 1023;
            if (MODE == 0) {   // registers only: the dependent multiply -> add
#pragma unroll
                for (int u = 0; u < GU; ++u) acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
            } else if (MODE == 1) {   // + one LDS store per step (k_gae's)
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    dst[base + u + lane * 0] = acc;
                }
            } else if (MODE == 2) {   // + the next batch's LDS reads in flight (k_gae's pipelining)
                double xn[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) xn[u] = src[((j + 1) * GU + u) & 1023];
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    dst[base + u] = acc;
                }
#pragma unroll
                for (int u = 0; u < GU; ++u) xv[u] = xn[u];
            } else if (MODE == 3) {   // outputs kept in registers, stored once per batch
                double o[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    o[u] = acc;
                }
#pragma unroll
                for (int u = 0; u < GU; ++u) dst[base + u] = o[u];
            } else if (MODE == 4) {   // fused multiply-add (NOT the reference's rounding: latency only)
#pragma unroll
                for (int u = 0; u < GU; ++u) acc = __fma_rn(c, acc, xv[u]);
            } else if (MODE == 6) {   // outputs of batch j - 1 stored while batch j's chain runs
                double o[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    o[u] = acc;
                    if (u % 8 == 7) {
#pragma unroll
                        for (int q = u - 7; q <= u; ++q) dst[((base + q) & 1023)] = o[q];
                    }
                }
            } else if (MODE == 7) {   // outputs to global memory, one batch of stores
                double o[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    o[u] = acc;
                }
#pragma unroll
                for (int u = 0; u < GU; ++u) out[64 + ((base + u) & 1023) * 4 + lane] = o[u];
            } else if (MODE == 8) {   // mul -> add with every lane active (lane count)
#pragma unroll
                for (int u = 0; u < GU; ++u) acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
            } else if (MODE == 5) {   // two independent chains interleaved (latency vs issue)
                double acc2 = acc;
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    acc = __dadd_rn(xv[u], __dmul_rn(c, acc));
                    acc2 = __dadd_rn(xv[GU - 1 - u], __dmul_rn(c, acc2));
                }
                acc += acc2;
            }
        }
        out[lane] = acc + dst[lane & 1023];
    }
}

template <int MODE>
float run(const double* in, double* out, int nb, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, in, out, nb, 0.995);
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, 0, in, out, nb, 0.995);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}


// k_gae_lp's chain-wave pattern (round 6): lanes = paths, each lane its own LDS row
// (stride 257 doubles: conflict-free), 16-step batches, the reads of batch k + 2
// issued before batch k's steps.  NL lanes active; MODE 0 reads + writes back (the
// kernel's pattern), 1 reads only, 2 writes only, 3 reads + outputs to global
// (dwordx2 per step, lane rows in HBM), 4 registers only.
constexpr int RW = 256, RLD = 257, RB = 16;
template <int MODE, int NL>
__global__ void __launch_bounds__(64) k_lane(double* __restrict__ out, int nw, double c) {
    __shared__ double row_s[NL * RLD];
    const int lane = threadIdx.x;
    for (int i = lane; i < NL * RLD; i += 64) row_s[i] = 0.001 * (i % 97) - 0.03;
    __syncthreads();
    if (lane >= NL) return;
    double* row = row_s + lane * RLD;
    double acc = 0.0;
    double* o = out + 64 + (size_t)lane * RW;
    for (int j = 0; j < nw; ++j) {
        constexpr int NB = RW / RB;
        double X[3][RB];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
#pragma unroll
            for (int g = 0; g < RB; ++g) X[k][g] = (MODE == 2 || MODE == 4) ? 0.5 * g : row[RW - (k + 1) * RB + g];
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k + 2 < NB && MODE != 2 && MODE != 4) {
#pragma unroll
                for (int g = 0; g < RB; ++g) X[(k + 2) % 3][g] = row[RW - (k + 3) * RB + g];
            } else if (k + 2 < NB) {
#pragma unroll
                for (int g = 0; g < RB; ++g) X[(k + 2) % 3][g] = 0.25 * g + k;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int g = RB - 1; g >= 0; --g) {
                acc = __dadd_rn(X[k % 3][g], __dmul_rn(c, acc));
                X[k % 3][g] = acc;
            }
            __builtin_amdgcn_sched_barrier(0);
            if (MODE == 0 || MODE == 2) {
#pragma unroll
                for (int g = 0; g < RB; ++g) row[RW - (k + 1) * RB + g] = X[k % 3][g];
            } else if (MODE == 3) {
#pragma unroll
                for (int g = 0; g < RB; ++g) o[RW - (k + 1) * RB + g] = X[k % 3][g];
            }
        }
    }
    out[lane] = acc + row[lane & 7];
}

template <int MODE, int NL>
float run_lane(double* out, int nw, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_lane<MODE, NL>), dim3(1), dim3(64), 0, 0, out, nw, 0.995);
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_lane<MODE, NL>), dim3(1), dim3(64), 0, 0, out, nw, 0.995);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    double *in, *out;
    hipMalloc(&in, 2048 * sizeof(double));
    hipMalloc(&out, (64 + 4096) * sizeof(double));
    double h[2048];
    for (int i = 0; i < 2048; ++i) h[i] = 0.001 * (i % 97) - 0.03;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    const int nb = 4096;   // 131072 steps per launch
    const char* names[] = {"mul->add registers", "+ LDS store per step", "+ next batch LDS reads (k_gae)",
                           "outputs in registers, one store batch", "fma (latency only)",
                           "two chains interleaved (per chain step)", "outputs stored every 8 steps",
                           "outputs to global, one store batch", "mul->add, all 64 lanes active"};
    constexpr int NM = 9;
    float t[NM];
    for (int pass = 0; pass < 2; ++pass) {
        t[0] = run<0>(in, out, nb, 5);
        t[1] = run<1>(in, out, nb, 5);
        t[2] = run<2>(in, out, nb, 5);
        t[3] = run<3>(in, out, nb, 5);
        t[4] = run<4>(in, out, nb, 5);
        t[5] = run<5>(in, out, nb, 5);
        t[6] = run<6>(in, out, nb, 5);
        t[7] = run<7>(in, out, nb, 5);
        t[8] = run<8>(in, out, nb, 5);
    }
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("gfx950 serial fp64 chain, one wave, %d steps per launch, shader clock %.0f MHz\n", nb * GU, clk / 1e3);
    for (int i = 0; i < NM; ++i) {
        const double ns = t[i] * 1e6 / (nb * GU);
        printf("%-42s %7.3f ns/step  %6.1f cycles/step\n", names[i], ns, ns * clk / 1e6);
    }
    // the lanes = paths chain of k_gae_lp (one wave, nw windows of 256 steps)
    double* out2;
    hipMalloc(&out2, (64 + 64 * RW) * sizeof(double));
    const int nw = 512;
    const char* lnames[] = {"lanes: 8 paths, LDS reads + writes (k_gae_lp)", "lanes: 8 paths, LDS reads only",
                            "lanes: 8 paths, LDS writes only", "lanes: 8 paths, LDS reads, outputs to global",
                            "lanes: 64 paths, LDS reads + writes", "lanes: 8 paths, registers only"};
    float lt[6];
    for (int pass = 0; pass < 2; ++pass) {
        lt[0] = run_lane<0, 8>(out2, nw, 5);
        lt[1] = run_lane<1, 8>(out2, nw, 5);
        lt[2] = run_lane<2, 8>(out2, nw, 5);
        lt[3] = run_lane<3, 8>(out2, nw, 5);
        lt[4] = run_lane<0, 64>(out2, nw, 5);
        lt[5] = run_lane<4, 8>(out2, nw, 5);
    }
    for (int i = 0; i < 6; ++i) {
        const double ns = lt[i] * 1e6 / (nw * RW);
        printf("%-46s %7.3f ns/step  %6.1f cycles/step\n", lnames[i], ns, ns * clk / 1e6);
    }
    hipFree(out2);
    hipFree(in);
    hipFree(out);
    return 0;
}
