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
    hipFree(in);
    hipFree(out);
    return 0;
}
