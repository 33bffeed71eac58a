// rollout.hip — the batched policy forward of vectorised sampling (SURVEY.md §8f
// row f3): the mean action of the Gaussian policy for the current observation of
// every environment of a lock-stepped batch, one launch per environment step.
//
// Reference: mjrl/policies/gaussian_mlp.py:92-98 (get_action: the mean of
// MuNet.forward, :168-182, plus host noise) and gaussian_linear.py; the loop it
// serves is mjrl/samplers/base_sampler.py:64-74.  Latency-bound (a few hundred
// rows): one 64-lane wave per row, 4 rows per workgroup, the row's activations in
// LDS, weights from the packed parameter set (L2-resident across steps).  fp32
// dot products per output unit in index order.
#include "common.h"

using namespace mjrl;

namespace {

constexpr int ACT_ROWS = 4;   // rows (waves) per workgroup

__global__ void __launch_bounds__(64 * ACT_ROWS) k_policy_mean(mjrl_shape s, const float* __restrict__ obs, int64_t N,
                                                              const float* __restrict__ P,
                                                              const float* __restrict__ in_shift,
                                                              const float* __restrict__ in_scale,
                                                              const float* __restrict__ out_shift,
                                                              const float* __restrict__ out_scale,
                                                              float* __restrict__ mean) {
    extern __shared__ float sm[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = s.n, m = s.m, np = s.np, h0 = s.h0, h1 = s.h1;
    const Packed pk(h0, h1, np, s.mp);
    const int64_t row = (int64_t)blockIdx.x * ACT_ROWS + w;
    const bool live = row < N;
    float* xs = sm + w * (np + h0 + h1);
    float* a0 = xs + np;
    float* a1 = a0 + h0;
    // xhat = (obs - in_shift) / (in_scale + 1e-8), bias column n = 1 (MuNet.forward:177)
    for (int c = lane; c < np; c += 64) {
        float x = 0.f;
        if (live && c < n) {
            x = obs[row * n + c];
            if (in_shift) x = (x - in_shift[c]) / (in_scale[c] + 1e-8f);
        } else if (c == n) {
            x = 1.f;
        }
        xs[c] = x;
    }
    __syncthreads();
    if (h0 == 0) {   // linear policy: Wp [MP][NP] with the bias in column n
        for (int j = lane; j < m; j += 64) {
            float acc = 0.f;
            for (int k = 0; k < np; ++k) acc += P[pk.W0 + j * np + k] * xs[k];
            if (live) mean[row * m + j] = out_scale ? acc * out_scale[j] + out_shift[j] : acc;
        }
        return;
    }
    for (int j = lane; j < h0; j += 64) {   // tanh(fc0): W0 [h0][np], b0 in column n
        float acc = 0.f;
        for (int k = 0; k < np; ++k) acc += P[pk.W0 + j * np + k] * xs[k];
        a0[j] = tanhf(acc);
    }
    __syncthreads();
    for (int j = lane; j < h1; j += 64) {   // tanh(fc1): W1T [h0][h1] (coalesced over j)
        float acc = 0.f;
        for (int k = 0; k < h0; ++k) acc += P[pk.W1T + k * h1 + j] * a0[k];
        a1[j] = tanhf(acc + P[pk.b1 + j]);
    }
    __syncthreads();
    for (int j = lane; j < m; j += 64) {    // fc2, de-normalised: W2T [h1][mp]
        float acc = 0.f;
        for (int k = 0; k < h1; ++k) acc += P[pk.W2T + k * s.mp + j] * a1[k];
        acc += P[pk.b2 + j];
        if (live) mean[row * m + j] = out_scale ? acc * out_scale[j] + out_shift[j] : acc;
    }
}

}  // namespace

extern "C" {

int mjrl_policy_mean(const mjrl_shape* s, const float* obs, int64_t N, const float* packed_theta,
                     const float* in_shift, const float* in_scale, const float* out_shift, const float* out_scale,
                     float* mean, void* stream) {
    if (!s || !packed_theta || !mean || N < 0 || (N > 0 && !obs)) return MJRL_EINVAL;
    if ((in_shift == nullptr) != (in_scale == nullptr) || (out_shift == nullptr) != (out_scale == nullptr))
        return MJRL_EINVAL;
    if (N == 0) return MJRL_OK;
    const size_t lds = (size_t)ACT_ROWS * (s->np + s->h0 + s->h1) * sizeof(float);
    const int64_t g = (N + ACT_ROWS - 1) / ACT_ROWS;
    hipLaunchKernelGGL(k_policy_mean, dim3((unsigned)g), dim3(64 * ACT_ROWS), lds, (hipStream_t)stream, *s, obs, N,
                       packed_theta, in_shift, in_scale, out_shift, out_scale, mean);
    return (int)hipGetLastError();
}

}  // extern "C"
