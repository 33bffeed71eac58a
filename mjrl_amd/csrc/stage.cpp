// stage.cpp — host side of the sampler paths -> HBM staging.
//
// The reference concatenates every path's f64 observations (npg_cg.py:87-89) and
// the policy casts them to f32 on every forward (gaussian_mlp.py:103).  Staging
// does that cast once, on the host thread pool, straight into a pinned slab, and
// takes each column's range in the same pass: the split rows' column scales then
// need no device pass over the batch (mjrl_obs_colscale_range), and the pack of a
// chunk never waits for a whole-batch reduction on the device.  Plain C++ built
// with g++ into libmjrl_amd.so; loops the compiler vectorises (min / max written
// as the compare-select that maps to minps / maxps, NaN skipped).
#include <cstdint>

#include "../../include/mjrl_amd.h"

namespace {

template <typename S>
int stage_rows(const S* __restrict__ src, int64_t rows, int32_t n, float* __restrict__ dst, float* __restrict__ cmin,
               float* __restrict__ cmax) {
    if (rows < 0 || n <= 0 || (rows > 0 && (!src || !dst))) return MJRL_EINVAL;
    if ((cmin == nullptr) != (cmax == nullptr)) return MJRL_EINVAL;
    const int64_t ne = rows * (int64_t)n;
    if (!cmin) {
        for (int64_t i = 0; i < ne; ++i) dst[i] = (float)src[i];
        return MJRL_OK;
    }
    for (int64_t r = 0; r < rows; ++r) {
        const S* __restrict__ s = src + r * n;
        float* __restrict__ d = dst + r * n;
        for (int32_t k = 0; k < n; ++k) {
            const float v = (float)s[k];
            d[k] = v;
            const float lo = cmin[k], hi = cmax[k];
            cmin[k] = v < lo ? v : lo;   // a NaN compares false: skipped
            cmax[k] = v > hi ? v : hi;
        }
    }
    return MJRL_OK;
}

}  // namespace

extern "C" {

int mjrl_host_stage_f64(const double* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    return stage_rows(src, rows, n, dst, cmin, cmax);
}

int mjrl_host_stage_f32(const float* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax) {
    return stage_rows(src, rows, n, dst, cmin, cmax);
}

}  // extern "C"
