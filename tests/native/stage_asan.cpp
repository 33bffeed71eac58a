// Host AddressSanitizer check of the staging conversion (csrc/stage.cpp): every
// path (AVX-512 when the CPU has it, the portable loop, the batched per-chunk call)
// over exactly-sized heap buffers, for column counts with and without a masked
// vector tail, destinations at every float misalignment of a 64-byte line, and
// row counts that leave a partial block.  Built and run by tests/test_staging.py;
// exits non-zero on a mismatch (ASan aborts on an out-of-bounds access).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../mjrl_amd/csrc/stage.cpp"

static int check(int n, int rows, int shift) {
    std::vector<double> src((size_t)rows * n);
    for (size_t i = 0; i < src.size(); ++i) src[i] = std::sin(0.37 * (double)i) * std::pow(10.0, (int)(i % n) % 7 - 3);
    float* raw = static_cast<float*>(std::malloc(sizeof(float) * ((size_t)rows * n + shift)));
    float* dst = raw + shift;   // exactly rows * n floats past the shift
    float* ref = static_cast<float*>(std::malloc(sizeof(float) * (size_t)rows * n));
    float* lo = static_cast<float*>(std::malloc(sizeof(float) * n));
    float* hi = static_cast<float*>(std::malloc(sizeof(float) * n));
    float* lo2 = static_cast<float*>(std::malloc(sizeof(float) * n));
    float* hi2 = static_cast<float*>(std::malloc(sizeof(float) * n));
    for (int k = 0; k < n; ++k) lo[k] = lo2[k] = INFINITY, hi[k] = hi2[k] = -INFINITY;
    int bad = 0;
    bad |= mjrl_host_stage_f64(src.data(), rows, n, dst, lo, hi);
    bad |= mjrl_host_stage_f64_portable(src.data(), rows, n, ref, lo2, hi2);
    bad |= std::memcmp(dst, ref, sizeof(float) * (size_t)rows * n) != 0;
    bad |= std::memcmp(lo, lo2, sizeof(float) * n) != 0 || std::memcmp(hi, hi2, sizeof(float) * n) != 0;
    // the batched call over three pieces of the same rows
    const int r1 = rows / 3, r2 = rows / 2;
    const double* srcs[3] = {src.data(), src.data() + (size_t)r1 * n, src.data() + (size_t)r2 * n};
    const int64_t rr[3] = {r1, r2 - r1, rows - r2};
    std::memset(dst, 0, sizeof(float) * (size_t)rows * n);
    bad |= mjrl_host_stage_paths_f64(srcs, rr, 3, n, dst, nullptr, nullptr);
    bad |= std::memcmp(dst, ref, sizeof(float) * (size_t)rows * n) != 0;
    // no range, and the f32 source
    std::memset(dst, 0, sizeof(float) * (size_t)rows * n);
    bad |= mjrl_host_stage_f64(src.data(), rows, n, dst, nullptr, nullptr);
    bad |= std::memcmp(dst, ref, sizeof(float) * (size_t)rows * n) != 0;
    std::memset(dst, 0, sizeof(float) * (size_t)rows * n);
    bad |= mjrl_host_stage_f32(ref, rows, n, dst, lo, hi);
    bad |= std::memcmp(dst, ref, sizeof(float) * (size_t)rows * n) != 0;
    std::free(raw); std::free(ref); std::free(lo); std::free(hi); std::free(lo2); std::free(hi2);
    if (bad) std::printf("mismatch n=%d rows=%d shift=%d\n", n, rows, shift);
    return bad;
}

int main() {
    int bad = 0;
    const int ns[] = {1, 15, 16, 17, 37, 191, 192, 193, 376, 9000};
    for (int n : ns)
        for (int rows : {1, 7, 64})
            for (int shift = 0; shift < 16; shift += 5) bad |= check(n, n > 1000 ? 2 : rows, shift);
    std::printf("stage_asan avx512=%d %s\n", mjrl_host_stage_avx512(), bad ? "FAILED" : "ok");
    return bad;
}
