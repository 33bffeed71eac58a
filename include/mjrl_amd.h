/*
 * mjrl_amd.h — C ABI of the MI355X (gfx950) NPG / TRPO / DAPG update path.
 *
 * Drop-in boundary for bennevans/mjrl's per-iteration policy update.  The
 * reference is pure Python (no FFI); each entry point below replaces one
 * reference function, cited as path:line under the reference tree, and a
 * maintainer would bind them from Python with ctypes.
 *
 * Conventions (all entry points):
 *   - every pointer is DEVICE memory owned by the caller (hipMalloc / torch);
 *   - every call is stream-ordered on the caller's `stream` (a hipStream_t,
 *     passed as void*), never synchronises, never allocates, never throws;
 *   - return 0 on success, a negative MJRL_E* code on bad arguments, or a
 *     positive hipError_t if a launch failed;
 *   - reductions are deterministic (fixed order, no float atomics).
 *
 * Device data layout:
 *   rows t = 0..T-1 are the concatenated timesteps of the caller's paths
 *   (np.concatenate order, mjrl/algos/npg_cg.py:87-89);
 *   NP = round_up(n + 1, 16): xhat[T][NP] holds the normalised observation in
 *   columns 0..n-1, 1.0 in column n (the bias column) and zeros after;
 *   MP = round_up(m, 16) (m <= 64);  hidden sizes h0, h1 in {32, 64, 128, 256},
 *   or h0 = h1 = 0 for the linear policy (mjrl/policies/gaussian_linear.py).
 *   The flat parameter vector theta[d] is in the reference's trainable_params
 *   order [W0(h0 x n), b0, W1(h1 x h0), b1, W2(m x h1), b2, log_std]
 *   (mjrl/policies/gaussian_mlp.py:33-38, 61-64).
 */
#ifndef MJRL_AMD_H
#define MJRL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MJRL_OK 0
#define MJRL_EINVAL (-1)      /* bad argument (null pointer, negative size) */
#define MJRL_ESHAPE (-2)      /* policy shape not supported by the kernels */

/* Policy shape and the padded sizes every buffer is laid out with. */
typedef struct mjrl_shape {
    int32_t n, m;             /* obs_dim, act_dim */
    int32_t h0, h1;           /* hidden sizes; 0, 0 = linear policy */
    int32_t np, mp;           /* padded: round_up(n+1,16), round_up(m,16) */
    int32_t d;                /* flat parameter count */
    int32_t packed;           /* floats in one packed parameter set */
} mjrl_shape;

/* Row-local buffers of one shard (all device, row-major, T rows). */
typedef struct mjrl_rows {
    int64_t T;                /* rows in this shard */
    const float* xhat;        /* [T][np] */
    const float* act;         /* [T][m]  actions, f32 */
    const float* adv;         /* [T]     whitened advantages, f32 (surrogate) */
    const float* adv_vpg;     /* [T]     advantages driving the VPG (DAPG: all_adv) */
    float* a0;                /* [T][h0] cached tanh activations (layer 0) */
    float* a1;                /* [T][h1] cached tanh activations (layer 1) */
    float* mu0;               /* [T][m]  cached means at the old parameters */
    float* ll0;               /* [T]     cached log-likelihoods at the old parameters */
    float* gu0;               /* [T][h0] per-row upstream gradient at layer 0 */
    float* gu1;               /* [T][h1] per-row upstream gradient at layer 1 */
    float* gp;                /* [T][mp] per-row upstream gradient at the output */
    /* Split-f16 observation rows (alternative to xhat, MLP(64,64) with np % 128 == 0,
     * see mjrl_split_supported): row t = [hi np][lo np] f16 of
     * y[t][k] = xhat[t][k] / (xc[k] xu[t]), hi = f16(y), lo = f16(y - hi);
     * xc[k] a power of two per column (mjrl_obs_colscale), xu[t] a power of two per
     * row with max_k |y[t][k]| in [2^14, 2^15).  Element bound:
     * |xc xu (hi + lo) - xhat| <= 2^-23 |xhat| + 2^-38 colmax_k, colmax_k the
     * column's max |xhat| over the batch.
     * When xs is non-null the policy passes read xs / xu / xc and ignore xhat. */
    const void* xs;           /* [T][2][np] f16 */
    const float* xu;          /* [T] */
    const float* xc;          /* [np] */
} mjrl_rows;

/* Scratch the caller allocates once per (shape, T) — sizes from
 * mjrl_scratch_size(). */
typedef struct mjrl_scratch {
    float* wpart;             /* weight-gradient partial slabs */
    double* rpart;            /* per-workgroup scalar partials */
    int32_t slices;           /* T-slices of the weight-gradient reduction */
} mjrl_scratch;

/* Fills padded sizes / d / packed-set size for a policy shape.
 * Returns MJRL_ESHAPE if the kernels were not built for it. */
int mjrl_shape_init(mjrl_shape* s, int32_t n, int32_t m, int32_t h0, int32_t h1);

/* Build variant of the loaded library (bits): MJRL_BUILD_ABLATION = a timing-
 * ablation build (tools/fvp_time.py; its results are wrong by construction: the
 * engine refuses it unless MJRL_AMD_ALLOW_ABLATION=1), MJRL_BUILD_PROF = the
 * phase-profiling build, MJRL_BUILD_CHECKS = the slab-guard debug build. */
#define MJRL_BUILD_ABLATION 1
#define MJRL_BUILD_PROF 2
#define MJRL_BUILD_CHECKS 4
int mjrl_build_flags(void);

/* Scratch sizes (in elements) for T rows: *wpart_floats, *rpart_doubles; also
 * returns the T-slice count the kernels will use. */
int mjrl_scratch_size(const mjrl_shape* s, int64_t T, int64_t* wpart_floats,
                      int64_t* rpart_doubles, int32_t* slices);

/* ---- batch assembly (npg_cg.py:87-89 concatenate + gaussian_mlp.py:103,177) ----
 * obs f64 [T][n] -> xhat f32 [T][np] = (float(obs) - in_shift) / (in_scale + 1e-8),
 * bias column 1.0, zero padding; act f64 [T][m] -> act32 f32 [T][m]. */
int mjrl_pack_batch(const double* obs, const double* act, int64_t T, const mjrl_shape* s,
                    const float* in_shift, const float* in_scale, float* xhat, float* act32,
                    void* stream);

/* Column scales of the split form: xc[k] = 2^E with max_t |xhat[t][k]| 2^-E in
 * [1/2, 1) (1 for an all-zero column; the bias column's max is 1).  One pass over
 * the observations (xhat computed as mjrl_pack_batch does); xc holds np floats. */
int mjrl_obs_colscale(const double* obs, int64_t T, const mjrl_shape* s, const float* in_shift,
                      const float* in_scale, float* xc, void* stream);
int mjrl_obs_colscale_f32(const float* obs, int64_t T, const mjrl_shape* s, const float* in_shift,
                          const float* in_scale, float* xc, void* stream);
/* The same xc from per-column ranges of the f32 observations, cmin[n] / cmax[n]
 * (device), as the host staging pass takes them (mjrl_host_stage_*): the
 * normalisation is monotone in x, so the column max of |xhat| sits at one end of
 * the range and xc equals mjrl_obs_colscale's bit for bit, without a pass over
 * the batch.  cmin[k] > cmax[k] marks an empty range (scale 1). */
int mjrl_obs_colscale_range(const float* cmin, const float* cmax, const mjrl_shape* s, const float* in_shift,
                            const float* in_scale, float* xc, void* stream);
/* Same batch assembly into the split-f16 form of mjrl_rows.xs / xu, given the
 * column scales xc of mjrl_obs_colscale (one wave per row: the row's max
 * |xhat / xc| picks xu[t], then hi / lo as described at mjrl_rows).  Only for
 * shapes with mjrl_split_supported(s). */
int mjrl_pack_batch_split(const double* obs, const double* act, int64_t T, const mjrl_shape* s,
                          const float* in_shift, const float* in_scale, const float* xc, void* xs,
                          float* xu, float* act32, void* stream);
/* The same two with observations / actions staged as f32 by the host (the
 * policy's own input precision: gaussian_mlp.py:103 casts every observation to
 * f32, so the policy passes see identical values). */
int mjrl_pack_batch_f32(const float* obs, const float* act, int64_t T, const mjrl_shape* s,
                        const float* in_shift, const float* in_scale, float* xhat, float* act32,
                        void* stream);
int mjrl_pack_batch_split_f32(const float* obs, const float* act, int64_t T, const mjrl_shape* s,
                              const float* in_shift, const float* in_scale, const float* xc, void* xs,
                              float* xu, float* act32, void* stream);
/* 1 if the policy passes for this shape accept split-f16 rows (mjrl_rows.xs): every
 * product of the passes then runs as three f16 MFMAs (hi*hi + hi*lo + lo*hi, f32
 * accumulate) on operands split with power-of-two block scales. */
int mjrl_split_supported(const mjrl_shape* s);
/* ---- returns / GAE (process_samples.py:3-44) ----
 * One lane per path, reverse recurrence in fp64, multiply-then-add (no FMA),
 * bit-identical to discount_sum.  use_gae = 0 selects returns - baseline
 * (process_samples.py:10-13).  Also path_ret[p] = sum(rewards of path p) in the
 * order Python's builtin sum uses (npg_cg.py:97). */
int mjrl_gae(const double* rew, const double* base, const int64_t* path_off,
             const uint8_t* terminated, int64_t P, double gamma, double gae_lambda,
             int32_t use_gae, double* ret, double* adv, double* path_ret, void* stream);

/* The same outputs (bit for bit) by the one-wave-per-path kernel of rounds 1-5
 * (mjrl_gae now runs 32 paths per workgroup, lanes = paths); kept for A/B. */
int mjrl_gae_wave(const double* rew, const double* base, const int64_t* path_off,
                  const uint8_t* terminated, int64_t P, double gamma, double gae_lambda,
                  int32_t use_gae, double* ret, double* adv, double* path_ret, void* stream);

/* The same outputs by a wave-parallel scan (one wave per path, 64 lane chunks per
 * window of 1024 steps composed with wave shuffles): not bit-identical to
 * discount_sum — the products are regrouped — but within ~1e-14 of each path's
 * largest |value|; path_ret is a fixed-order wave reduction.  mjrl_gae stays the
 * exact default (UpdateEngine.gae_mode = "serial" | "scan"). */
int mjrl_gae_scan(const double* rew, const double* base, const int64_t* path_off,
                  const uint8_t* terminated, int64_t P, double gamma, double gae_lambda,
                  int32_t use_gae, double* ret, double* adv, double* path_ret, void* stream);

/* ---- LinearBaseline.predict on device (baselines/linear_baseline.py:10-18, 46-49) ----
 * out[t] = [clip(obs_t, +-10), a, a^2, a^3, 1] . coeffs[n+4], a = (t - path start)/1000,
 * for every row of every path (the input of mjrl_gae, process_samples.py:23). */
int mjrl_linear_baseline(const double* obs, int64_t T, int32_t n, const int64_t* path_off,
                         int64_t P, const double* coeffs, double* out, void* stream);

/* The same from f32-staged observations (features computed in fp64 from them). */
int mjrl_linear_baseline_f32(const float* obs, int64_t T, int32_t n, const int64_t* path_off,
                             int64_t P, const double* coeffs, double* out, void* stream);

/* ---- LinearBaseline.fit normal equations on device (baselines/linear_baseline.py:20-44) ----
 * Gram matrix of the augmented rows [f_t, y_t], f_t = [clip(obs_t, +-10), a, a^2, a^3, 1]
 * (a = (t - path start)/1000, as _features), y_t = returns: out[K][K] row-major fp64 with
 * K = n + 5, so out[:k][:k] = F^T F, out[:k][k] = F^T y, out[k][k] = y^T y (k = n + 4).
 * The (F^T F + reg I) c = F^T y lstsq retry loop stays with the caller (k x k, host).
 * scratch: mjrl_linear_baseline_gram_scratch() doubles (split-K slabs + path times);
 * deterministic (fixed slice order, no atomics). */
int mjrl_linear_baseline_gram_scratch(int32_t n, int64_t T, int64_t* doubles);
int mjrl_linear_baseline_gram(const double* obs, const double* returns, int64_t T, int32_t n,
                              const int64_t* path_off, int64_t P, double* scratch, double* out,
                              void* stream);
int mjrl_linear_baseline_gram_f32(const float* obs, const double* returns, int64_t T, int32_t n,
                                  const int64_t* path_off, int64_t P, double* scratch, double* out,
                                  void* stream);
/* out[t] = returns[t] - f_t . coeffs (fit(return_errors=True)'s residuals);
 * scratch as for mjrl_linear_baseline_gram. */
int mjrl_linear_baseline_residual(const double* obs, const double* returns, int64_t T, int32_t n,
                                  const int64_t* path_off, int64_t P, const double* coeffs,
                                  double* scratch, double* out, void* stream);
int mjrl_linear_baseline_residual_f32(const float* obs, const double* returns, int64_t T, int32_t n,
                                      const int64_t* path_off, int64_t P, const double* coeffs,
                                      double* scratch, double* out, void* stream);
/* Both from observations staged as an f32 pair, obs = hi + lo (mjrl_host_stage_paths_f64x
 * rows + mjrl_host_stage_lo_paths_f64 low halves): the features are formed in fp64 from
 * (double)hi + (double)lo, i.e. from the sampler's f64 values to 2^-48, so the fit
 * matches LinearBaseline.fit on observations that are not float32s. */
int mjrl_linear_baseline_gram_f32x2(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                    int32_t n, const int64_t* path_off, int64_t P, double* scratch, double* out,
                                    void* stream);
int mjrl_linear_baseline_residual_f32x2(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                        int32_t n, const int64_t* path_off, int64_t P, const double* coeffs,
                                        double* scratch, double* out, void* stream);

/* QuadraticBaseline.fit (mjrl/baselines/quadratic_baseline.py:10-65) on the device:
 * the same augmented Gram [F y]^T [F y] with the quadratic features o = clip(obs,
 * +-10) / 10, [o, o_i o_j (i <= j, row-major), 1, a, a^2, a^3, a^4] (a = step
 * within the path / 1000): out is K x K, K = n + n(n+1)/2 + 6; n <= 64.  The caller
 * keeps the reference's lstsq retry loop on the (K-1) x (K-1) system.  _residual:
 * r_t = y_t - F_t . coeffs (fit(return_errors=True)).  _f32: f32-staged
 * observations, obs_lo their low halves (mjrl_host_stage_lo_paths_f64) or null.
 * Scratch sizes from mjrl_quadratic_baseline_gram_scratch. */
int mjrl_quadratic_baseline_gram_scratch(int32_t n, int64_t T, int64_t* doubles);
int mjrl_quadratic_baseline_gram(const double* obs, const double* returns, int64_t T, int32_t n,
                                 const int64_t* path_off, int64_t P, double* scratch, double* out, void* stream);
int mjrl_quadratic_baseline_gram_f32(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                     int32_t n, const int64_t* path_off, int64_t P, double* scratch, double* out,
                                     void* stream);
int mjrl_quadratic_baseline_residual(const double* obs, const double* returns, int64_t T, int32_t n,
                                     const int64_t* path_off, int64_t P, const double* coeffs, double* scratch,
                                     double* out, void* stream);
int mjrl_quadratic_baseline_residual_f32(const float* obs, const float* obs_lo, const double* returns, int64_t T,
                                         int32_t n, const int64_t* path_off, int64_t P, const double* coeffs,
                                         double* scratch, double* out, void* stream);

/* ---- subsampled Fisher rows (npg_cg.py:58-62: obs[rand_idx], act[rand_idx]) ----
 * dst row i = src row idx[i] for i < n, rows of row_bytes bytes (a multiple of 4);
 * indices may repeat (np.random.choice draws with replacement).  Used to build
 * the compact xhat / a0 / a1 rows one Fisher-vector product runs on. */
int mjrl_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t n, void* dst,
                     void* stream);

/* ---- moments for whitening / stats (npg_cg.py:91, 97-102; dapg.py:70) ----
 * out[0] = sum(x - c), out[1] = sum((x - c)^2), out[2] = N, out[3] = min(x),
 * out[4] = max(x), out[5] = -min(x) over x[0..N-1] (out needs 6 doubles),
 * c = center[0] / center[2] read from device
 * (the out[] of an uncentred pass, i.e. its mean; center may be null: c = 0).
 * Two launches (per-block partials into rpart[>= 4*256], fixed-order fold);
 * the caller all-reduces out[0..2] between passes when sharded. */
int mjrl_moments(const double* x, int64_t N, const double* center, double* rpart,
                 double* out, void* stream);
int mjrl_moments_f32(const float* x, int64_t N, const double* center, double* rpart,
                     double* out, void* stream);

/* One-launch forms (the last workgroup folds the block partials in fixed order):
 * mjrl_moments2: the moments of x1 [N1] and x2 [N2] together (out1 / out2 as
 * mjrl_moments; out2 may be null to do x1 alone); mjrl_whiten_moments: mjrl_whiten
 * (adv32 required) plus the moments of the f32 whitened values into out[6].
 * rpart: MJRL_MOM_SCRATCH doubles (zero-filled before the first use). */
#define MJRL_MOM_SCRATCH 2056
int mjrl_moments2(const double* x1, int64_t N1, const double* c1, const double* x2, int64_t N2,
                  const double* c2, double* rpart, double* out1, double* out2, void* stream);
int mjrl_whiten_moments(const double* adv, int64_t T, const double* m1, const double* m2, double eps,
                        float* adv32, double* w64, double* rpart, double* out, void* stream);

/* Sharded moments in ONE collective (npg_cg.py:91, 97-102 over the union of the
 * shards): each rank runs pass 1 (center null) and pass 2 centred on its OWN mean
 * into a record of `rec` doubles — group j's pass-1 out[6] at 16 j, its pass-2
 * out[6] at 16 j + 8 — the records are all-gathered (gathered[world][rec], rank
 * order), and this folds them: global pass-1 moments to out[16 j ..], pass-2
 * moments about the GLOBAL mean to out[16 j + 8 ..], M2 = sum_r [M2_r + 2 (m_r -
 * mean) D_r + n_r (m_r - mean)^2].  With world = 1 the outputs equal the
 * unsharded two passes bit for bit.  One workgroup, ngroups <= 64. */
int mjrl_moments_combine(const double* gathered, int32_t world, int32_t rec, int32_t ngroups, double* out,
                         void* stream);

/* w = (adv[t] - mean) / (std + eps), mean = m1[0]/m1[2], std = sqrt(m2[1]/m1[2]);
 * adv32[t] = float(w) (eps = 1e-6: npg_cg.py:91 then the .float() of
 * batch_reinforce.py:38) and/or w64[t] = w (eps = 1e-8: the `normalize` option of
 * process_samples.py:14-19).  Either output may be null, not both. */
int mjrl_whiten(const double* adv, int64_t T, const double* m1, const double* m2,
                double eps, float* adv32, double* w64, void* stream);

/* DAPG augmented advantages (dapg.py:65-70): adv_vpg[t] = float(1e-2 * w[t] /
 * (std(w) + 1e-8)) for t < T (std from the moments mw1/mw2 of w64), and
 * float(1e-2 * demo_coef) for the T_demo demo rows that follow. */
int mjrl_dapg_adv(const double* w64, int64_t T, const double* mw1, const double* mw2,
                  int64_t T_demo, double demo_coef, float* adv_vpg, void* stream);

/* ---- parameter packing (gaussian_mlp.py:66-88 set_param_values) ----
 * flat theta[d] -> packed[s->packed] (padded weights + transposes + log_std).
 * clamp_log_std != 0 applies max(log_std, min_log_std) as set_param_values does. */
int mjrl_pack_params(const mjrl_shape* s, const float* theta, float* packed,
                     int32_t clamp_log_std, float min_log_std, void* stream);

/* ---- policy passes; each writes UNSCALED sums over this shard's rows ----
 * vpg:   gsum[d] = sum_t adv_vpg[t] * dLL_t/dtheta at old == new (LR == 1),
 *        and caches a0/a1/mu0/ll0 (batch_reinforce.py:51-55, gaussian_mlp.py:100-128).
 *        rows->T rows get the forward; only the first T_surr rows feed caches used
 *        later (DAPG: RL rows first, demo rows after, dapg.py:68-69).
 * fvp:   gsum[d] = sum_{t < T_fvp} J_t^T W J_t v (Gauss-Newton form of the
 *        double-backprop HVP, npg_cg.py:55-74); the log_std block is left 0 and
 *        added in closed form by mjrl_cg_step.
 * eval:  sums[0] = sum_t exp(LL_new - LL_old) * adv[t], sums[1] = sum_t KL_t
 *        (CPI_surrogate + kl_old_new at new params, batch_reinforce.py:37-49).
 * `done` (device int, may be null): when *done != 0 the call is a no-op (lets a
 * converged CG loop keep launching without host syncs, cg_solve.py:19-20). */
int mjrl_policy_vpg(const mjrl_shape* s, const mjrl_rows* rows, const float* packed_theta,
                    const float* out_shift, const float* out_scale,
                    const mjrl_scratch* sc, float* gsum, void* stream);
int mjrl_policy_fvp(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_fvp,
                    const float* packed_theta, const float* packed_v,
                    const float* out_scale, const mjrl_scratch* sc, const int32_t* done,
                    float* gsum, void* stream);
int mjrl_policy_eval(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval,
                     const float* packed_theta_new, const float* packed_theta_old,
                     const float* out_shift, const float* out_scale,
                     const mjrl_scratch* sc, double* sums, void* stream);
/* The same, skipped whole (nothing written) while *skip != 0: the speculative
 * evaluations of the device TRPO line search (mjrl_trpo_trial). */
int mjrl_policy_eval_if(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_eval, const float* packed_theta_new,
                        const float* packed_theta_old, const float* out_shift, const float* out_scale,
                        const mjrl_scratch* sc, double* sums, const int32_t* skip, void* stream);

/* The two steps behind the composites above, for callers that time or overlap
 * them separately.  *_accumulate writes per-slice partial sums of every weight /
 * bias gradient ("slabs" in sc->wpart); gather_grads folds the slabs in slice
 * order into gsum[d] (with_log_std = 1 after vpg_accumulate).  For hidden widths
 * 32 / 64 (m <= 32, n <= 383) accumulate is ONE persistent fused kernel (row chain
 * + register-resident weight-gradient sums); otherwise the row-chain kernel plus
 * the split-K weight-gradient kernel.  mjrl_fused_path(s) reports which. */
int mjrl_vpg_accumulate(const mjrl_shape* s, const mjrl_rows* rows, const float* packed_theta,
                        const float* out_shift, const float* out_scale, const mjrl_scratch* sc,
                        void* stream);
/* mjrl_vpg_accumulate / mjrl_policy_vpg with the batch assembly (a5,
 * npg_cg.py:87-89; mjrl_pack_batch_split_f32 with null in_shift / in_scale) fused
 * in: the forward pass reads the staged f32 observations obs[T][n] and writes the
 * split rows rows->xs / rows->xu (outputs here; rows->xc must hold the column
 * scales) bit for bit as the pack does, for the FVP and evaluation passes after
 * it.  The identity input normalisation only (MuNet's default; with in_shift /
 * in_scale, pack first).  Split shapes (mjrl_split_supported) with n % 4 == 0 and
 * 16-byte-aligned obs / xs, else MJRL_ESHAPE; rows->act must hold f32 actions. */
int mjrl_vpg_accumulate_pack(const mjrl_shape* s, const mjrl_rows* rows, const float* obs,
                             const float* packed_theta, const float* out_shift, const float* out_scale,
                             const mjrl_scratch* sc, void* stream);
int mjrl_policy_vpg_pack(const mjrl_shape* s, const mjrl_rows* rows, const float* obs,
                         const float* packed_theta, const float* out_shift, const float* out_scale,
                         const mjrl_scratch* sc, float* gsum, void* stream);
int mjrl_fvp_accumulate(const mjrl_shape* s, const mjrl_rows* rows, int64_t T_fvp,
                        const float* packed_theta, const float* packed_v, const float* out_scale,
                        const int32_t* done, const mjrl_scratch* sc, void* stream);
int mjrl_gather_grads(const mjrl_shape* s, const mjrl_rows* rows, int64_t T,
                      const mjrl_scratch* sc, int32_t with_log_std, const int32_t* done,
                      float* gsum, void* stream);
/* Which accumulate kernel mjrl_{vpg,fvp}_accumulate run for this shape:
 * 2 = K-split persistent (MLP(64,64), act_dim <= 32, np % 32 == 0),
 * 1 = fused persistent (hidden 32/64), 0 = row kernel + split-K weight gradients.
 * The gather and the results do not depend on it. */
int mjrl_fused_path(const mjrl_shape* s);

/* ---- conjugate gradient on device (cg_solve.py:3-22) ----
 * State cg[MJRL_CG_STATE] (f32, device): cg[0] rdotr, cg[1] iterations run,
 * cg[2] v, cg[3] mu, cg[4] p.z; cg[8..1023] scratch of the multi-workgroup step
 * (ticket and per-workgroup partials), cg[1024..] the p.z partials of the fused
 * gather (one double per 64 parameters).
 * init: x = 0, r = b, p = b, rdotr = b.b; packs p into packed_p.
 * step: z = gsum * inv_T + c(sigma) * p_logstd + damping * p, then the
 *       reference's update of x, r, p, rdotr and the residual_tol break
 *       (three multi-workgroup launches; fixed-order fp64 dot products). */
#define MJRL_CG_STATE 4096
int mjrl_cg_init(const mjrl_shape* s, const float* b, float* x, float* r, float* p,
                 float* packed_p, float* cg, int32_t* done, void* stream);
/* mjrl_cg_init with b = float(double(gsum) * scale) formed in the same launch and
 * written to g (the VPG's mean from its all-reduced sums: mjrl_scale_vec + mjrl_cg_init
 * in one launch; npg_cg.py:118-125). */
int mjrl_cg_init_scaled(const mjrl_shape* s, const float* gsum, double scale, float* g, float* x, float* r, float* p,
                        float* packed_p, float* cg, int32_t* done, void* stream);
int mjrl_cg_step(const mjrl_shape* s, const float* gsum, double inv_T, float damping,
                 const float* packed_theta, float* x, float* r, float* p, float* z,
                 float* packed_p, float* cg, int32_t* done, float residual_tol,
                 void* stream);

/* The same iteration with the gradient gather fused in (one process, no
 * all-reduce between the gather and the step): mjrl_gather_cg_z folds the
 * accumulate slabs (as mjrl_gather_grads, with_log_std = 0, also writing gsum)
 * and, in the same launch, forms z = gsum * inv_T + c(sigma) * p_logstd +
 * damping * p and one p.z partial per 64 parameters; mjrl_cg_step_xr_p (one
 * launch) folds those partials and the new r.r in every workgroup (the same
 * fixed order: no grid-wide atomic in the gather, no second launch), sets
 * p.z -> cg[4], v -> cg[2], then updates x, r (into r_out != r: the caller
 * alternates the two buffers), rdotr, mu, done and p / packed_p.  Same arithmetic as mjrl_cg_step (the p.z partials are
 * folded per 64 parameters instead of per 1024).  Needs
 * d <= 64 * (MJRL_CG_STATE - 1024) / 2 (else MJRL_EINVAL: use the unfused pair). */
int mjrl_gather_cg_z(const mjrl_shape* s, const mjrl_rows* rows, int64_t T, const mjrl_scratch* sc,
                     const int32_t* done, float* gsum, double inv_T, float damping,
                     const float* packed_theta, const float* p, float* z, float* cg, void* stream);
int mjrl_cg_step_xr_p(const mjrl_shape* s, float* x, const float* r, float* r_out, float* p,
                      const float* z, float* packed_p, float* cg, int32_t* done, float residual_tol,
                      void* stream);

/* The z step of that iteration from an all-reduced gradient sum (the sharded
 * path: gather, all-reduce of gsum, then this, then mjrl_cg_step_xr_p): z and the
 * per-64-parameter p.z partials exactly as mjrl_gather_cg_z writes them, so one
 * rank reproduces the one-process iteration bit for bit. */
int mjrl_cg_z(const mjrl_shape* s, const float* gsum, double inv_T, float damping, const float* packed_theta,
              const float* p, float* z, float* cg, const int32_t* done, void* stream);

/* The whole iteration of mjrl_cg_step in one launch (the sharded path: gsum is
 * the all-reduced sum): every workgroup forms z for all of d on the fly and folds
 * p.z and the new r.r itself, then updates x, r and p of its own chunk; r and p
 * go to r_out / p_out (!= r / p: the caller alternates each pair).  Same
 * arithmetic as mjrl_cg_step up to the order of the fp64 dot-product sums. */
int mjrl_cg_step1(const mjrl_shape* s, const float* gsum, double inv_T, float damping,
                  const float* packed_theta, float* x, const float* r, float* r_out, const float* p,
                  float* p_out, float* packed_p, float* cg, int32_t* done, float residual_tol,
                  void* stream);

/* Generic CG (cg_solve.py:3-22 with a caller-supplied operator): init from b,
 * then one update per z = A p the caller computed.  Same scalar arithmetic and
 * residual_tol break as mjrl_cg_step. */
int mjrl_cg_init_vec(int32_t d, const float* b, float* x, float* r, float* p, float* cg,
                     int32_t* done, void* stream);
int mjrl_cg_update(int32_t d, const float* z, float* x, float* r, float* p, float* cg,
                   int32_t* done, float residual_tol, void* stream);

/* g[d] = gsum * scale  (VPG normalisation: 1/T, DAPG: 1/T_rl, dapg.py:97-98) */
int mjrl_scale_vec(const float* gsum, int32_t d, double scale, float* g, void* stream);

/* ---- step (npg_cg.py:128-141, trpo.py:100-108, dapg.py:111-118) ----
 * mode 0: alpha = sqrt(|delta / (g.x + 1e-20)|);  mode 1: alpha = alpha_in
 * (const learn-rate or a TRPO backtrack trial); out[0] = alpha, out[1] = g.x,
 * out[2] = delta (mode 1 with const_lr: alpha^2 * g.x).
 * theta_new = clamp_logstd(theta + alpha * x); packs theta_new.
 * out holds MJRL_STEP_OUT floats (out[8..] is the multi-workgroup g.x scratch). */
#define MJRL_STEP_OUT 1024
int mjrl_npg_step(const mjrl_shape* s, const float* g, const float* x, const float* theta,
                  int32_t mode, float delta, float alpha_in, int32_t const_lr,
                  float min_log_std, float* theta_new, float* packed_new, float* out,
                  void* stream);

/* ---- TRPO line search on the device (trpo.py:105-118) ----
 * Trial k >= 1: logs trial k - 1's evaluation (sums = [surr sum, kl sum] of
 * mjrl_policy_eval; kl = float(sums[1] * inv_T)), and if kl >= kl_dist steps to
 * alpha_k = float32(0.9) * alpha_{k-1} (f32), writing theta + alpha_k x (log-std
 * clamp, packed copy) for the next mjrl_policy_eval_if; an accepted trial sets *skip,
 * after which the remaining trials and evaluations of the sequence do nothing
 * (out[0] = the accepted alpha, as a host step leaves it).
 * apply = 0: log and test only.  alpha_0 is out[0] of the mode-0 mjrl_npg_step.
 * ls: MJRL_LS_STATE floats, [1] accepted, [2] trials logged, [MJRL_LS_LOG + 3 t ..]
 * trial t's (alpha, kl, surr); one readback after the sequence replaces a host round
 * trip per trial (the host continues past the sequence's last trial as before). */
#define MJRL_LS_LOG 32
#define MJRL_LS_STATE 128
int mjrl_trpo_trial(const mjrl_shape* s, const float* x, const float* theta, float min_log_std, float* theta_new,
                    float* packed_new, float* out, const double* sums, double inv_T, double kl_dist, int32_t k,
                    int32_t apply, float* ls, int32_t* skip, void* stream);

/* ---- batched policy forward for vectorised sampling ----
 * Replaces the per-observation MuNet forward inside policy.get_action
 * (mjrl/policies/gaussian_mlp.py:92-98, gaussian_linear.py:90-96) for the N
 * lock-stepped environments of one sampling step (mjrl/samplers/base_sampler.py:64-74):
 * mean[N][m] (f32) = out_scale * MuNet((obs - in_shift) / (in_scale + 1e-8)) + out_shift
 * from obs f32 [N][n] and the packed parameters of mjrl_pack_params.  The Gaussian
 * noise stays on the host (each trajectory's own numpy stream). */
int mjrl_policy_mean(const mjrl_shape* s, const float* obs, int64_t N, const float* packed_theta,
                     const float* in_shift, const float* in_scale, const float* out_shift,
                     const float* out_scale, float* mean, void* stream);

/* ---- host staging of sampler paths (base_sampler.py:76-83,
 * npg_cg.py:87-89 concatenate) — HOST memory, runs on the calling CPU thread ----
 * dst[rows][n] = float(src) (round to nearest, as torch .float()), and when cmin /
 * cmax (n floats each) are given, cmin[k] = min(cmin[k], column k), cmax likewise
 * (NaN skipped, as the device column max skips it) in the same pass, so the
 * column scales of the split rows (mjrl_obs_colscale_range) cost no pass over the
 * batch.  Callers initialise cmin = +inf, cmax = -inf.  Thread-safe for disjoint
 * dst / cmin / cmax. */
int mjrl_host_stage_f64(const double* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax);
int mjrl_host_stage_f32(const float* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax);
/* mjrl_host_stage_f64 over `count` arrays srcs[i] (rows[i] x n, row-major, f64)
 * written one after another into dst: one call per chunk of paths. */
int mjrl_host_stage_paths_f64(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n, float* dst,
                              float* cmin, float* cmax);
/* The same pass with LinearBaseline.predict's input taken from the sampler's own f64
 * values (baselines/linear_baseline.py:10-18, 46-49; process_samples.py:23): for the
 * first npred arrays (the RL paths; demonstration paths follow them) pred receives,
 * one path after another, [clip(x, +-10), a, a^2, a^3, 1] . coeffs[n+4] in fp64
 * (a = row index in the path / 1000) when coeffs / pred are given (both or neither),
 * and *inexact (nullable) is set to 1 when any value is not exactly a float32 (the
 * caller then stages the low halves below for the device fit).  The block's source
 * is re-read from the core's cache, not DRAM. */
int mjrl_host_stage_paths_f64x(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n, float* dst,
                               float* cmin, float* cmax, const double* coeffs, double* pred, int32_t npred,
                               int32_t* inexact);
/* dst = float(x - double(float(x))) for `count` arrays one after another: with the
 * f32 rows above, hi + lo carries every observation to 2^-48 relative (lo = 0 where
 * float(x) overflows).  The input of mjrl_linear_baseline_gram_f32x2. */
int mjrl_host_stage_lo_paths_f64(const double* const* srcs, const int64_t* rows, int32_t count, int32_t n,
                                 float* dst);
/* Rows bound for different places (the vectorised sampler's streaming sink: one row
 * per environment per step, each into its trajectory's pinned slab): row i of src
 * (rows x n f64, contiguous) converted into dst_rows[i] (n f32), folded into cmin /
 * cmax (nullable, both or neither), with pred[i] = its LinearBaseline prediction at
 * path index tidx[i] when coeffs is given (coeffs / pred / tidx together), and
 * *inexact (nullable) raised as above: the same per-row arithmetic as
 * mjrl_host_stage_paths_f64x, so a batch built row by row is bit-identical. */
int mjrl_host_stage_rows_f64x(const double* src, int64_t rows, int32_t n, float* const* dst_rows, float* cmin,
                              float* cmax, const double* coeffs, const int64_t* tidx, double* pred,
                              int32_t* inexact);
/* The extras of mjrl_host_stage_paths_f64x for one array through the portable loop
 * (tests compare it with the vector path). */
int mjrl_host_extras_portable(const double* src, int64_t rows, int32_t n, const double* coeffs, double* pred,
                              int32_t* inexact);
/* The portable (non-AVX-512) path of mjrl_host_stage_f64, whatever the CPU, and
 * whether the CPU runs the AVX-512 path (1) or not (0); both for tests.  All the
 * mjrl_host_stage_* entry points are also in the host-only lib/libmjrl_stage.so. */
int mjrl_host_stage_f64_portable(const double* src, int64_t rows, int32_t n, float* dst, float* cmin, float* cmax);
int mjrl_host_stage_avx512(void);
/* Same-type concatenation: `count` byte runs srcs[i] (nbytes[i] bytes) copied one
 * after another into dst (the 1-D slots of a chunk of paths: rewards, advantages,
 * host baseline predictions; npg_cg.py:87-89 concatenate).  One call per chunk,
 * no Python per path. */
int mjrl_host_gather(const void* const* srcs, const int64_t* nbytes, int32_t count, void* dst);

#ifdef __cplusplus
}
#endif
#endif /* MJRL_AMD_H */
