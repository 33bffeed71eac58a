"""ctypes binding of the gfx950 C ABI (include/mjrl_amd.h).

The library is mjrl_amd/lib/libmjrl_amd.so, built in-tree by
`python -m mjrl_amd.build` (or __graft_entry__.build()).  There is no CPU
fallback: if the library or a GPU is missing, `lib()` raises.

torch is imported first on purpose: torch-ROCm ships the HIP runtime
(libamdhip64.so.7) and our library resolves against that already-loaded copy, so
torch's hipStream_t handles are valid arguments.
"""
import ctypes as C
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmjrl_amd.so")

MJRL_OK = 0
MJRL_EINVAL = -1
MJRL_ESHAPE = -2
CG_STATE = 4096   # MJRL_CG_STATE: floats of the device CG state
CG_PZ_PARTS = 1024   # float offset of the fused gather's p.z partials (csrc/common.h)
STEP_OUT = 1024   # MJRL_STEP_OUT: floats of mjrl_npg_step's out buffer
LS_LOG, LS_STATE = 32, 128   # MJRL_LS_LOG / MJRL_LS_STATE (device TRPO line search state)
MOM_SCRATCH = 2056   # MJRL_MOM_SCRATCH: doubles of the one-launch moments scratch


class Shape(C.Structure):
    _fields_ = [("n", C.c_int32), ("m", C.c_int32), ("h0", C.c_int32), ("h1", C.c_int32),
                ("np", C.c_int32), ("mp", C.c_int32), ("d", C.c_int32), ("packed", C.c_int32)]


class Rows(C.Structure):
    _fields_ = [("T", C.c_int64)] + [(k, C.c_void_p) for k in (
        "xhat", "act", "adv", "adv_vpg", "a0", "a1", "mu0", "ll0", "gu0", "gu1", "gp", "xs", "xu", "xc")]


class Scratch(C.Structure):
    _fields_ = [("wpart", C.c_void_p), ("rpart", C.c_void_p), ("slices", C.c_int32)]


P = C.c_void_p
I32 = C.c_int32
I64 = C.c_int64
F32 = C.c_float
F64 = C.c_double
SP = C.POINTER(Shape)

# name -> argtypes, in header order; every function returns int
SIGNATURES = {
    "mjrl_shape_init": [SP, I32, I32, I32, I32],
    "mjrl_scratch_size": [SP, I64, C.POINTER(I64), C.POINTER(I64), C.POINTER(I32)],
    "mjrl_pack_batch": [P, P, I64, SP, P, P, P, P, P],
    "mjrl_obs_colscale": [P, I64, SP, P, P, P, P],
    "mjrl_obs_colscale_f32": [P, I64, SP, P, P, P, P],
    "mjrl_obs_colscale_range": [P, P, SP, P, P, P, P],
    "mjrl_pack_batch_split": [P, P, I64, SP, P, P, P, P, P, P, P],
    "mjrl_pack_batch_f32": [P, P, I64, SP, P, P, P, P, P],
    "mjrl_pack_batch_split_f32": [P, P, I64, SP, P, P, P, P, P, P, P],
    "mjrl_split_supported": [SP],
    "mjrl_gae": [P, P, P, P, I64, F64, F64, I32, P, P, P, P],
    "mjrl_gae_wave": [P, P, P, P, I64, F64, F64, I32, P, P, P, P],
    "mjrl_gae_scan": [P, P, P, P, I64, F64, F64, I32, P, P, P, P],
    "mjrl_linear_baseline": [P, I64, I32, P, I64, P, P, P],
    "mjrl_linear_baseline_f32": [P, I64, I32, P, I64, P, P, P],
    "mjrl_moments": [P, I64, P, P, P, P],
    "mjrl_moments_f32": [P, I64, P, P, P, P],
    "mjrl_moments2": [P, I64, P, P, I64, P, P, P, P, P],
    "mjrl_whiten_moments": [P, I64, P, P, F64, P, P, P, P, P],
    "mjrl_moments_combine": [P, I32, I32, I32, P, P],
    "mjrl_whiten": [P, I64, P, P, F64, P, P, P],
    "mjrl_dapg_adv": [P, I64, P, P, I64, F64, P, P],
    "mjrl_pack_params": [SP, P, P, I32, F32, P],
    "mjrl_policy_vpg": [SP, C.POINTER(Rows), P, P, P, C.POINTER(Scratch), P, P],
    "mjrl_policy_fvp": [SP, C.POINTER(Rows), I64, P, P, P, C.POINTER(Scratch), P, P, P],
    "mjrl_policy_eval": [SP, C.POINTER(Rows), I64, P, P, P, P, C.POINTER(Scratch), P, P],
    "mjrl_policy_eval_if": [SP, C.POINTER(Rows), I64, P, P, P, P, C.POINTER(Scratch), P, P, P],
    "mjrl_vpg_accumulate": [SP, C.POINTER(Rows), P, P, P, C.POINTER(Scratch), P],
    "mjrl_vpg_accumulate_pack": [SP, C.POINTER(Rows), P, P, P, P, C.POINTER(Scratch), P],
    "mjrl_policy_vpg_pack": [SP, C.POINTER(Rows), P, P, P, P, C.POINTER(Scratch), P, P],
    "mjrl_fvp_accumulate": [SP, C.POINTER(Rows), I64, P, P, P, P, C.POINTER(Scratch), P],
    "mjrl_gather_grads": [SP, C.POINTER(Rows), I64, C.POINTER(Scratch), I32, P, P, P],
    "mjrl_fused_path": [SP],
    "mjrl_cg_init": [SP, P, P, P, P, P, P, P, P],
    "mjrl_cg_init_scaled": [SP, P, F64, P, P, P, P, P, P, P, P],
    "mjrl_cg_step": [SP, P, F64, F32, P, P, P, P, P, P, P, P, F32, P],
    "mjrl_gather_cg_z": [SP, C.POINTER(Rows), I64, C.POINTER(Scratch), P, P, F64, F32, P, P, P, P, P],
    "mjrl_cg_step_xr_p": [SP, P, P, P, P, P, P, P, P, F32, P],
    "mjrl_cg_z": [SP, P, F64, F32, P, P, P, P, P, P],
    "mjrl_cg_step1": [SP, P, F64, F32, P, P, P, P, P, P, P, P, P, F32, P],
    "mjrl_cg_init_vec": [I32, P, P, P, P, P, P, P],
    "mjrl_cg_update": [I32, P, P, P, P, P, P, F32, P],
    "mjrl_scale_vec": [P, I32, F64, P, P],
    "mjrl_gather_rows": [P, I64, P, I64, P, P],
    "mjrl_linear_baseline_gram_scratch": [I32, I64, C.POINTER(I64)],
    "mjrl_linear_baseline_gram": [P, P, I64, I32, P, I64, P, P, P],
    "mjrl_linear_baseline_residual": [P, P, I64, I32, P, I64, P, P, P, P],
    "mjrl_linear_baseline_gram_f32": [P, P, I64, I32, P, I64, P, P, P],
    "mjrl_linear_baseline_residual_f32": [P, P, I64, I32, P, I64, P, P, P, P],
    "mjrl_linear_baseline_gram_f32x2": [P, P, P, I64, I32, P, I64, P, P, P],
    "mjrl_linear_baseline_residual_f32x2": [P, P, P, I64, I32, P, I64, P, P, P, P],
    "mjrl_quadratic_baseline_gram_scratch": [I32, I64, C.POINTER(I64)],
    "mjrl_quadratic_baseline_gram": [P, P, I64, I32, P, I64, P, P, P],
    "mjrl_quadratic_baseline_gram_f32": [P, P, P, I64, I32, P, I64, P, P, P],
    "mjrl_quadratic_baseline_residual": [P, P, I64, I32, P, I64, P, P, P, P],
    "mjrl_quadratic_baseline_residual_f32": [P, P, P, I64, I32, P, I64, P, P, P, P],
    "mjrl_npg_step": [SP, P, P, P, I32, F32, F32, I32, F32, P, P, P, P],
    "mjrl_trpo_trial": [SP, P, P, F32, P, P, P, P, F64, F64, I32, I32, P, P, P],
    "mjrl_policy_mean": [SP, P, I64, P, P, P, P, P, P, P],
    "mjrl_build_flags": [],
    "mjrl_host_stage_f64": [P, I64, I32, P, P, P],
    "mjrl_host_stage_f32": [P, I64, I32, P, P, P],
    "mjrl_host_stage_paths_f64": [P, P, I32, I32, P, P, P],
    "mjrl_host_stage_paths_f64x": [P, P, I32, I32, P, P, P, P, P, I32, P],
    "mjrl_host_stage_lo_paths_f64": [P, P, I32, I32, P],
    "mjrl_host_extras_portable": [P, I64, I32, P, P, P],
    "mjrl_host_stage_rows_f64x": [P, I64, I32, P, P, P, P, P, P, P],
    "mjrl_host_stage_f64_portable": [P, I64, I32, P, P, P],
    "mjrl_host_stage_avx512": [],
    "mjrl_host_gather": [P, P, I32, P],
}

BUILD_ABLATION, BUILD_PROF, BUILD_CHECKS = 1, 2, 4   # mjrl_build_flags()
_LIB = None


class MjrlError(RuntimeError):
    pass


def load(path=None):
    """Loads the shared library and declares every entry point (no GPU needed).
    $MJRL_AMD_LIB selects another build of it (e.g. the profiling variant)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("MJRL_AMD_LIB") or LIB_PATH
    if not os.path.isabs(path) and not os.path.exists(path):
        # a relative MJRL_AMD_LIB names a file under the repository root (pool
        # workers and train_agent run from other working directories)
        path = os.path.join(os.path.dirname(HERE), path)
    if not os.path.exists(path):
        raise MjrlError("mjrl_amd HIP library not built: %s (run `python -m mjrl_amd.build`)" % path)
    lib = C.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    if lib.mjrl_build_flags() & BUILD_ABLATION and os.environ.get("MJRL_AMD_ALLOW_ABLATION") != "1":
        raise MjrlError("%s is a timing-ablation build (MJRL_KX_ABL_*: its results are wrong by construction); "
                        "set MJRL_AMD_ALLOW_ABLATION=1 to load it for timing" % path)
    _LIB = lib
    return lib


STAGE_LIB_PATH = os.path.join(HERE, "lib", "libmjrl_stage.so")
STAGE_FUNCS = ("mjrl_host_stage_f64", "mjrl_host_stage_f32", "mjrl_host_stage_paths_f64",
               "mjrl_host_stage_paths_f64x", "mjrl_host_stage_lo_paths_f64", "mjrl_host_extras_portable",
               "mjrl_host_stage_rows_f64x",
               "mjrl_host_stage_f64_portable", "mjrl_host_stage_avx512", "mjrl_host_gather")
_STAGE = None


def stage_lib():
    """The host-only staging library (csrc/stage.cpp, lib/libmjrl_stage.so): the
    f64 -> f32 convert-and-range pass of the staging threads and of the pool
    controller, without loading the HIP library or its code objects."""
    global _STAGE
    if _STAGE is None:
        if not os.path.exists(STAGE_LIB_PATH):
            raise MjrlError("mjrl_amd staging library not built: %s (run `python -m mjrl_amd.build`)"
                            % STAGE_LIB_PATH)
        lib = C.CDLL(STAGE_LIB_PATH)
        for name in STAGE_FUNCS:
            fn = getattr(lib, name)
            fn.argtypes = SIGNATURES[name]
            fn.restype = C.c_int
        _STAGE = lib
    return _STAGE


def lib():
    """The library, for compute calls: requires a visible GPU."""
    if not torch.cuda.is_available():
        raise MjrlError("mjrl_amd needs an AMD GPU (torch.cuda.is_available() is False); "
                        "there is no CPU fallback")
    return load()


def check(rc, what):
    if rc != MJRL_OK:
        msg = {MJRL_EINVAL: "invalid argument", MJRL_ESHAPE: "unsupported policy shape"}.get(
            rc, "HIP error %d" % rc)
        raise MjrlError("%s failed: %s" % (what, msg))


def make_shape(n, m, h0, h1, loader=load):
    s = Shape()
    rc = loader().mjrl_shape_init(C.byref(s), n, m, h0, h1)
    check(rc, "mjrl_shape_init(n=%d, m=%d, hidden=(%d, %d))" % (n, m, h0, h1))
    return s


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
