"""Builds the gfx950 shared library mjrl_amd/lib/libmjrl_amd.so (the C-ABI of
include/mjrl_amd.h) with hipcc.  One object per .hip source, compiled in
parallel, then linked.  Rebuilds only when a source or header is newer.

    python -m mjrl_amd.build [--force] [-j N]
"""
import argparse
import concurrent.futures as cf
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUTDIR = os.path.join(HERE, "lib")
LIB = os.path.join(OUTDIR, "libmjrl_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = [
    "-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH,
    "-ffp-contract=off",          # keep the reference's multiply-then-add order
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]
SOURCES = ["batch.hip", "policy.hip", "cg.hip", "baseline.hip", "rollout.hip"]
# host-only C++ (the staging conversion of csrc/stage.cpp), built with g++
HOST_SOURCES = ["stage.cpp"]
# no -m flag: the AVX-512 path is selected at run time (csrc/stage.cpp)
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall"]
STAGE_LIB = os.path.join(OUTDIR, "libmjrl_stage.so")


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(ROOT, "include", "mjrl_amd.h"))
    return max(os.path.getmtime(h) for h in hdrs)


def _compile(src, force, prof=False, tag="", extra=()):
    s = os.path.join(CSRC, src)
    host = src.endswith(".cpp")
    o = os.path.join(OUTDIR, src.replace(".hip", "").replace(".cpp", "") + ("_prof" if prof else "") + tag + ".o")
    if not force and os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), _deps()):
        return o
    if host:
        cmd = [os.environ.get("CXX", "g++")] + HOST_FLAGS + ["-c", s, "-o", o]
    else:
        cmd = [HIPCC] + FLAGS + list(extra) + (["-DMJRL_KX_PROF"] if prof else []) + ["-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr[-8000:]))
    return o


def build(force=False, jobs=None, prof=False, tag="", extra=()):
    """prof=True builds the phase-profiling variant lib/libmjrl_amd_prof.so
    (-DMJRL_KX_PROF; select it with MJRL_AMD_LIB=<path>).  tag / extra: an
    experimental variant lib/libmjrl_amd<tag>.so built with extra hipcc flags."""
    os.makedirs(OUTDIR, exist_ok=True)
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 1, 16)
    lib = LIB.replace(".so", ("_prof" if prof else "") + tag + ".so")
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, prof, tag, extra), SOURCES + HOST_SOURCES))
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "--offload-arch=" + ARCH, "-fPIC"] + objs + ["-o", lib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr[-8000:]))
    # the host-only staging library (no HIP): the same stage object, linked by g++
    stage_o = [o for o in objs if os.path.basename(o).startswith("stage")]
    slib = STAGE_LIB.replace(".so", tag + ".so") if tag else STAGE_LIB
    if not prof and (force or not os.path.exists(slib) or os.path.getmtime(slib) < os.path.getmtime(stage_o[0])):
        cmd = [os.environ.get("CXX", "g++"), "-shared", "-fPIC"] + stage_o + ["-o", slib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr[-8000:]))
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--prof", action="store_true", help="phase-profiling variant (libmjrl_amd_prof.so)")
    ap.add_argument("--tag", default="", help="variant suffix: lib/libmjrl_amd<tag>.so")
    ap.add_argument("--extra", default="", help="extra hipcc flags of the variant (space separated)")
    ap.add_argument("--debug", action="store_true",
                    help="device-checked variant lib/libmjrl_amd_dbg.so (-DMJRL_DEVICE_CHECKS: slab indices "
                         "against the scratch; select it with MJRL_AMD_LIB=<path>)")
    args = ap.parse_args()
    if args.debug:
        args.tag, args.extra = args.tag or "_dbg", args.extra + " -DMJRL_DEVICE_CHECKS"
    print(build(args.force, args.j, args.prof, args.tag, args.extra.split()))
