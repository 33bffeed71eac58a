"""Times mjrl_obs_colscale_f32 (column maxima + power-of-two column scales of the
split rows) alone at the Humanoid width, for several grid caps
(MJRL_AMD_COLMAX_G is read once per process, so each cap runs in a child).
Usage: python tools/colmax_probe.py [caps...]"""
import os
import subprocess
import sys


def child(T_list):
    import ctypes as C
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mjrl_amd import _lib
    L = _lib.lib()
    s = _lib.Shape()
    _lib.check(L.mjrl_shape_init(C.byref(s), 376, 17, 64, 64), "shape")
    dev = torch.device("cuda:0")
    st = _lib.stream_ptr()
    out = []
    for T in T_list:
        obs = torch.randn(T, 376, device=dev) * torch.logspace(-4, 3, 376, device=dev)
        sh = torch.zeros(376, device=dev)
        sc = torch.ones(376, device=dev)
        xc = torch.zeros(s.np, device=dev)
        for _ in range(3):
            _lib.check(L.mjrl_obs_colscale_f32(_lib.ptr(obs), T, C.byref(s), _lib.ptr(sh), _lib.ptr(sc),
                                                _lib.ptr(xc), st), "colscale")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            L.mjrl_obs_colscale_f32(_lib.ptr(obs), T, C.byref(s), _lib.ptr(sh), _lib.ptr(sc), _lib.ptr(xc), st)
        e1.record()
        torch.cuda.synchronize()
        ref = obs.abs().amax(0)
        got = xc[:376]
        ok = bool(((got >= ref) & (got <= 2 * ref + (ref == 0))).all())   # power of two above the max
        out.append("T=%d %.1f us ok=%s" % (T, e0.elapsed_time(e1) / n * 1e3, ok))
        del obs
    print(os.environ.get("MJRL_AMD_COLMAX_G", "default"), " | ".join(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child([125000, 1000000])
        sys.exit(0)
    caps = sys.argv[1:] or ["256", "512", "1024", "2048"]
    for c in caps:
        env = dict(os.environ, MJRL_AMD_COLMAX_G=c)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
