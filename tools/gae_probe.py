"""Times mjrl_gae (exact serial chains) and mjrl_gae_scan on the bench's path
shapes with HIP events, and checks the exact kernel against the oracle's
discount_sum chains bit for bit on the first paths.  GPU box:
    python tools/gae_probe.py
GAE_PROBE_ONLY=1: mjrl_gae alone; GAE_PROBE_NOCHECK=1 (with MJRL_AMD_ALLOW_ABLATION=1):
time a timing-ablation build of the kernel (-DMJRL_GAE_ABL_*), results unchecked."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mjrl_amd import _lib  # noqa: E402


def run(P, H, reps=20):
    L = _lib.lib()
    dev = torch.device("cuda:0")
    rs = np.random.RandomState(P)
    rew = torch.from_numpy(rs.randn(P * H)).to(dev)
    base = torch.from_numpy(rs.randn(P * H)).to(dev)
    off = torch.from_numpy(np.arange(P + 1, dtype=np.int64) * H).to(dev)
    term = torch.zeros(P, dtype=torch.uint8, device=dev)
    ret = torch.empty(P * H, dtype=torch.float64, device=dev)
    adv = torch.empty_like(ret)
    pr = torch.empty(P, dtype=torch.float64, device=dev)
    st = _lib.stream_ptr()
    out = {}
    only = os.environ.get("GAE_PROBE_ONLY") == "1"
    nocheck = os.environ.get("GAE_PROBE_NOCHECK") == "1"
    for name in ("mjrl_gae",) if only else ("mjrl_gae", "mjrl_gae_wave", "mjrl_gae_scan"):
        fn = getattr(L, name)
        args = (_lib.ptr(rew), _lib.ptr(base), _lib.ptr(off), _lib.ptr(term), P, 0.995, 0.97, 1, _lib.ptr(ret),
                _lib.ptr(adv), _lib.ptr(pr), st)
        _lib.check(fn(*args), name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _lib.check(fn(*args), name)
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / reps * 1e3
        if name in ("mjrl_gae", "mjrl_gae_wave") and not nocheck:
            from oracle import npg_cpu as O
            r, b = rew.cpu().numpy(), base.cpu().numpy()
            lengths = np.full(P, H)
            rr, aa = O.returns_and_advantages(r[:3 * H], b[:3 * H], lengths[:3], np.zeros(3, bool), 0.995, 0.97)
            assert np.array_equal(ret[:3 * H].cpu().numpy(), rr) and np.array_equal(adv[:3 * H].cpu().numpy(), aa)
    return out


if __name__ == "__main__":
    for P, H in ((125, 1000), (1000, 1000), (25, 500), (100, 1000), (200, 200), (1, 1000), (125, 250), (125, 500),
                 (125, 1024), (125, 2000), (125, 4000), (1, 4000)):
        o = run(P, H)
        print("P %5d H %5d  gae (lanes = paths) %7.2f us  gae_wave (round 5) %7.2f us  gae_scan %7.2f us"
              % (P, H, o["mjrl_gae"], o.get("mjrl_gae_wave", float("nan")), o.get("mjrl_gae_scan", float("nan"))),
              flush=True)
