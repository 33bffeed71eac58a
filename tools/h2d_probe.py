"""H2D throughput from pinned host memory on the GPU box: 1.5 GB in chunks of
`chunk` MB issued round-robin on 1 / 2 / 4 copy streams, and as one copy.
    python tools/h2d_probe.py"""
import time

import torch


def run(nbytes=1_504_000_000):
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h.fill_(1)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(4)]
    for chunk_mb in (16, 64):
        cb = chunk_mb << 20
        for ns in (1, 2, 4):
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k, b0 in enumerate(range(0, nbytes, cb)):
                    s = streams[k % ns]
                    with torch.cuda.stream(s):
                        d[b0:b0 + cb].copy_(h[b0:b0 + cb], non_blocking=True)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            print("chunk %3d MB streams %d: %.2f ms = %.1f GB/s" % (chunk_mb, ns, best * 1e3, nbytes / best / 1e9),
                  flush=True)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print("one copy: %.2f ms = %.1f GB/s" % (best * 1e3, nbytes / best / 1e9), flush=True)


if __name__ == "__main__":
    run()
