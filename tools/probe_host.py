"""GPU-box host probe: CPU share (affinity / cgroup quota), OpenSSL presence, and the H2D
rates the host-buffer entry points can reach (pageable vs pinned, one copy vs chunked).
Writes one JSON object to stdout. Not product code."""
import ctypes.util
import json
import os
import threading
import time

import numpy as np
import torch


def cpu_info():
    d = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/memory.max"):
        try:
            with open(p) as f:
                d[os.path.basename(p)] = f.read().strip()
        except OSError:
            d[os.path.basename(p)] = None
    try:
        with open("/proc/cpuinfo") as f:
            d["model"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        d["model"] = None
    d["libcrypto"] = ctypes.util.find_library("crypto")
    d["OMP_NUM_THREADS"] = os.environ.get("OMP_NUM_THREADS")
    return d


def h2d(nbytes=1 << 30, reps=3):
    dev = torch.device("cuda", 0)
    out = {}
    src = torch.from_numpy(np.ones(nbytes, dtype=np.uint8))
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def rate(fn):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return round(nbytes * reps / (time.perf_counter() - t) / 1e9, 2)

    out["pageable_GBps"] = rate(lambda: dst.copy_(src, non_blocking=True))
    pin = src.pin_memory()
    out["pinned_GBps"] = rate(lambda: dst.copy_(pin, non_blocking=True))
    # host memcpy pageable -> pinned with k threads (the staging leg)
    a, b = src.numpy(), pin.numpy()
    for k in (1, 4, 8, 16):
        def cp():
            n = len(a)
            ths = [threading.Thread(target=np.copyto, args=(b[n * j // k:n * (j + 1) // k], a[n * j // k:n * (j + 1) // k]))
                   for j in range(k)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        cp()
        t = time.perf_counter()
        for _ in range(reps):
            cp()
        out[f"memcpy_{k}t_GBps"] = round(nbytes * reps / (time.perf_counter() - t) / 1e9, 2)
    return out


if __name__ == "__main__":
    r = {"cpu": cpu_info()}
    r["h2d"] = h2d()
    print(json.dumps(r))
