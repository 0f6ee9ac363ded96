"""Probe the GPU box: CPU share, affinity, cgroup quota, PCIe H2D/D2H bandwidth."""
import os, time, json
out = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    try:
        out[p] = open(p).read().strip()
    except Exception as e:
        out[p] = str(e)
try:
    out["loadavg"] = open("/proc/loadavg").read().strip()
    out["meminfo"] = open("/proc/meminfo").read().split("\n")[0]
except Exception:
    pass
import torch
dev = torch.device("cuda:0")
for mb in (4, 16, 64):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter(); k = 20
    for _ in range(k):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_GBs_%dMB" % mb] = round(k * n / (time.perf_counter() - t) / 1e9, 2)
    t = time.perf_counter()
    for _ in range(k):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    out["d2h_GBs_%dMB" % mb] = round(k * n / (time.perf_counter() - t) / 1e9, 2)
# host memcpy bandwidth, 1 thread (numpy)
import numpy as np
a = np.ones(64 << 20, np.uint8); b = np.empty_like(a)
t = time.perf_counter()
for _ in range(10): np.copyto(b, a)
out["host_memcpy_GBs_1thr"] = round(10 * a.nbytes / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(out))
