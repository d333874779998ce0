"""Host -> HBM copy rates on the box (not part of the library): what the C4 leg's link
roofline should be.  Sources: hipHostMalloc'd memory (torch pinned), pageable numpy,
numpy registered with hipHostRegister, a /dev/shm file mapping registered read-only;
one copy at a time vs several streams in flight.

run: python scripts/h2d_probe.py"""
import ctypes
import mmap
import os
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
GiB = 1 << 30
dev = torch.empty(4 * GiB, dtype=torch.uint8, device="cuda")


def rate(host_u8, streams=1, reps=4):
    n = host_u8.numel()
    per = n // streams
    ss = [torch.cuda.Stream() for _ in range(streams)]
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, s in enumerate(ss):
            with torch.cuda.stream(s):
                dev[i * per:(i + 1) * per].copy_(host_u8[i * per:(i + 1) * per], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return n / best / 1e9


def show(name, host):
    for st in (1, 2, 4):
        print(f"{name:34s} {host.numel() / GiB:.0f} GiB streams {st}: {rate(host, st):7.2f} GB/s", flush=True)


pinned = torch.empty(4 * GiB, dtype=torch.uint8, pin_memory=True)
pinned.fill_(1)
show("hipHostMalloc (torch pinned)", pinned[:GiB])
show("hipHostMalloc (torch pinned)", pinned)
del pinned

arr = np.ones(4 * GiB + 8192, np.uint8)
off = (-arr.ctypes.data) % 4096
a = arr[off:off + 4 * GiB]
show("pageable numpy", torch.from_numpy(a))
assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 0) == 0
show("numpy + hipHostRegister", torch.from_numpy(a))
hip.hipHostUnregister(a.ctypes.data)
del a, arr

path = f"/dev/shm/h2d_probe_{os.getpid()}"
with open(path, "wb") as f:
    f.truncate(4 * GiB)
try:
    with open(path, "r+b") as f:
        mm = mmap.mmap(f.fileno(), 4 * GiB)
        m = np.frombuffer(mm, np.uint8)
        m[:] = 1
        del m
        mm.close()
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 4 * GiB, prot=mmap.PROT_READ)
        m = np.frombuffer(mm, np.uint8)
        show("shm mmap (pageable)", torch.frombuffer(mm, dtype=torch.uint8))
        print("register", hip.hipHostRegister(m.ctypes.data, m.nbytes, 8))  # 8 = hipHostRegisterReadOnly
        show("shm mmap + hipHostRegister(RO)", torch.frombuffer(mm, dtype=torch.uint8))
        hip.hipHostUnregister(m.ctypes.data)
finally:
    os.remove(path)
