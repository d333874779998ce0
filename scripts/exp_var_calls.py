"""C-ABI call log of one var(w, binby=[x, y], shape=1024) query over 1e9 resident rows (the
bench's var leg), after warm-up: host time between library calls and time inside them."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vaex_amd  # noqa: E402
from vaex_amd import _lib  # noqa: E402
from vaex_amd.device import DeviceArray  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10 ** 9
df = vaex_amd.from_arrays(x=DeviceArray.random(n, "normal", seed=2), y=DeviceArray.random(n, "normal", seed=3),
                          w=DeviceArray.random(n, "uniform", seed=4))
q = lambda: df.var("w", binby=["x", "y"], limits=[[-4, 4], [-4, 4]], shape=1024)  # noqa: E731
for _ in range(3):
    q()
log = []
orig = _lib.call
T0 = [0.0]


def traced(name, *a):
    t = time.perf_counter()
    try:
        return orig(name, *a)
    finally:
        log.append((name, t - T0[0], time.perf_counter() - T0[0]))


_lib.call = traced
for rep in range(3):
    log.clear()
    _lib.synchronize()
    T0[0] = time.perf_counter()
    q()
    _lib.synchronize()
    total = time.perf_counter() - T0[0]
print(f"query {total * 1e3:.3f} ms")
prev = 0.0
for name, a, b in log:
    if (b - a) > 0.05e-3 or (a - prev) > 0.05e-3:
        print(f"{a * 1e3:8.3f} +{(a - prev) * 1e3:6.3f} host | {(b - a) * 1e3:7.3f} in call  {name}")
    prev = b
