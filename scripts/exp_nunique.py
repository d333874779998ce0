"""nunique timing: df.count-style binned AggNUnique over HBM columns (1e8 rows, 300 cells),
low-cardinality int8 values and high-cardinality int32 values.  Run with VH_NU_LDS=0 / 1."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vaex_amd import _lib, superagg as sa
    from vaex_amd.device import DeviceArray
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    rng = np.random.default_rng(1)
    x = DeviceArray.from_numpy(rng.integers(0, 300, n).astype(np.int64))
    for name, v in (("int8 card 100", rng.integers(0, 100, n).astype(np.int8)),
                    ("int32 card 1e6", rng.integers(0, 1_000_000, n).astype(np.int32))):
        dv = DeviceArray.from_numpy(v)

        def run():
            b = sa.BinnerOrdinal_int64("x", 300, 0)
            b.set_data(x)
            g = sa.Grid([b])
            a = getattr(sa, "AggNUnique_" + v.dtype.name)(g, False, False)
            a.set_data(dv, 0)
            g.bin([a])
            return np.asarray(a).copy()
        r = run()
        _lib.synchronize()
        _lib.timing_reset()
        _lib.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(3):
            run()
        t = (time.perf_counter() - t0) / 3
        _lib.timing_enable(False)
        per = {}
        for k in ("nunique_collect", "nunique_dedup"):
            c, ms = _lib.timing_read(k)
            if c:
                per[k] = round(ms / c, 3)
        print(f"VH_NU_LDS={os.environ.get('VH_NU_LDS', '0')} {name}: {t * 1e3:.2f} ms/query {per} total={int(r.sum())}",
              flush=True)


if __name__ == "__main__":
    main()
