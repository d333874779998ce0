"""Timing-only ablation of the XCD-resident kernel (VH_TILE_DEBUG bits; results wrong by
construction for nonzero bits): 256 consumers only acknowledge, 512 no slot stores, 1024 no
cold-region stores, 2048 loads + cell math only (consumers see no batches: aborts by timeout
are avoided because every producer still publishes nb)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vaex_amd import _lib, superagg
    from vaex_amd.device import DeviceArray
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    x = DeviceArray.random(n, "normal", seed=2)
    y = DeviceArray.random(n, "normal", seed=3)
    w = DeviceArray.random(n, "uniform", seed=4)
    for sums in ((False, True) if os.environ.get("ABL_SUMS", "1") == "1" else (False,)):
        for dbg in [int(v) for v in os.environ.get("ABL", "0,256,768,1792,2304,6144").split(",")]:
            os.environ["VH_TILE_DEBUG"] = str(dbg)

            def step():
                bx = superagg.BinnerScalar_float64("x", -4.0, 4.0, 1024)
                by = superagg.BinnerScalar_float64("y", -4.0, 4.0, 1024)
                bx.set_data(x)
                by.set_data(y)
                grid = superagg.Grid([bx, by])
                aggs = [superagg.AggCount_int64(grid)]
                if sums:
                    aggs.append(superagg.AggSum_float64(grid))
                    aggs[1].set_data(w, 0)
                grid.bin(aggs)
            step()
            _lib.synchronize()
            _lib.timing_reset()
            _lib.timing_enable(True)
            for _ in range(3):
                step()
            _lib.synchronize()
            _lib.timing_enable(False)
            per = {}
            for k in ("tile_scatter_f64", "tile_resident", "tile_reduce"):
                c, ms = _lib.timing_read(k)
                if c:
                    per[k] = round(ms / c, 3)
            print(f"sums={sums} debug={dbg:5d} {per}", flush=True)
    os.environ["VH_TILE_DEBUG"] = "0"


if __name__ == "__main__":
    main()
