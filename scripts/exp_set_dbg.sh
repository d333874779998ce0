for d in 0 1 2 3; do VH_SI_DEBUG=$d timeout -k 10 120 python3 scripts/exp_set.py 1e9 2 2>&1 | tail -1 | sed "s/^/dbg=$d /"; done
