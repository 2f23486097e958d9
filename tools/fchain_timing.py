"""Timing and driver statistics of one reference-order chain set
(pp2_fchain.hip) on realistic 256^2 rows: the uniform belief's accumulate
with its running sums (the sampling cdf), a child belief's accumulate, and
FIB-like / reward inner products.  Diagnostic (tools/), via the library's
pp2_debug_fchain_row2 entry point."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from path_planning_2d_amd import _lib, synthetic as S
    from oracle import oracle as O
    lib = _lib.load()
    f = lib.pp2_debug_fchain_row2
    fp = C.POINTER(C.c_float)
    f.argtypes = [C.c_int, fp, fp, C.c_int, fp, fp, C.POINTER(C.c_int), fp]
    N = int(os.environ.get("PP2_N", "256"))
    g = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(g)
    T, L, R = O.model_pomdp(g, goal)
    b = S.uniform_belief(g)
    c = O.belief_update(N, N, T, L, b, 3, 5)
    cn = (c / np.float32(c.sum(dtype=np.float64))).astype(np.float32)
    A = np.stack([np.float32(-20.0 - i) + np.zeros(N * N, np.float32) for i in range(9)])
    A += -np.random.default_rng(1).random((9, N * N), dtype=np.float32)
    Rr = np.ascontiguousarray(R.reshape(-1, 9).T)
    cases = [("uniform belief, accumulate + cdf", b, None, True),
             ("child, accumulate", c, None, False),
             ("child, 9 FIB-like dots", cn, A, False),
             ("uniform belief, 9 reward dots", b, Rr, False)]
    for name, x, P, cdf in cases:
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros(16, np.float32)
        cd = np.zeros(x.size, np.float32) if cdf else None
        st = (C.c_int * 8)()
        ms = C.c_float()
        Pp = np.ascontiguousarray(P, np.float32) if P is not None else None
        rc = f(x.size, x.ctypes.data_as(fp), Pp.ctypes.data_as(fp) if Pp is not None else fp(),
               9 if P is not None else 0, out.ctypes.data_as(fp),
               cd.ctypes.data_as(fp) if cd is not None else fp(), st, C.byref(ms))
        assert rc == 0, rc
        nc = max(1, st[7])
        print(f"{name:36s} {ms.value * 1e3:8.1f} us  driver: iterations {st[0]}, fallback "
              f"chunks {st[1]}, exact rounds {st[2]}, stash hits {st[3]}; per chain: flags "
              f"{st[4] / nc / 100:.1f} us, window+stash {st[5] / nc / 100:.1f} us, walk "
              f"{st[6] / nc / 100:.1f} us", flush=True)


if __name__ == "__main__":
    main()
