"""Diagnostic: the device's chunk sums and table entries for the uniform 256^2
belief (pp2_debug_fchain_tables) against a numpy restatement of k_fc_sums /
k_fc_tables, and where the driver's chunk start states sit."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from path_planning_2d_amd import _lib, synthetic as S
    lib = _lib.load()
    f = lib.pp2_debug_fchain_tables
    fp = C.POINTER(C.c_float)
    f.argtypes = [C.c_int, fp, fp, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
    g = S.synth_grid(256, 256, seed=256)
    b = S.uniform_belief(g)
    n = b.size
    nch = (n + 255) // 256
    cs = np.zeros(nch, np.float32)
    tab = np.zeros(2 * nch, np.uint32)
    cst = np.zeros(2 * (nch + 1), np.int32)
    rc = f(n, b.ctypes.data_as(fp), cs.ctypes.data_as(fp),
           tab.ctypes.data_as(C.POINTER(C.c_uint32)), cst.ctypes.data_as(C.POINTER(C.c_int)))
    assert rc == 0, rc
    want = b.reshape(nch, 256).astype(np.float64).sum(1)
    print("csum rel err max", float(np.max(np.abs(cs - want) / np.maximum(want, 1e-30))))
    P = np.concatenate([[0.0], np.cumsum(want)[:-1]]).astype(np.float32)
    e = tab[0::2]
    E = (e >> 24).astype(np.int64) - 128
    d = e & 0xffffff
    ne = int((e == 0xffffffff).sum())
    Pe = ((P.view(np.uint32) >> 23) & 0xff).astype(np.int64)
    Pd = np.where(Pe <= 1, -126, Pe - 127)
    print("no-entry", ne, "of", nch, "; E == domain(P):", int((E == Pd)[e != 0xffffffff].sum()))
    for j in (0, 1, 2, 100, 200, 255):
        u = 2.0 ** (int(Pd[j]) - 23)
        print(j, "P", P[j], "tabE", int(E[j]), "domP", int(Pd[j]), "d", int(d[j]),
              "expect d", int(np.rint(b[j * 256:(j + 1) * 256].astype(np.float64) / u).sum()),
              "flags", int(tab[2 * j + 1]), "start", cst[2 * j], cst[2 * j + 1])


if __name__ == "__main__":
    main()
