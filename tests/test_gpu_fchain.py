"""GPU: the reference-order sums of pp2_fchain.hip equal the reference's
sequential x86 fp32 chains bit for bit (std::accumulate, std::partial_sum,
std::inner_product: search_tree_cuda.cu:168-183, :225-229; evaluateFibCpu
fast_informed_bound_cuda.cu:278-297), on adversarial rows: ties at half an
ulp, binade crossings onto powers of two, subnormals, -0, all-non-positive and
mixed-sign chains, a single huge term, a uniform belief of 65536 cells, and
sizes across the chunk geometry (1 .. 2^20 cells).

The checker is numpy's float32 add.accumulate (one left-to-right fp32 chain,
checked against the oracle's orc_sum_seq below) over IEEE float32 products.
The planner-level parity of the same kernels (children's masses, FIB dots,
rewards, the sampling cdf) is tests/test_gpu_planner.py's reference-order
tests."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_f32p = C.POINTER(C.c_float)


def _fn():
    from path_planning_2d_amd import _lib
    lib = _lib.load()
    f = lib.pp2_debug_fchain_row
    f.argtypes = [C.c_int, _f32p, _f32p, C.c_int, _f32p, _f32p]
    f.restype = C.c_int
    return f


def _ptr(a):
    return a.ctypes.data_as(_f32p) if a is not None else _f32p()


def device_row(x, partners=None, cdf=False):
    x = np.ascontiguousarray(x, np.float32)
    K = 9 if partners is not None else 0
    out = np.zeros(16, np.float32)
    c = np.zeros(x.size, np.float32) if cdf else None
    p = np.ascontiguousarray(partners, np.float32) if partners is not None else None
    st = _fn()(x.size, _ptr(x), _ptr(p), K, _ptr(out), _ptr(c))
    assert st == 0, st
    return out[:9] if K else out[0], c


def seq(t):
    t = np.asarray(t, np.float32)
    # the chain starts at +0.0 (+0.0 + -0.0 = +0.0)
    c = np.add.accumulate(np.concatenate([np.zeros(1, np.float32), t]), dtype=np.float32)[1:]
    return (c[-1] if t.size else np.float32(0.0)), c


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def rows(rng):
    U = lambda n: rng.random(n, dtype=np.float32)  # noqa: E731
    yield "uniform", U(70001)
    yield "wide", np.ldexp(U(65536), -rng.integers(0, 60, 65536)).astype(np.float32)
    yield "constant", np.full(65536, 1.0 / 52429.0, np.float32)
    yield "sparse", np.where(rng.random(65536) < 0.15, U(65536) * 1e-5, 0).astype(np.float32)
    yield "nonpositive", (-U(40000) * 37).astype(np.float32)
    yield "few bits (ties)", np.ldexp(rng.integers(0, 8, 65536), -20).astype(np.float32)
    yield "subnormal", np.ldexp(U(30000), -140).astype(np.float32)
    yield "mixed sign", (U(30000) - 0.5).astype(np.float32)
    t = np.full(3001, np.ldexp(1.0, -25), np.float32)
    t[:3] = [0.5, 0.25, 0.25]
    yield "onto 2^0", t
    t = np.full(5001, np.ldexp(1.0, -24), np.float32)
    t[0] = 1.0
    yield "half-ulp ties", t
    t = U(50000) * 1e-3
    t[25000] = 1e30
    yield "one huge term", t.astype(np.float32)
    t = np.zeros(4096, np.float32)
    t[::2] = -0.0
    yield "-0 and +0", t
    # a concentrated, normalised belief, then a tail far below half an ulp of
    # its sum (entries of d = 0 tabled for the binade below the exact sum's)
    for m, tail in ((200, "tiny"), (3000, "zeros + 2^-26")):
        t = U(m)
        t = (t / seq(t)[0]).astype(np.float32)
        if tail == "tiny":
            tl = np.ldexp(U(60000), -40)
        else:
            tl = np.where(np.arange(60000) % 7 == 0, np.float32(np.ldexp(1.0, -26)), 0)
        yield f"concentrated m={m} + {tail} tail", np.concatenate([t, tl]).astype(np.float32)
    yield "empty", np.zeros(0, np.float32)
    yield "single", np.array([-3.5], np.float32)
    for n in (1, 63, 64, 65, 255, 256, 257, 4000, 65535, 262144 + 7, 1 << 20):
        yield f"n={n}", U(n)


def test_numpy_accumulate_is_the_sequential_chain(oracle):
    rng = np.random.default_rng(3)
    t = rng.random(100003, dtype=np.float32)
    lib = oracle.lib()
    lib.orc_sum_seq.restype = C.c_float
    lib.orc_sum_seq.argtypes = [C.c_size_t, _f32p]
    assert bits(seq(t)[0]) == bits(lib.orc_sum_seq(t.size, _ptr(t)))


@pytest.fixture(params=[1, 0], ids=["walk+sumtab", "drive+two-launch"])
def driver(request):
    """The chain sets' passes: k_fc_sumtab (sums and tables as one launch,
    round 6, opt-in) with k_fc_walk (the default where a chain has <= 1024
    chunks), or k_fc_sums + k_fc_tables (the default) with k_fc_drive (every
    size)."""
    from path_planning_2d_amd import _lib
    lib = _lib.load()
    f, g = lib.pp2_debug_fc_walk, lib.pp2_debug_fc_sumtab
    for h in (f, g):
        h.argtypes = [C.c_int]
        h.restype = C.c_int
    prev, prev2 = f(request.param), g(request.param)
    yield request.param
    f(prev)
    g(prev2)


def test_fchain_sums_and_running_sums_bit_exact(driver):
    rng = np.random.default_rng(11)
    for name, t in rows(rng):
        want, wc = seq(t)
        got, gc = device_row(t, cdf=True)
        assert bits(got) == bits(want), f"{name}: sum {got!r} != {want!r}"
        assert np.array_equal(bits(gc), bits(wc)), \
            f"{name}: running sums differ at {np.flatnonzero(bits(gc) != bits(wc))[:5]}"


def test_fchain_dots_bit_exact(driver):
    """inner_product(x, a_i): the product rounded, then the chain."""
    rng = np.random.default_rng(12)
    for name, t in rows(rng):
        n = t.size
        A = np.empty((9, n), np.float32)
        A[0] = -(20 + 20 * rng.random(n, dtype=np.float32))   # FIB-like alphas
        A[1] = rng.random(n, dtype=np.float32) - 0.5            # mixed sign
        A[2] = 0.0
        A[3] = -2.0                                              # rewards
        A[4] = np.ldexp(1.0, -rng.integers(0, 30, n))
        A[5] = -np.float32(1.0 / 3.0)
        A[6] = rng.random(n, dtype=np.float32) * 1e20
        A[7] = -0.0
        A[8] = 1.0
        got, _ = device_row(t, partners=A)
        for i in range(9):
            want, _ = seq(t * A[i])
            assert bits(got[i]) == bits(want), f"{name} partner {i}: {got[i]!r} != {want!r}"


def test_fchain_pair_dots_bit_exact(driver):
    """The planner's PBVI leaf dots (FC_LIST: evaluatePbviCpu's inner_product
    of a row with an alpha, point_based_value_iteration_cuda.cu:678-699, for
    a device list of (row, alpha) pairs): every listed dot equal to the
    sequential chain, every other entry untouched."""
    from path_planning_2d_amd import _lib
    f = _lib.load().pp2_debug_fchain_pairs
    f.argtypes = [C.c_int, C.c_int, _f32p, C.c_int, _f32p, C.POINTER(C.c_int), C.c_int, _f32p]
    f.restype = C.c_int
    rng = np.random.default_rng(13)
    for n in (4000, 65536, 70001):
        U = lambda k: rng.random(k, dtype=np.float32)  # noqa: E731
        X = np.stack([U(n) / np.float32(n),                                   # a belief
                      np.where(rng.random(n) < 0.1, U(n) * 1e-4, 0),          # sparse
                      np.ldexp(U(n), -rng.integers(0, 40, n)),                # wide
                      np.ldexp(rng.integers(0, 8, n), -20),                   # few bits: ties
                      U(n) - 0.5]).astype(np.float32)                         # mixed sign
        S = 37
        A = -(20 + 40 * rng.random((S, n), dtype=np.float32))                 # PBVI-like alphas
        A[3] = rng.random(n, dtype=np.float32) - 0.5
        A[5] = 0.0
        A[7] = -2.0
        A[11] = np.ldexp(1.0, -rng.integers(0, 30, n))
        A[13] = A[2]                                                          # duplicates
        A[36] = -np.float32(1.0 / 3.0)
        pairs = np.array([(r, i) for r in (3, 0, 4, 1) for i in range(S) if (r + i) % 3 != 1],
                         np.int32)
        rng.shuffle(pairs)
        out = np.full((5, S), np.nan, np.float32)
        st = f(n, 5, _ptr(X), S, _ptr(A), pairs.ctypes.data_as(C.POINTER(C.c_int)), len(pairs),
               _ptr(out))
        assert st == 0, st
        listed = np.zeros((5, S), bool)
        for r, i in pairs:
            listed[r, i] = True
            want, _ = seq(X[r] * A[i])
            assert bits(out[r, i]) == bits(want), f"n={n} row {r} alpha {i}: {out[r, i]!r} != {want!r}"
        assert np.isnan(out[~listed]).all(), "an unlisted entry was written"


# ------------------------------------------------------- fused chain sets (round 6)
def _fx():
    from path_planning_2d_amd import _lib
    f = _lib.load().pp2_debug_fx
    f.argtypes = [C.c_int, C.c_int, _f32p, _f32p, C.c_int, _f32p, _f32p, C.POINTER(C.c_int),
                  C.c_int, _f32p, _f32p, _f32p, _f32p]
    f.restype = C.c_int
    return f


def fx_row(x, partners=None, cdf=False):
    x = np.ascontiguousarray(x, np.float32)
    K = 9 if partners is not None else 0
    out = np.zeros(16, np.float32)
    c = np.zeros(x.size, np.float32) if cdf else None
    p = np.ascontiguousarray(partners, np.float32) if partners is not None else None
    st = _fx()(0, x.size, _ptr(x), _ptr(p), K, None, None, None, 0, _ptr(out), _ptr(c), None, None)
    assert st == 0, st
    return out[:9] if K else out[0], c


def fx_rows(rng):
    for name, t in rows(rng):
        if 0 < t.size <= 65536:
            yield name, t
    U = lambda n: rng.random(n, dtype=np.float32)  # noqa: E731
    for n in (8193, 16384, 16385, 32768, 32769, 65536):
        yield f"n={n}", U(n)
    b = U(65536)
    yield "a 256^2 belief", (b / b.sum(dtype=np.float64)).astype(np.float32)


def test_fx_sums_and_running_sums_bit_exact():
    """k_fx_chain / k_fx_cdf_sample (one launch per chain set, the terms in
    registers) against the sequential chain on the adversarial rows that fit
    one workgroup (n <= 65536)."""
    rng = np.random.default_rng(11)
    for name, t in fx_rows(rng):
        want, wc = seq(t)
        got, _ = fx_row(t)
        assert bits(got) == bits(want), f"{name}: sum {got!r} != {want!r}"
        got, gc = fx_row(t, cdf=True)
        assert bits(got) == bits(want), f"{name}: cdf kernel's sum {got!r} != {want!r}"
        assert np.array_equal(bits(gc), bits(wc)), \
            f"{name}: running sums differ at {np.flatnonzero(bits(gc) != bits(wc))[:5]}"


def test_fx_dots_bit_exact():
    rng = np.random.default_rng(12)
    for name, t in fx_rows(rng):
        n = t.size
        A = np.empty((9, n), np.float32)
        A[0] = -(20 + 20 * rng.random(n, dtype=np.float32))
        A[1] = rng.random(n, dtype=np.float32) - 0.5
        A[2] = 0.0
        A[3] = -2.0
        A[4] = np.ldexp(1.0, -rng.integers(0, 30, n))
        A[5] = -np.float32(1.0 / 3.0)
        A[6] = rng.random(n, dtype=np.float32) * 1e20
        A[7] = -0.0
        A[8] = 1.0
        got, _ = fx_row(t, partners=A)
        for i in range(9):
            want, _ = seq(t * A[i])
            assert bits(got[i]) == bits(want), f"{name} partner {i}: {got[i]!r} != {want!r}"


def ftz(v):
    v = np.asarray(v, np.float32)
    return np.where(np.abs(v) < np.finfo(np.float32).tiny, np.copysign(np.float32(0), v), v)


@pytest.mark.parametrize("n", [9000, 40000, 65536])
def test_fx_children_and_kept_dots_bit_exact(n):
    """FX_CHILD (the 144 children's masses: accumulate of fl_ftz(pred_a *
    fl_ftz(L_z)), search_tree_cuda.cu:225-227) and FX_KEPT (the kept
    children normalised, :228-229, and their 9 FIB dots, evaluateFibCpu)
    against numpy: masses, stored rows and dots bit for bit."""
    rng = np.random.default_rng(n)
    pred = (rng.random((9, n), dtype=np.float32) / np.float32(n)).astype(np.float32)
    pred[:, rng.random(n) < 0.3] = 0.0
    pred[3] = np.ldexp(pred[3], -100)                 # products into the FTZ range
    L = rng.random((16, n), dtype=np.float32)
    L[5, ::7] = np.float32(1e-39)                     # subnormal likelihoods flushed
    L[9] = 0.0
    A = -(20 + 20 * rng.random((9, n), dtype=np.float32))
    A[4] = rng.random(n, dtype=np.float32) - 0.5
    # kept children have mass (the planner keeps sampled observations only)
    live = [c for c in range(144) if seq(ftz(pred[c % 9] * ftz(L[c // 9])))[0] > 0]
    klist = np.array(sorted(rng.choice(live, 46, replace=False)), np.int32)
    out = np.zeros(144 + 144 * 9, np.float32)
    rows_ = np.zeros((144, n), np.float32)
    st = _fx()(1, n, None, _ptr(A), 9, _ptr(pred), _ptr(L),
               klist.ctypes.data_as(C.POINTER(C.c_int)), len(klist), _ptr(out), None,
               _ptr(rows_), None)
    assert st == 0, st
    for c in range(144):
        a, z = c % 9, c // 9
        v = ftz(pred[a] * ftz(L[z]))
        m, _ = seq(v)
        assert bits(out[c]) == bits(m), f"child {c}: mass {out[c]!r} != {m!r}"
        if c in klist:
            b = (v / m).astype(np.float32)
            assert np.array_equal(bits(rows_[c]), bits(b)), f"child {c}: row"
            for i in range(9):
                want, _ = seq(b * A[i])
                got = out[144 + 9 * c + i]
                assert bits(got) == bits(want), f"child {c} dot {i}: {got!r} != {want!r}"


@pytest.mark.parametrize("n,opts", [(9000, 0), (9000, 1), (9000, 3), (65536, 1), (65536, 3)])
def test_fc_kept_sets_bit_exact(n, opts):
    """The planner's chain sets for an expansion (pp2_debug_fx mode 2, as
    pp2_tree.cpp runs them): FC_CHILD masses, then the kept children's
    FC_KEPT sums, tables (normalised rows stored) and walk -- with the sums
    over the unnormalised cells (opts bit 0, kept_unit) and the FIB candidate
    masks (bit 1: a pruned dot is -inf, the first maximum stays) -- against
    numpy: masses, rows and dots bit for bit.  Alphas: negative, one mixed-sign
    row, one positive row, one row of tiny magnitudes (products that underflow
    unnormalised, not normalised)."""
    rng = np.random.default_rng(n + 7 * opts)
    pred = (rng.random((9, n), dtype=np.float32) / np.float32(n)).astype(np.float32)
    pred[:, rng.random(n) < 0.3] = 0.0
    pred[3] = np.ldexp(pred[3], -100)                 # products into the FTZ range
    L = rng.random((16, n), dtype=np.float32)
    L[5, ::7] = np.float32(1e-39)                     # subnormal likelihoods flushed
    L[9] = 0.0
    A = -(20 + 20 * rng.random((9, n), dtype=np.float32))
    A[4] = rng.random(n, dtype=np.float32) - 0.5
    A[7] = 20 + 20 * rng.random(n, dtype=np.float32)
    A[8] = -np.ldexp(rng.random(n, dtype=np.float32) + 0.5, -30)
    live = [c for c in range(144) if seq(ftz(pred[c % 9] * ftz(L[c // 9])))[0] > 0]
    klist = np.array(sorted(rng.choice(live, 46, replace=False)), np.int32)
    out = np.zeros(144 + 144 * 9, np.float32)
    rows_ = np.zeros((144, n), np.float32)
    st = _fx()(2, n, None, _ptr(A), opts, _ptr(pred), _ptr(L),
               klist.ctypes.data_as(C.POINTER(C.c_int)), len(klist), _ptr(out), None,
               _ptr(rows_), None)
    assert st == 0, st
    for c in range(144):
        a, z = c % 9, c // 9
        v = ftz(pred[a] * ftz(L[z]))
        m, _ = seq(v)
        assert bits(out[c]) == bits(m), f"child {c}: mass {out[c]!r} != {m!r}"
        if c not in klist:
            continue
        b = (v / m).astype(np.float32)
        assert np.array_equal(bits(rows_[c]), bits(b)), f"child {c}: row"
        want = np.array([seq(b * A[i])[0] for i in range(9)], np.float32)
        got = out[144 + 9 * c:144 + 9 * c + 9]
        if opts & 2:
            # (first_max9: the value of the first maximum)
            assert bits(np.float32(max(got.tolist()))) == bits(np.float32(max(want.tolist()))), c
            kept = got != -np.inf
            assert np.array_equal(bits(got[kept]), bits(want[kept])), f"child {c}: kept dots"
        else:
            assert np.array_equal(bits(got), bits(want)), f"child {c}: dots {got} != {want}"


@pytest.mark.parametrize("ksplit", [1, 4])
def test_pbvi_candidate_filter_finds_the_first_maximum(ksplit):
    """The opt-in PBVI candidate filter (k_pbvi_cands after the split-x MFMA
    GEMM, its error bound priced from launch_gemm_nt's own kchunk through
    gemm_kchunk; round-5 ADVICE) never drops the true maximum: alphas
    clustered within a few ulps of each other, exact duplicates (the first
    one wins) and a mixed-sign alpha, against the brute-force first argmax of
    every sequential chain (evaluatePbviCpu, point_based_value_iteration_cuda.cu:678-699)."""
    from path_planning_2d_amd import _lib
    f = _lib.load().pp2_debug_pbvi_cands
    f.argtypes = [C.c_int, C.c_int, _f32p, C.c_int, _f32p, C.c_int, C.POINTER(C.c_int), _f32p,
                  C.POINTER(C.c_int)]
    f.restype = C.c_int
    rng = np.random.default_rng(40 + ksplit)
    n, R, S = 3000, 6, 150
    X = rng.random((R, n), dtype=np.float32)
    X[1, rng.random(n) < 0.8] = 0.0
    X[2] = np.ldexp(X[2], -rng.integers(0, 20, n))
    X = (X / X.sum(axis=1, keepdims=True, dtype=np.float64)).astype(np.float32)
    base = -(20 + 20 * rng.random(n, dtype=np.float32))
    A = np.empty((S, n), np.float32)
    for i in range(S):  # within a few ulps of base
        A[i] = np.nextafter(base, np.float32(0)) if i % 3 == 0 else base
        k = rng.integers(0, n, 5)
        A[i, k] = base[k] + np.float32(i % 7) * np.spacing(base[k])
    A[77] = A[13]                                  # exact duplicate: the first wins
    A[90] = rng.random(n, dtype=np.float32) - 30.0
    A[91] = rng.random(n, dtype=np.float32) - 0.5  # mixed sign
    idx = np.zeros(R, np.int32)
    val = np.zeros(R, np.float32)
    nc = C.c_int(0)
    st = f(n, R, _ptr(X), S, _ptr(A), ksplit, idx.ctypes.data_as(C.POINTER(C.c_int)), _ptr(val),
           C.byref(nc))
    assert st == 0, st
    for r in range(R):
        vals = np.array([seq(X[r] * A[i])[0] for i in range(S)], np.float32)
        want = int(np.argmax(vals))
        assert idx[r] == want, (r, idx[r], want, vals[idx[r]], vals[want])
        assert bits(val[r]) == bits(vals[want])
    assert 0 < nc.value < R * S  # the filter dropped some, kept the maximum
