"""ctypes/numpy wrapper over the CPU oracle (``oracle/libpp2_oracle.so``).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module; the product
package ``path_planning_2d_amd`` never does.  Parity is unpinned by reference
tests (the reference ships none) -- see ``pp2_oracle.h`` for the citations each
function follows.

All arrays use the reference layouts: ``T[hw, 9, 9]``, ``L[hw, 16]``,
``R/C[hw, 9]`` with ``idx = y * W + x``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpp2_oracle.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in
            ("pp2_oracle.c", "pp2_oracle_tree.c", "pp2_oracle_pbvi.c", "pp2_oracle.h")]
    if force or not os.path.exists(LIB_PATH) or any(
            os.path.getmtime(LIB_PATH) < os.path.getmtime(s) for s in srcs):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        I, F, D, S = C.c_int, C.c_float, C.c_double, C.c_size_t
        sig = {
            "orc_model_pomdp": (None, [I, I, _u8p, I, I, _f32p, _f32p, _f32p]),
            "orc_model_mdp": (None, [I, I, _u8p, I, I, _f32p, _f32p]),
            "orc_belief_update": (None, [I, I, _f32p, _f32p, _f32p, I, I, _f32p, I]),
            "orc_belief_update_rows": (None, [I, I, _f32p, _f32p, _f32p, I, I, _f32p, I, I, I]),
            "orc_normalize_seq": (F, [S, _f32p]),
            "orc_normalize_f64": (D, [S, _f32p]),
            "orc_sum_seq": (F, [S, _f32p]),
            "orc_sum_f64": (D, [S, _f32p]),
            "orc_mdp_sweep": (None, [I, I, F, _f32p, _f32p, _f32p, _f32p, _u8p]),
            "orc_mdp_sweep_rows": (None, [I, I, F, _f32p, _f32p, _f32p, _f32p, _u8p, I, I]),
            "orc_loop_run_mt": (I, [I, I, F, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                    _u8p, I, _u8p, _u8p, I]),
            "orc_mdp_solve": (I, [I, I, F, _f32p, _f32p, _f32p, _u8p, I, C.POINTER(D)]),
            "orc_fib_sweep": (None, [I, I, F, _f32p, _f32p, _f32p, _f32p, _f32p]),
            "orc_fib_solve": (I, [I, I, F, _f32p, _f32p, _f32p, _f32p, I, C.POINTER(F)]),
            "orc_fib_eval": (None, [S, _f32p, _f32p, C.POINTER(F), C.POINTER(C.c_uint8)]),
            "orc_reward_dot": (F, [S, _f32p, _f32p, I]),
            "orc_sim_predict": (None, [I, I, _u8p, _f32p, I, _f32p]),
            "orc_sim_correct": (None, [I, I, _u8p, _f32p, I, _f32p]),
            "orc_curand_xorwow": (None, [C.c_uint64, C.c_uint64, C.c_uint64, I, _u32p]),
            "orc_curand_uniform": (F, [C.c_uint32]),
            "orc_synth_map": (None, [I, I, C.c_uint64, D, _u8p]),
            "orc_synth_goal": (I, [I, I, _u8p, C.POINTER(I), C.POINTER(I)]),
            "orc_synth_trajectory": (I, [I, I, _u8p, I, I, C.c_uint64, I, _u8p, _u8p, _i32p]),
            "orc_rand_seed": (None, [C.c_void_p, C.c_uint32]),
            "orc_rand_next": (C.c_int32, [C.c_void_p]),
            "orc_pbvi_belief_set": (I, [I, I, _f32p, _f32p, _f32p, I, C.c_void_p, _f32p]),
            "orc_pbvi_backup": (I, [I, I, F, _f32p, _f32p, _f32p, I, _f32p, _f32p, _u8p, I]),
            "orc_pbvi_iterations": (I, [F]),
            "orc_pbvi_eval": (None, [S, _f32p, I, _f32p, _u8p, C.POINTER(F),
                                     C.POINTER(C.c_uint8)]),
            "orc_heap_sort_desc": (None, [S, _f32p, np.ctypeslib.ndpointer(np.uintp,
                                                                          flags="C_CONTIGUOUS")]),
            "orc_planner_create": (C.c_void_p, [I, I, _f32p, _f32p, _f32p, _f32p, F, I, I,
                                                C.c_uint32, C.c_uint32, C.c_uint64, I]),
            "orc_planner_step": (I, [C.c_void_p, C.c_uint8, C.c_uint8, C.c_void_p,
                                     C.POINTER(C.c_uint8), C.POINTER(F)]),
            "orc_planner_reset": (None, [C.c_void_p]),
            "orc_planner_set_pbvi": (None, [C.c_void_p, I, _f32p, _u8p]),
            "orc_planner_skip_rand": (None, [C.c_void_p, C.c_uint64]),
            "orc_planner_info": (None, [C.c_void_p, C.c_void_p]),
            "orc_planner_destroy": (None, [C.c_void_p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# ---------------------------------------------------------------- model
def model_pomdp(grid: np.ndarray, goal):
    H, W = grid.shape
    hw = H * W
    T = np.zeros((hw, 9, 9), np.float32)
    Lk = np.zeros((hw, 16), np.float32)
    R = np.zeros((hw, 9), np.float32)
    lib().orc_model_pomdp(H, W, np.ascontiguousarray(grid, np.uint8),
                          int(goal[0]), int(goal[1]), T, Lk, R)
    return T, Lk, R


def model_mdp(grid: np.ndarray, goal):
    H, W = grid.shape
    hw = H * W
    T = np.zeros((hw, 9, 9), np.float32)
    Cc = np.zeros((hw, 9), np.float32)
    lib().orc_model_mdp(H, W, np.ascontiguousarray(grid, np.uint8),
                        int(goal[0]), int(goal[1]), T, Cc)
    return T, Cc


# ---------------------------------------------------------------- belief
def belief_update(H, W, T, L, b, u, z, ftz=True):
    out = np.empty(H * W, np.float32)
    lib().orc_belief_update(H, W, T, L, np.ascontiguousarray(b, np.float32),
                            int(u), int(z), out, int(ftz))
    return out


def normalize_seq(b):
    b = np.array(b, np.float32, copy=True)
    s = lib().orc_normalize_seq(b.size, b)
    return b, s


def normalize_f64(b):
    b = np.array(b, np.float32, copy=True)
    s = lib().orc_normalize_f64(b.size, b)
    return b, s


def belief_step(H, W, T, L, b, u, z, mode="seq"):
    """One reference plan-tree belief step: kernel + host renormalisation
    (search_tree_cuda.cu:601-612)."""
    out = belief_update(H, W, T, L, b, u, z)
    return normalize_seq(out)[0] if mode == "seq" else normalize_f64(out)[0]


# ---------------------------------------------------------------- MDP
def mdp_sweep(H, W, gamma, T, Cc, J):
    Jo = np.empty(H * W, np.float32)
    A = np.empty(H * W, np.uint8)
    lib().orc_mdp_sweep(H, W, float(gamma), T, Cc,
                        np.ascontiguousarray(J, np.float32), Jo, A)
    return Jo, A


def mdp_solve(H, W, gamma, T, Cc, max_sweeps=0):
    J = np.zeros(H * W, np.float32)
    A = np.zeros(H * W, np.uint8)
    nrm = C.c_double()
    n = lib().orc_mdp_solve(H, W, float(gamma), T, Cc, J, A, int(max_sweeps),
                            C.byref(nrm))
    return J, A, n, nrm.value


# ---------------------------------------------------------------- FIB
def fib_sweep(H, W, gamma, T, L, R, a):
    out = np.empty((H * W, 9), np.float32)
    lib().orc_fib_sweep(H, W, float(gamma), T, L, R,
                        np.ascontiguousarray(a, np.float32), out)
    return out


def fib_solve(H, W, gamma, T, L, R, max_sweeps=0):
    a = np.zeros((H * W, 9), np.float32)
    nrm = C.c_float()
    n = lib().orc_fib_solve(H, W, float(gamma), T, L, R, a, int(max_sweeps),
                            C.byref(nrm))
    return a, n, nrm.value


def fib_eval(b, alphas):
    v = C.c_float()
    a = C.c_uint8()
    lib().orc_fib_eval(b.size, np.ascontiguousarray(b, np.float32),
                       np.ascontiguousarray(alphas, np.float32), C.byref(v),
                       C.byref(a))
    return v.value, a.value


def reward_dot(b, R, a):
    return lib().orc_reward_dot(b.size, np.ascontiguousarray(b, np.float32),
                                np.ascontiguousarray(R, np.float32), int(a))


# ---------------------------------------------------------------- simulator
def sim_step(grid, b, u, z):
    H, W = grid.shape
    g = np.ascontiguousarray(grid, np.uint8)
    p = np.empty(H * W, np.float32)
    lib().orc_sim_predict(H, W, g, np.ascontiguousarray(b, np.float32), int(u), p)
    out = np.empty(H * W, np.float32)
    lib().orc_sim_correct(H, W, g, p, int(z), out)
    return out


# ---------------------------------------------------------------- RNG
def curand_xorwow(seed, subsequence, offset, n):
    out = np.empty(n, np.uint32)
    lib().orc_curand_xorwow(seed, subsequence, offset, n, out)
    return out


def curand_uniform(x):
    return lib().orc_curand_uniform(int(x))


# ---------------------------------------------------------------- synthetic
def synth_map(H, W, seed, p_occ=0.20):
    m = np.empty((H, W), np.uint8)
    lib().orc_synth_map(H, W, seed, p_occ, m)
    return m


def synth_goal(grid):
    H, W = grid.shape
    gx, gy = C.c_int(), C.c_int()
    rc = lib().orc_synth_goal(H, W, np.ascontiguousarray(grid, np.uint8),
                              C.byref(gx), C.byref(gy))
    if rc != 0:
        raise ValueError("no free cell for the goal")
    return gx.value, gy.value


def synth_trajectory(grid, goal, seed, n):
    H, W = grid.shape
    us = np.empty(n, np.uint8)
    zs = np.empty(n, np.uint8)
    st = np.empty(n, np.int32)
    rc = lib().orc_synth_trajectory(H, W, np.ascontiguousarray(grid, np.uint8),
                                    int(goal[0]), int(goal[1]), seed, n, us, zs, st)
    if rc != 0:
        raise ValueError("no free start cell")
    return us, zs, st


# ---------------------------------------------------------------- QV-tree
class TreeInfo(C.Structure):
    _fields_ = [("depth", C.c_uint32), ("root_upper_bound", C.c_float),
                ("root_lower_bound", C.c_float), ("root_heuristic", C.c_float),
                ("n_root_children", C.c_uint32),
                ("q_upper_bound", C.c_float * 9), ("q_lower_bound", C.c_float * 9),
                ("q_reward", C.c_float * 9), ("q_heuristic", C.c_float * 9),
                ("q_depth", C.c_uint32 * 9), ("q_nchildren", C.c_uint32 * 9),
                ("q_obs", (C.c_uint8 * 16) * 9), ("q_weight", (C.c_float * 16) * 9),
                ("v_upper_bound", (C.c_float * 16) * 9),
                ("v_lower_bound", (C.c_float * 16) * 9),
                ("total_vnodes", C.c_uint32), ("total_qnodes", C.c_uint32),
                ("expansions", C.c_uint32)]

    def as_dict(self):
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = np.ctypeslib.as_array(v).copy() if hasattr(v, "_length_") else v
        return out


class Planner:
    """The reference QV-tree planner restated on the host (every node keeps
    its own belief; sequential fp32 sums; linear find_if sampling)."""

    def __init__(self, grid, T, L, R, alphas, gamma=0.95, max_depth=50,
                 max_iter=15, rand_seed=1, sample_num=50, curand_seed=1234,
                 accurate=False):
        H, W = grid.shape
        self.n = H * W
        self._keep = [np.ascontiguousarray(a, np.float32) for a in (T, L, R, alphas)]
        self._h = lib().orc_planner_create(H, W, *self._keep, float(gamma),
                                           int(max_depth), int(max_iter), rand_seed,
                                           sample_num, curand_seed, int(accurate))

    def step(self, action, observation, belief=None):
        a = C.c_uint8()
        v = C.c_float()
        bp = None
        if belief is not None:
            belief = np.ascontiguousarray(belief, np.float32)
            self._b = belief
            bp = belief.ctypes.data_as(C.c_void_p)
        rc = lib().orc_planner_step(self._h, int(action), int(observation), bp,
                                    C.byref(a), C.byref(v))
        if rc != 0:
            raise RuntimeError(f"orc_planner_step failed ({rc})")
        return a.value, v.value

    def reset(self):
        lib().orc_planner_reset(self._h)

    def set_pbvi(self, alphas, actions):
        """Lower bounds from PBVI alpha vectors (evaluatePbviCpu)."""
        self._pbvi = (np.ascontiguousarray(alphas, np.float32),
                      np.ascontiguousarray(actions, np.uint8))
        lib().orc_planner_set_pbvi(self._h, self._pbvi[0].shape[0], *self._pbvi)

    def skip_rand(self, n):
        lib().orc_planner_skip_rand(self._h, int(n))

    def info(self):
        t = TreeInfo()
        lib().orc_planner_info(self._h, C.byref(t))
        return t.as_dict()

    def close(self):
        if self._h:
            lib().orc_planner_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- PBVI
class RandState:
    """glibc rand() state (orc_rand_state), srand(seed)."""

    def __init__(self, seed=1):
        self.buf = C.create_string_buffer(34 * 4 + 8)
        lib().orc_rand_seed(self.buf, int(seed))

    def next(self):
        return lib().orc_rand_next(self.buf)


def pbvi_belief_set(H, W, T, L, b0, S, rand_state=None):
    """generateBeliefSet: (b_set[S, hw], rand state after it)."""
    rs = rand_state or RandState(1)
    out = np.zeros((S, H * W), np.float32)
    st = lib().orc_pbvi_belief_set(H, W, T, L, np.ascontiguousarray(b0, np.float32), int(S),
                                   rs.buf, out)
    if st != 0:
        raise ValueError("orc_pbvi_belief_set failed")
    return out, rs


def pbvi_backup(H, W, gamma, T, L, R, b_set, alphas=None, iterations=0):
    """backupAlphaVectors from `alphas` (zeros by default): (alphas, actions, iters)."""
    S = b_set.shape[0]
    al = (np.zeros((S, H * W), np.float32) if alphas is None
          else np.array(alphas, np.float32, copy=True).reshape(S, H * W))
    act = np.zeros(S, np.uint8)
    n = lib().orc_pbvi_backup(H, W, float(gamma), T, L, R, int(S),
                              np.ascontiguousarray(b_set, np.float32), al, act, int(iterations))
    if n < 0:
        raise MemoryError("orc_pbvi_backup")
    return al, act, n


def pbvi_iterations(gamma):
    return lib().orc_pbvi_iterations(float(gamma))


def pbvi_eval(b, alphas, actions):
    v = C.c_float()
    a = C.c_uint8()
    alphas = np.ascontiguousarray(alphas, np.float32)
    lib().orc_pbvi_eval(b.size, np.ascontiguousarray(b, np.float32), alphas.shape[0], alphas,
                        np.ascontiguousarray(actions, np.uint8), C.byref(v), C.byref(a))
    return v.value, a.value


def heap_sort_desc(key):
    key = np.ascontiguousarray(key, np.float32)
    idx = np.zeros(key.size, np.uintp)
    lib().orc_heap_sort_desc(key.size, key, idx)
    return idx
