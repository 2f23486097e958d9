"""Online QV-tree POMDP planner over a GridContext (C ABI pp2_planner_*).

Mirrors PomdpPathPlanning2d's plan step (src/pomdp/path_planning_2d.cu:199-241)
and its SearchTree (include/path_planning_2d/search_tree.h:31-165): the tree
logic runs in C++ inside libpp2_hip.so, every belief update / renormalisation
/ leaf bound of a VNode expansion is one batched gfx950 pass.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import call
from .core import GridContext


class PlannerParams(C.Structure):
    _fields_ = [("max_search_tree_depth", C.c_int32),
                ("max_online_iteration", C.c_int32),
                ("lower_bound_mode", C.c_int32),
                ("rand_seed", C.c_uint32),
                ("sample_num", C.c_uint32),
                ("curand_seed", C.c_uint64),
                ("rand_skip", C.c_uint64),
                ("reference_order", C.c_int32)]


class TreeInfo(C.Structure):
    _fields_ = [("depth", C.c_uint32),
                ("root_upper_bound", C.c_float),
                ("root_lower_bound", C.c_float),
                ("root_heuristic", C.c_float),
                ("n_root_children", C.c_uint32),
                ("q_upper_bound", C.c_float * 9),
                ("q_lower_bound", C.c_float * 9),
                ("q_reward", C.c_float * 9),
                ("q_heuristic", C.c_float * 9),
                ("q_depth", C.c_uint32 * 9),
                ("q_nchildren", C.c_uint32 * 9),
                ("q_obs", (C.c_uint8 * 16) * 9),
                ("q_weight", (C.c_float * 16) * 9),
                ("v_upper_bound", (C.c_float * 16) * 9),
                ("v_lower_bound", (C.c_float * 16) * 9),
                ("total_vnodes", C.c_uint32),
                ("total_qnodes", C.c_uint32),
                ("expansions", C.c_uint32)]

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = np.ctypeslib.as_array(v).copy() if hasattr(v, "_length_") else v
        return out


def default_params() -> PlannerParams:
    p = PlannerParams()
    call("pp2_planner_default_params", C.byref(p))
    return p


class QVTreePlanner:
    """The POMDP planner node's algorithm without ROS transport.

    Parameters are the launch-file parameters (launch/pomdp_path_planning_2d.
    launch:11-14): ``max_search_tree_depth`` (50), ``max_online_iteration``
    (15); the context must hold the model and FIB alphas (``fib_solve``)."""

    def __init__(self, ctx: GridContext, **params):
        self.ctx = ctx
        prm = default_params()
        for k, v in params.items():
            if not hasattr(prm, k):
                raise TypeError(f"unknown planner parameter {k!r}")
            setattr(prm, k, v)
        self.params = prm
        h = C.c_void_p()
        call("pp2_planner_create", C.byref(h), ctx.handle, C.byref(prm))
        self._h = h

    def step(self, action: int, observation: int, belief=None):
        """One beliefCallback: returns (action, Q upper bound)."""
        bp = C.POINTER(C.c_float)()
        if belief is not None:
            belief = np.ascontiguousarray(belief, np.float32).reshape(self.ctx.cells)
            bp = belief.ctypes.data_as(C.POINTER(C.c_float))
        a = C.c_uint8()
        v = C.c_float()
        call("pp2_planner_step", self._h, int(action), int(observation), bp,
             C.byref(a), C.byref(v))
        return a.value, v.value

    def reset(self):
        call("pp2_planner_reset", self._h)

    def info(self) -> dict:
        t = TreeInfo()
        call("pp2_planner_info", self._h, C.byref(t))
        return t.as_dict()

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            from ._lib import load
            load().pp2_planner_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def curand_uniforms(seed: int, n: int):
    """(u1, u2): the two curand_uniform draws of curand_init(seed, i, 0)."""
    u1 = np.empty(n, np.float32)
    u2 = np.empty(n, np.float32)
    call("pp2_curand_uniforms", C.c_uint64(seed), int(n),
         u1.ctypes.data_as(C.POINTER(C.c_float)),
         u2.ctypes.data_as(C.POINTER(C.c_float)))
    return u1, u2


class BatchedRollout:
    """Batched fp16 QV-tree rollouts (pp2_rollout_*; BASELINE configs[4]):
    ``copies`` copies of a root belief, each following its own ``depth``-step
    (u, z) sequence; per-copy rewards, observation likelihoods, FIB leaf bound
    and discounted value."""

    def __init__(self, ctx: GridContext, copies: int, depth: int):
        self.ctx = ctx
        self.copies = int(copies)
        self.depth = int(depth)
        h = C.c_void_p()
        call("pp2_rollout_create", C.byref(h), ctx.handle, self.copies, self.depth)
        self._h = h

    def set_root(self, belief):
        b = np.ascontiguousarray(belief, np.float32).reshape(self.ctx.cells)
        call("pp2_rollout_set_root", self._h, b.ctypes.data_as(C.POINTER(C.c_float)))

    def run(self, us, zs):
        us = np.ascontiguousarray(us, np.uint8).reshape(self.depth, self.copies)
        zs = np.ascontiguousarray(zs, np.uint8).reshape(self.depth, self.copies)
        call("pp2_rollout_run", self._h, us.ctypes.data_as(C.POINTER(C.c_uint8)),
             zs.ctypes.data_as(C.POINTER(C.c_uint8)))

    def results(self):
        f = C.POINTER(C.c_float)
        r = np.empty((self.depth, self.copies), np.float32)
        p = np.empty((self.depth, self.copies), np.float32)
        ub = np.empty(self.copies, np.float32)
        v = np.empty(self.copies, np.float32)
        call("pp2_rollout_results", self._h, r.ctypes.data_as(f), p.ctypes.data_as(f),
             ub.ctypes.data_as(f), v.ctypes.data_as(f))
        return {"rewards": r, "obs_prob": p, "leaf_upper": ub, "value": v}

    def belief(self, copy: int):
        out = np.empty(self.ctx.cells, np.float32)
        call("pp2_rollout_get_belief", self._h, int(copy),
             out.ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            from ._lib import load
            load().pp2_rollout_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
