"""Host-side handle over one ``pp2_ctx`` (a grid, or a row shard of one, on one
MI355X).  Thin numpy-facing layer over the C ABI in include/pp2.h; every call
goes to the gfx950 kernels in libpp2_hip.so -- there is no CPU path.

Arrays use the reference layouts (path_planning_2d/src/pomdp/
model_generation_cuda.cu:27-38): ``T[hw, 9, 9]``, ``L[hw, 16]``,
``R/C[hw, 9]``, beliefs and values ``[hw]`` with ``idx = y * W + x``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import call


def _f32(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


_NULLF = C.POINTER(C.c_float)()


class GridContext:
    """One device-resident grid: model tensors, belief, MDP values, FIB alphas.

    Mirrors the state the reference keeps in its ``dev_*``/``host_*`` globals
    (src/mdp/path_planning_2d_cuda.cu:26-38, src/pomdp/model_generation_cuda.cu:
    27-38, src/pomdp/fast_informed_bound_cuda.cu:43-51).
    """

    def __init__(self, grid: np.ndarray, goal, gamma: float = 0.95,
                 device: int = 0, rows: tuple[int, int] | None = None):
        grid = np.ascontiguousarray(grid, dtype=np.uint8)
        if grid.ndim != 2:
            raise ValueError("grid must be 2-D (H, W)")
        self.global_height, self.width = grid.shape
        self.goal = (int(goal[0]), int(goal[1]))
        self.gamma = float(gamma)
        self.device = int(device)
        h = C.c_void_p()
        if rows is None:
            call("pp2_create", C.byref(h), self.device, self.global_height,
                 self.width, _u8(grid), self.goal[0], self.goal[1],
                 C.c_float(self.gamma))
            self.row_begin, self.row_end = 0, self.global_height
        else:
            r0, r1 = int(rows[0]), int(rows[1])
            call("pp2_create_shard", C.byref(h), self.device,
                 self.global_height, self.width, r0, r1, _u8(grid),
                 self.goal[0], self.goal[1], C.c_float(self.gamma))
            self.row_begin, self.row_end = r0, r1
        self._h = h
        self.rows = self.row_end - self.row_begin
        self.cells = self.rows * self.width
        rs = C.c_uint32()
        call("pp2_get_geometry", self._h, None, None, C.byref(rs), None)
        self.row_stride = rs.value

    # ------------------------------------------------------------ lifetime
    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().pp2_destroy(self._h)
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

    def set_stream(self, stream_handle: int | None):
        call("pp2_set_stream", self._h, C.c_void_p(stream_handle or 0))

    def synchronize(self):
        call("pp2_synchronize", self._h)

    def set_cells_per_lane(self, cpt: int):
        call("pp2_set_cells_per_lane", self._h, int(cpt))

    TUNE_CELLS_PER_LANE = 1
    TUNE_NT_STREAMS = 2
    TUNE_CODED_MODEL = 3
    TUNE_HALO_DEPTH = 4
    TUNE_COMM_STREAM = 5
    TUNE_NORM_BLOCK = 6
    TUNE_STEP_PAIRS = 7
    TUNE_RESIDENT = 8
    TUNE_RESIDENT_HALO = 9
    TUNE_RESIDENT_CUS = 10
    TUNE_RESIDENT_STALL = 11
    TUNE_RESIDENT_TILE_COLS = 12
    TUNE_SHARD_LAG = 13
    TUNE_COMM_TIMING = 14

    def set_tuning(self, key: int, value: int):
        call("pp2_set_tuning", self._h, int(key), int(value))

    def comm_rounds(self, max_rounds: int = 256):
        """The RCCL rounds timed since TUNE_COMM_TIMING was set or the last
        call (pp2_comm_rounds): (durations in us as a float32 array, rounds
        beyond the 256 timed ones).  Synchronises; clears the record."""
        n = C.c_int(0)
        dropped = C.c_longlong(0)
        buf = np.zeros(max(1, max_rounds), np.float32)
        call("pp2_comm_rounds", self._h, C.byref(n), C.byref(dropped), _f32(buf),
             int(max_rounds))
        return buf[:min(n.value, max_rounds)].copy(), dropped.value

    # ------------------------------------------------------------ model
    def model_generate(self):
        call("pp2_model_generate", self._h)

    def model_dict_info(self):
        """(entries, active) of the dictionary-coded model (pp2_model_dict_info)."""
        e, a = C.c_int(0), C.c_int(0)
        call("pp2_model_dict_info", self._h, C.byref(e), C.byref(a))
        return e.value, bool(a.value)

    def resident_launches(self):
        """(tile-resident loop launches, resident MDP-solve launches) so far."""
        lo = C.c_int()
        so = C.c_int()
        call("pp2_resident_launches", self._h, C.byref(lo), C.byref(so))
        return lo.value, so.value

    def resident_status(self):
        """(resident launches re-run after a timeout, resident kernels enabled)."""
        f = C.c_int()
        e = C.c_int()
        call("pp2_resident_status", self._h, C.byref(f), C.byref(e))
        return f.value, bool(e.value)

    def loop_steps_per_launch(self) -> int:
        """Loop steps one kernel launch of pp2_loop_run covers (2048 resident,
        the resident halo depth on a shard, 2 for step pairs, else 1)."""
        n = C.c_int(0)
        call("pp2_loop_steps_per_launch", self._h, C.byref(n))
        return n.value

    def resident_tiling(self):
        """(tiles, rows per tile, tile columns) of the resident loop on this
        context, (0, 0, 0) when it does not run resident."""
        t, r, c = C.c_int(0), C.c_int(0), C.c_int(0)
        call("pp2_resident_tiling", self._h, C.byref(t), C.byref(r), C.byref(c))
        return t.value, r.value, c.value

    def model_download(self):
        n = self.cells
        T = np.empty((n, 9, 9), np.float32)
        L = np.empty((n, 16), np.float32)
        R = np.empty((n, 9), np.float32)
        Cc = np.empty((n, 9), np.float32)
        call("pp2_model_download", self._h, _f32(T), _f32(L), _f32(R), _f32(Cc))
        return T, L, R, Cc

    def model_upload(self, T=None, L=None, R=None, Cc=None):
        keep = []

        def p(a, shape):
            if a is None:
                return _NULLF
            a = np.ascontiguousarray(a, np.float32).reshape(shape)
            keep.append(a)
            return _f32(a)
        n = self.cells
        call("pp2_model_upload", self._h, p(T, (n, 9, 9)), p(L, (n, 16)),
             p(R, (n, 9)), p(Cc, (n, 9)))

    def model_save(self, directory: str):
        call("pp2_model_save", self._h, directory.encode())

    def model_load(self, directory: str):
        call("pp2_model_load", self._h, directory.encode())

    # ------------------------------------------------------------ belief
    def belief_set(self, b):
        b = np.ascontiguousarray(b, np.float32).reshape(self.cells)
        call("pp2_belief_set", self._h, _f32(b))

    def belief_get(self) -> np.ndarray:
        out = np.empty(self.cells, np.float32)
        call("pp2_belief_get", self._h, _f32(out))
        return out

    def belief_update(self, u: int, z: int):
        call("pp2_belief_update", self._h, int(u), int(z))

    def belief_get_raw(self):
        out = np.empty(self.cells, np.float32)
        m = C.c_float()
        call("pp2_belief_get_raw", self._h, _f32(out), C.byref(m))
        return out, m.value

    def belief_mass(self) -> float:
        m = C.c_float()
        call("pp2_belief_mass", self._h, C.byref(m))
        return m.value

    # ------------------------------------------------------------ MDP
    def mdp_reset(self):
        call("pp2_mdp_reset", self._h)

    def mdp_sweep(self, n: int = 1):
        call("pp2_mdp_sweep", self._h, int(n))

    def mdp_solve(self, max_sweeps: int = 0):
        s = C.c_int()
        nrm = C.c_double()
        call("pp2_mdp_solve", self._h, int(max_sweeps), C.byref(s), C.byref(nrm))
        return s.value, nrm.value

    def mdp_get(self):
        J = np.empty(self.cells, np.float32)
        A = np.empty(self.cells, np.uint8)
        call("pp2_mdp_get", self._h, _f32(J), _u8(A))
        return J, A

    # ------------------------------------------------------------ north star
    def loop_step(self, u: int, z: int):
        call("pp2_loop_step", self._h, int(u), int(z))

    def loop_run(self, us, zs):
        us = np.ascontiguousarray(us, np.uint8)
        zs = np.ascontiguousarray(zs, np.uint8)
        if us.shape != zs.shape:
            raise ValueError("us and zs must have the same length")
        call("pp2_loop_run", self._h, int(us.size), us.tobytes(), zs.tobytes())

    def loop_launcher(self, us, zs):
        """A zero-argument callable that runs pp2_loop_run on this trajectory:
        the arguments are converted once, here, so a timed call pays only the
        C-ABI call itself (what a compiled client pays)."""
        us = np.ascontiguousarray(us, np.uint8)
        zs = np.ascontiguousarray(zs, np.uint8)
        if us.shape != zs.shape:
            raise ValueError("us and zs must have the same length")
        lib = _lib.load()
        fn, h, n, ub, zb = lib.pp2_loop_run, self._h, int(us.size), us.tobytes(), zs.tobytes()

        def run():
            st = fn(h, n, ub, zb)
            if st != _lib.PP2_OK:
                msg = lib.pp2_last_error()
                raise _lib.Pp2Error(st, "pp2_loop_run", msg.decode() if msg else "")
        return run

    # ------------------------------------------------------------ FIB
    def fib_reset(self):
        call("pp2_fib_reset", self._h)

    def fib_sweep(self, n: int = 1):
        call("pp2_fib_sweep", self._h, int(n))

    def fib_solve(self, max_sweeps: int = 0):
        s = C.c_int()
        nrm = C.c_float()
        call("pp2_fib_solve", self._h, int(max_sweeps), C.byref(s), C.byref(nrm))
        return s.value, nrm.value

    def fib_get(self) -> np.ndarray:
        out = np.empty((self.cells, 9), np.float32)
        call("pp2_fib_get", self._h, _f32(out))
        return out

    def fib_set(self, alphas):
        a = np.ascontiguousarray(alphas, np.float32).reshape(self.cells, 9)
        call("pp2_fib_set", self._h, _f32(a))

    def fib_save(self, directory: str):
        call("pp2_fib_save", self._h, directory.encode())

    def fib_load(self, directory: str):
        call("pp2_fib_load", self._h, directory.encode())

    # ------------------------------------------------------------ PBVI
    def pbvi_belief_set(self, b0, set_size: int = 500, rand_seed: int = 1) -> int:
        """generateBeliefSet; returns the number of rand() draws it made."""
        b0 = np.ascontiguousarray(b0, np.float32).reshape(self.cells)
        n = C.c_uint64()
        call("pp2_pbvi_belief_set", self._h, _f32(b0), int(set_size), int(rand_seed),
             C.byref(n))
        return n.value

    def pbvi_set_beliefs(self, beliefs):
        B = np.ascontiguousarray(beliefs, np.float32).reshape(-1, self.cells)
        call("pp2_pbvi_set_beliefs", self._h, B.shape[0], _f32(B))

    def pbvi_info(self):
        s = C.c_uint32()
        h = C.c_int()
        call("pp2_pbvi_info", self._h, C.byref(s), C.byref(h))
        return s.value, bool(h.value)

    def pbvi_get_beliefs(self) -> np.ndarray:
        S, _ = self.pbvi_info()
        out = np.empty((S, self.cells), np.float32)
        call("pp2_pbvi_get_beliefs", self._h, _f32(out))
        return out

    def pbvi_backup(self, iterations: int = 0):
        call("pp2_pbvi_backup", self._h, int(iterations))

    def pbvi_solve(self, b0, set_size: int = 500, rand_seed: int = 1) -> int:
        """pointBasedValueIteration; returns the number of rand() draws."""
        b0 = np.ascontiguousarray(b0, np.float32).reshape(self.cells)
        n = C.c_uint64()
        call("pp2_pbvi_solve", self._h, _f32(b0), int(set_size), int(rand_seed), C.byref(n))
        return n.value

    def pbvi_get(self):
        S, _ = self.pbvi_info()
        al = np.empty((S, self.cells), np.float32)
        act = np.empty(S, np.uint8)
        call("pp2_pbvi_get", self._h, _f32(al), _u8(act))
        return al, act

    def pbvi_set(self, alphas, actions):
        al = np.ascontiguousarray(alphas, np.float32).reshape(-1, self.cells)
        act = np.ascontiguousarray(actions, np.uint8).reshape(al.shape[0])
        call("pp2_pbvi_set", self._h, al.shape[0], _f32(al), _u8(act))

    def pbvi_evaluate(self, beliefs):
        """evaluatePbviCpu over a batch: (values[n], actions[n])."""
        B = np.ascontiguousarray(beliefs, np.float32).reshape(-1, self.cells)
        v = np.empty(B.shape[0], np.float32)
        a = np.empty(B.shape[0], np.uint8)
        call("pp2_pbvi_evaluate", self._h, B.shape[0], _f32(B), _f32(v), _u8(a))
        return v, a

    def pbvi_save(self, directory: str):
        call("pp2_pbvi_save", self._h, directory.encode())

    def pbvi_load(self, directory: str, set_size: int = 500):
        call("pp2_pbvi_load", self._h, directory.encode(), int(set_size))

    # ------------------------------------------------------------ shards
    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.RCCL_ID_BYTES)()
        call("pp2_rccl_unique_id", buf)
        return bytes(buf)

    def shard_comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * _lib.RCCL_ID_BYTES).from_buffer_copy(uid)
        call("pp2_shard_comm_init", self._h, buf, int(nranks), int(rank))


def device_count() -> int:
    n = C.c_int()
    call("pp2_device_count", C.byref(n))
    return n.value


class ShardGroup:
    """Row shards of one grid driven from one process (pp2_shard_group_*):
    halo rows and the belief mass move by device copies between the shard
    contexts, which may live on one or several devices.

    ``bounds`` are the row boundaries, e.g. (0, 256, 512, ..., H)."""

    def __init__(self, grid: np.ndarray, goal, bounds, gamma: float = 0.95,
                 devices=None):
        bounds = [int(b) for b in bounds]
        n = len(bounds) - 1
        devices = list(devices) if devices is not None else [0] * n
        self.shards = [GridContext(grid, goal, gamma=gamma, device=devices[i],
                                   rows=(bounds[i], bounds[i + 1]))
                       for i in range(n)]
        arr = (C.c_void_p * n)(*[s.handle.value for s in self.shards])
        h = C.c_void_p()
        call("pp2_shard_group_create", C.byref(h), arr, n)
        self._h = h
        self.bounds = bounds

    def model_generate(self):
        for s in self.shards:
            s.model_generate()

    def belief_set(self, b):
        b = np.ascontiguousarray(b, np.float32).reshape(-1)
        for s in self.shards:
            s.belief_set(b[s.row_begin * s.width:s.row_end * s.width])

    def belief_get(self):
        return np.concatenate([s.belief_get() for s in self.shards])

    def mdp_reset(self):
        for s in self.shards:
            s.mdp_reset()
        self.synchronize()

    def mdp_get(self):
        parts = [s.mdp_get() for s in self.shards]
        return (np.concatenate([p[0] for p in parts]),
                np.concatenate([p[1] for p in parts]))

    def fib_get(self):
        return np.concatenate([s.fib_get() for s in self.shards])

    def fib_reset(self):
        for s in self.shards:
            s.fib_reset()
        self.synchronize()

    def set_halo_depth(self, k: int):
        """Loop steps per halo exchange (= halo rows exchanged), on every shard."""
        for s in self.shards:
            s.set_tuning(GridContext.TUNE_HALO_DEPTH, int(k))

    def loop_step(self, u, z):
        call("pp2_shard_group_loop_step", self._h, int(u), int(z))

    def loop_run(self, us, zs):
        us = np.ascontiguousarray(us, np.uint8)
        zs = np.ascontiguousarray(zs, np.uint8)
        if us.shape != zs.shape:
            raise ValueError("us and zs must have the same length")
        call("pp2_shard_group_loop_run", self._h, int(us.size), us.tobytes(), zs.tobytes())

    def set_tuning(self, key: int, value: int):
        for s in self.shards:
            s.set_tuning(key, value)

    def loop_steps_per_launch(self):
        return [s.loop_steps_per_launch() for s in self.shards]

    def belief_update(self, u, z):
        call("pp2_shard_group_belief_update", self._h, int(u), int(z))

    def mdp_sweep(self, n=1):
        call("pp2_shard_group_mdp_sweep", self._h, int(n))

    def mdp_solve(self, max_sweeps=0):
        s = C.c_int()
        nrm = C.c_double()
        call("pp2_shard_group_mdp_solve", self._h, int(max_sweeps), C.byref(s),
             C.byref(nrm))
        return s.value, nrm.value

    def fib_sweep(self, n=1):
        call("pp2_shard_group_fib_sweep", self._h, int(n))

    def synchronize(self):
        call("pp2_shard_group_synchronize", self._h)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().pp2_shard_group_destroy(self._h)
            self._h = None
        for s in getattr(self, "shards", []):
            s.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
