"""Synthetic planner inputs (DESIGN.md "Synthetic inputs").

* grid: i.i.d. obstacles from splitmix64(seed), occupied iff
  ``(x >> 11) * 2**-53 < p_occ`` (row-major, one draw per cell);
* goal: first free cell scanning left from (W-6, H-6), then upward;
* initial belief: uniform over free cells (src/pomdp/path_planning_2d.cu:99-107);
* (u, z) trajectory: splitmix64(seed) simulation of the true robot -- start at
  the free cell nearest the centre; u ~ U{0..8}; s' ~ T[s][u][:]; z ~ L[s'][:].

Pure numpy host code for generating benchmark/test inputs; the planner math
itself runs on the GPU.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# base motion kernels, src/pomdp/model_generation_cuda.cu:175-211
_BASE = np.zeros((9, 9), np.float32)
for _u, _entries in enumerate([
        {0: .7, 1: .1, 3: .1, 4: .1}, {0: .1, 1: .7, 2: .1, 4: .1},
        {1: .1, 2: .7, 4: .1, 5: .1}, {0: .1, 3: .7, 4: .1, 6: .1},
        {4: 1.0}, {2: .1, 4: .1, 5: .7, 8: .1}, {3: .1, 4: .1, 6: .7, 7: .1},
        {4: .1, 6: .1, 7: .7, 8: .1}, {4: .1, 5: .1, 7: .1, 8: .7}]):
    for _i, _v in _entries.items():
        _BASE[_u, _i] = np.float32(_v)


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


class SplitMix64:
    def __init__(self, seed: int):
        self.state = np.uint64(seed)

    def next(self) -> np.uint64:
        with np.errstate(over="ignore"):
            self.state = self.state + _GOLDEN
            return _mix(np.uint64(self.state))

    def u01(self) -> float:
        return float(int(self.next()) >> 11) * 2.0 ** -53

    def u01_array(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            k = np.arange(1, n + 1, dtype=np.uint64)
            z = _mix(self.state + k * _GOLDEN)
            self.state = self.state + np.uint64(n) * _GOLDEN
        return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def synth_grid(height: int, width: int, seed: int | None = None,
               p_occ: float = 0.20) -> np.ndarray:
    rng = SplitMix64(height if seed is None else seed)
    u = rng.u01_array(height * width)
    return (u < p_occ).astype(np.uint8).reshape(height, width)


def synth_goal(grid: np.ndarray):
    H, W = grid.shape
    x0 = W - 6 if W >= 6 else W - 1
    y0 = H - 6 if H >= 6 else H - 1
    for y in range(y0, -1, -1):
        free = np.nonzero(grid[y, :x0 + 1] == 0)[0]
        if free.size:
            return int(free[-1]), int(y)
    raise ValueError("no free cell for the goal")


def uniform_belief(grid: np.ndarray) -> np.ndarray:
    """initial_belief[i] = (1 - map[i]) / sum (src/pomdp/path_planning_2d.cu:101-107).
    The reference's sequential fp32 sum of 0/1 values is exact below 2**24
    cells, so the free-cell count stands in for it bit-for-bit."""
    free = (1 - grid.reshape(-1)).astype(np.float32)
    n = int(free.sum(dtype=np.int64))
    if free.size >= 1 << 24:
        raise ValueError("grid too large for an exact fp32 free-cell count")
    return (free / np.float32(n)).astype(np.float32)


def _local_map(grid, x, y):
    H, W = grid.shape
    lm = np.ones(9, np.uint8)
    for i in range(9):
        nx, ny = x + i % 3 - 1, y + i // 3 - 1
        if 0 <= nx < W and 0 <= ny < H:
            lm[i] = grid[ny, nx]
    return lm


def cell_transition(grid, x, y, u) -> np.ndarray:
    """T[x][u][:] (src/pomdp/model_generation_cuda.cu:161-236)."""
    lm = _local_map(grid, x, y)
    tp = _BASE[u].copy()
    for i in range(9):
        if lm[i] == 1 and i != 4:
            tp[4] = np.float32(tp[4] + tp[i])
            tp[i] = np.float32(0.0)
    if lm[4] == 1:
        tp[:] = 0
        tp[4] = 1
    return tp


def cell_likelihood(grid, x, y) -> np.ndarray:
    """L[x][:] (src/pomdp/model_generation_cuda.cu:238-264)."""
    lm = _local_map(grid, x, y)
    m = (lm[1], lm[3], lm[5], lm[7])
    hi, lo = np.float32(0.98), np.float32(0.02)
    out = np.empty(16, np.float32)
    for i in range(16):
        ls = [hi if ((i >> k) & 1) == m[k] else lo for k in range(4)]
        out[i] = np.float32(np.float32(np.float32(ls[0] * ls[1]) * ls[2]) * ls[3])
    return out


def start_cell(grid):
    H, W = grid.shape
    ys, xs = np.nonzero(grid == 0)
    if ys.size == 0:
        raise ValueError("no free cell")
    d = (xs.astype(np.int64) - W // 2) ** 2 + (ys.astype(np.int64) - H // 2) ** 2
    k = int(np.argmin(d))  # first minimum in row-major order
    return int(xs[k]), int(ys[k])


def synth_trajectory(grid: np.ndarray, n: int, seed: int = 42):
    """Returns (us, zs, states) -- uint8, uint8, int32 (true cell after step)."""
    H, W = grid.shape
    x, y = start_cell(grid)
    rng = SplitMix64(seed)
    us = np.empty(n, np.uint8)
    zs = np.empty(n, np.uint8)
    st = np.empty(n, np.int32)
    for k in range(n):
        u = min(int(rng.u01() * 9.0), 8)
        tp = cell_transition(grid, x, y, u)
        r, c, j = rng.u01(), 0.0, 4
        for i in range(9):
            c += float(tp[i])
            if tp[i] > 0 and r < c:
                j = i
                break
        x += j % 3 - 1
        y += j // 3 - 1
        lk = cell_likelihood(grid, x, y)
        r, c, z = rng.u01(), 0.0, 15
        for i in range(16):
            c += float(lk[i])
            if r < c:
                z = i
                break
        us[k], zs[k], st[k] = u, z, y * W + x
    return us, zs, st


def closed_loop(grid: np.ndarray, b0: np.ndarray, step_fn, max_steps: int,
                budget_s: float = 1e9, seed: int = 99, min_steps: int = 0):
    """Closed-loop plan steps, as the reference node runs against the dummy
    simulator: step_fn(a, z, belief) is one beliefCallback
    (src/pomdp/path_planning_2d.cu:199-241) returning (action, value); its
    action moves a simulated robot (s' ~ T[s][a]) whose observation
    (z ~ L[s']) is the next message.  The first call gets b0, later calls
    None.  splitmix64(seed) draws the motion and the observation, so two
    planners that choose the same actions see the same messages.  The loop
    stops after max_steps, or once budget_s has passed and at least
    min_steps ran.

    Returns (ms, actions, values): the wall time of each step, the chosen
    actions (uint8) and values (float32)."""
    import time
    rng = SplitMix64(seed)
    x, y = start_cell(grid)
    times, acts, vals = [], [], []
    a, z, first = 0, 0, True
    t_start = time.perf_counter()
    for _ in range(max_steps):
        t = time.perf_counter()
        a, v = step_fn(a, z, b0 if first else None)
        times.append(time.perf_counter() - t)
        acts.append(a)
        vals.append(v)
        first = False
        tp = cell_transition(grid, x, y, a)
        r, c, j = rng.u01(), 0.0, 4
        for i in range(9):
            c += float(tp[i])
            if tp[i] > 0 and r < c:
                j = i
                break
        x += j % 3 - 1
        y += j // 3 - 1
        lk = cell_likelihood(grid, x, y)
        r, c, z = rng.u01(), 0.0, 15
        for i in range(16):
            c += float(lk[i])
            if r < c:
                z = i
                break
        if len(times) >= min_steps and time.perf_counter() - t_start > budget_s:
            break
    return (np.array(times) * 1e3, np.array(acts, np.uint8),
            np.array(vals, np.float32))


def action_parity(acts_a, vals_a, acts_b, vals_b) -> dict:
    """Plan-step parity of two closed loops over their common steps: the
    actions equal and the values equal as fp32 bit patterns, step by step
    (the loops share their messages while the actions agree, so the first
    mismatch ends the comparison's meaning)."""
    n = int(min(len(acts_a), len(acts_b)))
    a_ok = np.asarray(acts_a[:n]) == np.asarray(acts_b[:n])
    v_ok = (np.asarray(vals_a[:n], np.float32).view(np.uint32)
            == np.asarray(vals_b[:n], np.float32).view(np.uint32))
    bad = np.nonzero(~(a_ok & v_ok))[0]
    return {"steps_compared": n,
            "actions_equal": bool(a_ok.all()),
            "values_bit_exact": bool(v_ok.all()),
            "first_mismatch": int(bad[0]) if bad.size else None}


def rollout_trajectories(grid: np.ndarray, belief: np.ndarray, copies: int, depth: int,
                         seed: int = 5):
    """(us, zs) of shape [depth, copies] for batched rollouts: each copy draws a
    true start cell from ``belief`` and simulates u ~ U{0..8}, s' ~ T, z ~ L,
    so every observation has positive likelihood under its copy's belief."""
    H, W = grid.shape
    rng = SplitMix64(seed)
    cdf = np.cumsum(belief.astype(np.float64))
    us = np.empty((depth, copies), np.uint8)
    zs = np.empty((depth, copies), np.uint8)
    for c in range(copies):
        cell = int(min(np.searchsorted(cdf, rng.u01() * cdf[-1], side="right"), H * W - 1))
        while belief[cell] <= 0:
            cell -= 1
        x, y = cell % W, cell // W
        for k in range(depth):
            u = min(int(rng.u01() * 9.0), 8)
            tp = cell_transition(grid, x, y, u)
            r, acc, j = rng.u01(), 0.0, 4
            for i in range(9):
                acc += float(tp[i])
                if tp[i] > 0 and r < acc:
                    j = i
                    break
            x += j % 3 - 1
            y += j // 3 - 1
            lk = cell_likelihood(grid, x, y)
            r, acc, z = rng.u01(), 0.0, 15
            for i in range(16):
                acc += float(lk[i])
                if r < acc:
                    z = i
                    break
            us[k, c], zs[k, c] = u, z
    return us, zs
