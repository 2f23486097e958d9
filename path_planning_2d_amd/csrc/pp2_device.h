// pp2_device.h -- device-side helpers shared by the gfx950 kernel files
// (pp2_kernels.hip, pp2_coded.hip): vector loads/stores over the SoA planes
// and the deterministic (fixed-association) wave/block reductions.
#pragma once
#include <float.h>
#include <stdint.h>

#include "pp2_internal.h"

namespace pp2 {

typedef float f4a __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2a __attribute__((ext_vector_type(2)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));

constexpr int kBlock = 256;

template <int N, bool ALIGNED>
__device__ __forceinline__ void ldv(const float* __restrict__ p, float (&v)[N]) {
  if constexpr (N == 4) {
    if constexpr (ALIGNED) {
      const f4a t = *reinterpret_cast<const f4a*>(p);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
      const f4u t = *reinterpret_cast<const f4u*>(p);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    }
  } else if constexpr (N == 2) {
    if constexpr (ALIGNED) {
      const f2a t = *reinterpret_cast<const f2a*>(p);
      v[0] = t[0]; v[1] = t[1];
    } else {
      const f2u t = *reinterpret_cast<const f2u*>(p);
      v[0] = t[0]; v[1] = t[1];
    }
  } else {
    v[0] = *p;
  }
}

// Non-temporal variant for streams read exactly once per launch (T, C).
template <int N, bool NT>
__device__ __forceinline__ void ldv_stream(const float* __restrict__ p, float (&v)[N]) {
  if constexpr (NT && N == 4) {
    const f4a t = __builtin_nontemporal_load(reinterpret_cast<const f4a*>(p));
    v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
  } else {
    ldv<N, true>(p, v);
  }
}

template <int N>
__device__ __forceinline__ void stv(float* __restrict__ p, const float (&v)[N]) {
  if constexpr (N == 4) {
    f4a t = {v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f4a*>(p) = t;
  } else if constexpr (N == 2) {
    f2a t = {v[0], v[1]};
    *reinterpret_cast<f2a*>(p) = t;
  } else {
    *p = v[0];
  }
}

// ---- deterministic reductions (fixed association order) --------------------
// xor-butterfly: partners always add the same two operands, so every lane of
// the wave ends with the bit-identical total.  Stages xor 32, 16, 8, 4, 2, 1
// (the association of a __shfl_xor loop from 32 down), without the LDS
// crossbar: xor 32 / 16 by v_permlane32_swap / v_permlane16_swap (a pair of
// half-swapped copies whose sum is v_i + v_{i^m} in every lane), xor 8 as
// row_mirror then row_half_mirror (i ^ 15 ^ 7), xor 4 as row_half_mirror then
// quad_perm [3,2,1,0] (i ^ 7 ^ 3), xor 2 / 1 as quad_perm -- 10 VALU
// instructions against 6 ds_bpermute_b32 round trips and 6 adds.
template <typename OP>
__device__ __forceinline__ float wave_butterfly(float v, OP op) {
  const uint32_t u = __float_as_uint(v);
  const auto h32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  v = op(__uint_as_float(h32[0]), __uint_as_float(h32[1]));
  const uint32_t u16 = __float_as_uint(v);
  const auto h16 = __builtin_amdgcn_permlane16_swap(u16, u16, false, false);
  v = op(__uint_as_float(h16[0]), __uint_as_float(h16[1]));
  auto dpp = [](float x, int ctrl) -> float {
    switch (ctrl) {  // the DPP control must be a constant
      case 0x140: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false));
      case 0x141: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false));
      case 0x1b: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x1b, 0xf, 0xf, false));
      case 0x4e: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4e, 0xf, 0xf, false));
      default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xb1, 0xf, 0xf, false));
    }
  };
  v = op(v, dpp(dpp(v, 0x140), 0x141));  // xor 8
  v = op(v, dpp(dpp(v, 0x141), 0x1b));   // xor 4
  v = op(v, dpp(v, 0x4e));               // xor 2
  v = op(v, dpp(v, 0xb1));               // xor 1
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_butterfly(v, [](float a, float b) { return a + b; });
}

// 128 per-lane values summed across the wave as a reduce-scatter: each
// butterfly stage (xor 32, 16, 8, 4, 2, 1) halves the values a lane carries
// -- it keeps the half its xor-group owns and adds the partner's copy of it --
// so the wave exchanges 126 values instead of 6 x 128, and lane l ends with
// the totals of values 2l and 2l + 1 in out[0], out[1].  Every total is
// v_i + v_{i^m} stage by stage from 32 down, i.e. wave_sum's association,
// bit for bit.  xor 32 / 16: one v_permlane32/16_swap of the kept pair (x =
// low half, y = high half) leaves x' + y' = the lane's own sum in every lane;
// xor 8 .. 1: send the half the partner keeps by DPP and add it to the kept
// half.
__device__ __forceinline__ void wave_sum_scatter128(const float (&lo)[64], const float (&hi)[64],
                                                   float (&out)[2]) {
  const int lane = threadIdx.x & 63;
  float v1[64], v2[32], v3[16], v4[8], v5[4], v6[2];
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo[j]), __float_as_uint(hi[j]),
                                                    false, false);
    v1[j] = __uint_as_float(h[0]) + __uint_as_float(h[1]);
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const auto h = __builtin_amdgcn_permlane16_swap(__float_as_uint(v1[j]),
                                                    __float_as_uint(v1[32 + j]), false, false);
    v2[j] = __uint_as_float(h[0]) + __uint_as_float(h[1]);
  }
  auto x8 = [](float x) {
    const float m = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false));
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x141, 0xf, 0xf, false));
  };
  auto x4 = [](float x) {
    const float m = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false));
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x1b, 0xf, 0xf, false));
  };
  auto x2 = [](float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4e, 0xf, 0xf, false));
  };
  auto x1 = [](float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xb1, 0xf, 0xf, false));
  };
  // keep the half this lane's xor-group owns, add the partner's copy of it
#define PP2_HALVE(SRC, DST, N, D, XF)                                  \
  {                                                                    \
    const bool h_ = lane & (D);                                        \
    _Pragma("unroll") for (int j = 0; j < (N); ++j) {                  \
      const float keep = h_ ? SRC[(N) + j] : SRC[j];                   \
      const float send = h_ ? SRC[j] : SRC[(N) + j];                   \
      DST[j] = keep + XF(send);                                        \
    }                                                                  \
  }
  PP2_HALVE(v2, v3, 16, 8, x8)
  PP2_HALVE(v3, v4, 8, 4, x4)
  PP2_HALVE(v4, v5, 4, 2, x2)
  PP2_HALVE(v5, v6, 2, 1, x1)
#undef PP2_HALVE
  out[0] = v6[0];
  out[1] = v6[1];
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_butterfly(v, [](float a, float b) { return fmaxf(a, b); });
}

// Sum over a 256-thread block; result valid in thread 0.
__device__ __forceinline__ float block_sum(float v, float* lds4) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds4[w] = v;
  __syncthreads();
  float r = 0.0f;
  if (threadIdx.x == 0) r = ((lds4[0] + lds4[1]) + lds4[2]) + lds4[3];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* lds4) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds4[w] = v;
  __syncthreads();
  float r = 0.0f;
  if (threadIdx.x == 0) r = fmaxf(fmaxf(lds4[0], lds4[1]), fmaxf(lds4[2], lds4[3]));
  return r;
}

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4u __attribute__((ext_vector_type(4), aligned(2)));

// Belief mass partials are written per wave (4 per 256-cell-thread block,
// wave order), so no kernel needs a block barrier after its stores.  The
// consumer folds each block's four as ((w0 + w1) + w2) + w3 -- block_sum's
// association -- then sums blocks lane-strided and xor-butterflies: the same
// tree in k_sum_finalize and in every fused step, so a mass finalised
// separately and one reduced inside a later kernel are bit-identical.
// n = number of wave partials (a multiple of 4, p 16-B aligned).
// The loads go out 8 quads per lane at a time, ahead of the (sequential,
// in-order) adds: one memory round trip per 2048 partials, not per 256.
__device__ __forceinline__ float wave_reduce_partials(const float* __restrict__ p, int n) {
  const int lane = threadIdx.x & 63;
  const int nq = n >> 2;
  const f4a* q = reinterpret_cast<const f4a*>(p);
  float s = 0.0f;
  for (int base = lane; base < nq; base += 64 * 8) {
    f4a w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + 64 * j;
      w[j] = q[i < nq ? i : base];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (base + 64 * j < nq) s += ((w[j][0] + w[j][1]) + w[j][2]) + w[j][3];
  }
  return wave_sum(s);
}

// Per-wave partial of a 256-thread block (or of one 256-thread quarter of a
// larger workgroup): lane 0 of wave w of the quarter writes p[4*blk + w].
__device__ __forceinline__ void write_wave_partial(float v, float* __restrict__ p, long long blk) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) p[4 * blk + ((threadIdx.x >> 6) & 3)] = v;
}

__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n / 8, r = n % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// codes of rows y-1, y, y+1 at x0-1 .. x0+4 (dword-aligned loads only)
struct CodeWin {
  uint32_t c[3][6];
};

__device__ __forceinline__ void load_codes(const uint16_t* __restrict__ code, int wp, int y,
                                           int x0, CodeWin& w) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const uint16_t* cp = code + (long long)(y + r - 1) * wp + x0;
    const uint2 m = *reinterpret_cast<const uint2*>(cp);
    const uint32_t lw = *reinterpret_cast<const uint32_t*>(cp - 2);
    const uint32_t rw = *reinterpret_cast<const uint32_t*>(cp + 4);
    w.c[r][0] = lw >> 16;
    w.c[r][1] = m.x & 0xffffu;
    w.c[r][2] = m.x >> 16;
    w.c[r][3] = m.y & 0xffffu;
    w.c[r][4] = m.y >> 16;
    w.c[r][5] = rw & 0xffffu;
  }
}

}  // namespace pp2
