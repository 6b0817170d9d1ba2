// Row-gather engine shared by the bf16 gather kernels (snd_fast_enc.hip) and the
// fused encoder heads (snd_head.hip): 8 lanes per CSR row, lane `sub` owns the
// 16-byte chunks sub, sub + 8 of a neighbour row.
#pragma once
#include "snd_common.hpp"

namespace snd {

constexpr int kLpr = 8;   // lanes per row (aligned DPP half-rows)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 gbf16x2 __attribute__((ext_vector_type(2)));

// a . b over one 8-column chunk of packed bf16 pairs (the per-edge logit z_i . z_j of the
// bf16 edge kernels): four v_dot2_f32_bf16 on the packed words, no widening
// (the words go through plain arrays first: bit-casting the ext_vector elements in place
// made hipcc feed the first word to all four dot2 instructions)
__device__ __forceinline__ float dot8_bf16(const u32x4& a, const u32x4& b, float acc) {
  const unsigned wa[4] = {a.x, a.y, a.z, a.w}, wb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int p = 0; p < 4; ++p)
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gbf16x2, wa[p]), __builtin_bit_cast(gbf16x2, wb[p]),
                                          acc, false);
  return acc;
}

// Lane u of each aligned 8-lane group to all 8 lanes (ds_swizzle bit mode:
// and-mask 0x18 keeps the group, or-mask u selects the lane; no LDS access).
template <int U>
__device__ __forceinline__ int bcast8(int v) {
  return __builtin_amdgcn_ds_swizzle(v, 0x18 | (U << 5));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// Per round the row's next 16 neighbour ids are loaded one or two per lane and
// broadcast inside the 8-lane group, and all 16 neighbour chunks are requested
// before any is consumed: a row of degree <= 16 costs one rowptr -> colidx ->
// gather latency chain.  The gathers are buffer loads with a 32-bit offset (one
// mad per neighbour, no 64-bit address arithmetic); a missing neighbour (past the
// row end, id -1) wraps its offset past the descriptor's range, so the hardware
// returns zeros with no select.  fn(u, v, valid) consumes neighbour u of the round
// in order; cross-lane work inside fn stays uniform over the row's 8 lanes.
template <int NQ, typename Fn>
__device__ __forceinline__ void gather_rows16(const int* colidx, int s, int e, __amdgpu_buffer_rsrc_t rs,
                                              unsigned row_bytes, int sub, Fn&& fn) {
  for (int k0 = s; k0 < e; k0 += 16) {
    const int id0 = k0 + sub < e ? colidx[k0 + sub] : -1;
    const int id1 = k0 + 8 + sub < e ? colidx[k0 + 8 + sub] : -1;
    int c[16];
    c[0] = bcast8<0>(id0); c[1] = bcast8<1>(id0); c[2] = bcast8<2>(id0); c[3] = bcast8<3>(id0);
    c[4] = bcast8<4>(id0); c[5] = bcast8<5>(id0); c[6] = bcast8<6>(id0); c[7] = bcast8<7>(id0);
    c[8] = bcast8<0>(id1); c[9] = bcast8<1>(id1); c[10] = bcast8<2>(id1); c[11] = bcast8<3>(id1);
    c[12] = bcast8<4>(id1); c[13] = bcast8<5>(id1); c[14] = bcast8<6>(id1); c[15] = bcast8<7>(id1);
    u32x4 v[16][NQ];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const unsigned off = (unsigned)c[u] * row_bytes + 16u * sub;   // id -1: out of range -> 0
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[u][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 128u * q, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);   // all 16 requests issue before the first is consumed
    const int nv = e - k0;               // neighbours of this round (the ids die with the loads)
#pragma unroll
    for (int u = 0; u < 16; ++u) fn(u, v[u], u < nv);
  }
}

// acc[0..7] += the 8 bf16 of a packed 16-byte chunk (exact widening + fp32 add)
// fp32 sums without widening: v_dot2_f32_bf16 with (1, 0) / (0, 1) adds the low / high
// bf16 of a word to an fp32 accumulator (x * 1 and y * 0 are exact: one rounding, the
// plain add's result), one instruction per element instead of a shift / mask and an add
// (the window SpMM's acc8_dot; round 5: every gather sum)
__device__ __forceinline__ void acc8v(float (&a)[8], const u32x4& v) {
  // (1, 0) and (0, 1) through SGPRs: hipcc encodes the bf16 pair (1, 0) as the inline
  // constant 1.0, which the hardware reads as the fp32 word 0x3F800000 = (0, 1)
  unsigned lo1u, hi1u;
  asm volatile("s_mov_b32 %0, 0x3f80" : "=s"(lo1u));
  asm volatile("s_mov_b32 %0, 0x3f800000" : "=s"(hi1u));
  const gbf16x2 lo1 = __builtin_bit_cast(gbf16x2, lo1u);
  const gbf16x2 hi1 = __builtin_bit_cast(gbf16x2, hi1u);
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const gbf16x2 x = __builtin_bit_cast(gbf16x2, w[p]);
    a[2 * p] = __builtin_amdgcn_fdot2_f32_bf16(x, lo1, a[2 * p], false);
    a[2 * p + 1] = __builtin_amdgcn_fdot2_f32_bf16(x, hi1, a[2 * p + 1], false);
  }
}

// the 8 bf16 of a packed chunk, widened
__device__ __forceinline__ void widen8(float (&a)[8], const u32x4& v) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const unsigned w = v[p];
    a[2 * p] = __uint_as_float(w << 16);
    a[2 * p + 1] = __uint_as_float(w & 0xFFFF0000u);
  }
}

__device__ __forceinline__ uint4 to_bf16x8(const float (&v)[8]) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
  return __builtin_bit_cast(uint4, o);
}

}  // namespace snd
