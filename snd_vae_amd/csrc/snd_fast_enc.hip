// bf16 fast path, encoder side (model.py:104-115, layers.py:115-125, model.py:153-161).
//
// GraphConvolution 0 is evaluated as (A X) W0 instead of A (X W0): the same
// product, but the SpMM gathers the 3-wide node features (12 B per
// neighbour) instead of 64-wide projected rows, and its backward needs no
// SpMM at all: dW0 = X^T A dP0 = (A X)^T dP0 (A symmetric).  gcn0_kernel
// computes AX, recomputes P0 = AX W0 in registers, applies lrelu -> frozen
// BN and writes H1 = [B0 | X] once (bf16, the next GEMM's operand).
//
// spmm_bf16_kernel gathers bf16 neighbour rows (one 128-byte line per
// neighbour for width 64), accumulates in fp32 and fuses the
// GraphConvolution 1 epilogue (lrelu -> BN -> concat X -> encoder_g BN).
#include "snd_fast.hpp"
#include "snd_gather.hpp"
#include "snd_pack.hpp"

#include <algorithm>

namespace snd {
namespace {

constexpr int NT = 256;
constexpr int LPR = kLpr;          // lanes per row (aligned DPP half-rows)
constexpr int RPB = NT / LPR;      // rows per block

// Row processed by this lane's 8-lane group: slot rb*RPB + threadIdx/LPR of the
// optional locality order (a per-graph reverse Cuthill-McKee permutation made at
// ingest: consecutive slots are graph neighbours, so a block's gathers share
// rows in L1), else the slot itself.  Results do not depend on the order.
__device__ __forceinline__ int row_of(const int* order, int rb, int R) {
  const int slot = rb * RPB + threadIdx.x / LPR;
  return (order && slot < R) ? order[slot] : slot;
}

// XCD-aware row-block order: blocks b and b + 8 share an XCD (and its L2), so
// row blocks of graph g go to block group g % 8 -- a graph's gathered rows
// (<= 1 MB) then stay in one L2.  nbg = row blocks per graph (0: identity).
__device__ __forceinline__ int xcd_rowblock(int b, int nbg) {
  if (nbg <= 0) return b;
  const int x = b & 7, s = b >> 3;
  const int gi = s / nbg, lb = s - gi * nbg;
  return (x + 8 * gi) * nbg + lb;
}

// ---------------------------------------------------------------- GCN layer 0
__global__ void __launch_bounds__(NT) gcn0_kernel(Gcn0Args a) {
  const int nrb = (a.R + RPB - 1) / RPB;
  if ((int)blockIdx.x >= nrb) {   // the weight images (pack_kernel's work, bit for bit)
    const int pb = blockIdx.x - nrb;
    int s = 0;
    while (s + 1 < a.npack && pb >= a.pack_blk[s + 1]) ++s;
    s = __builtin_amdgcn_readfirstlane(s);
    const PackDesc& d = a.pack[s];
    const int i = (pb - a.pack_blk[s]) * NT + threadIdx.x;
    if (i < pack_chunks(d)) pack_chunk(d, i);
    return;
  }
  __shared__ float sp[6][128];     // W0 rows (f <= 4), gamma0 * c, beta0
  for (int i = threadIdx.x; i < a.h0; i += NT) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sp[q][i] = q < a.f ? a.w0[q * a.h0 + i] : 0.f;
    sp[4][i] = a.g0[i] * kBnC;
    sp[5][i] = a.b0[i];
  }
  __syncthreads();
  const int sub = threadIdx.x & (LPR - 1);
  const int r = row_of(a.row_order, xcd_rowblock(blockIdx.x, a.xcd_nbg), a.R);
  const bool rv = r < a.R;
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
  if (rv) {
    const int s = a.rowptr[r], e = a.rowptr[r + 1];
    int k = s + sub;
    for (; k + LPR < e; k += 2 * LPR) {          // two neighbours in flight per lane
      const int c0 = a.colidx[k], c1 = a.colidx[k + LPR];
      float v0[4], v1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v0[j] = j < a.f ? a.x[(long long)c0 * a.ldx + j] : 0.f;
        v1[j] = j < a.f ? a.x[(long long)c1 * a.ldx + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[j] += v0[j] + v1[j];
    }
    if (k < e) {
      const int c0 = a.colidx[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[j] += j < a.f ? a.x[(long long)c0 * a.ldx + j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) ax[j] = row8_sum(ax[j]);
  if (!rv) return;
  // P0 = AX W0 -> lrelu -> BN0 -> H1[:, :h0]   (8 columns per lane per chunk)
  for (int c8 = sub; 8 * c8 < a.h0; c8 += LPR) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * c8 + j;
      float p = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) p += ax[q] * sp[q][col];
      o[j] = lrelu(p) * sp[4][col] + sp[5][col];
    }
    *reinterpret_cast<uint4*>(a.h1 + (long long)r * a.ldh1 + 8 * c8) = to_bf16x8(o);
  }
  if (sub == 0) {
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = j < a.f ? a.x[(long long)r * a.ldx + j] : 0.f;
    *reinterpret_cast<uint4*>(a.h1 + (long long)r * a.ldh1 + a.h0) = to_bf16x8(xv);   // concat X
    *reinterpret_cast<float4*>(a.ax + (long long)r * 4) = make_float4(ax[0], ax[1], ax[2], ax[3]);
    const float axp[8] = {ax[0], ax[1], ax[2], ax[3], 0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<uint4*>(a.axb + (long long)r * 8) = to_bf16x8(axp);
  }
}

// ---------------------------------------------------------------- bf16 SpMM
// Epilogue of a finished row (acc = A[r,:] @ h in fp32): plain bf16 store, or the
// GraphConvolution 1 epilogue (preact fp32, lrelu -> BN1 -> concat X -> encoder_g BN).
template <int EPI, int NQ>
__device__ __forceinline__ void spmm_row_epilogue(const SpmmBfArgs& a, int r, int sub,
                                                  const float (&acc)[NQ][8]) {
  const int nch = a.width >> 3;    // 8-column chunks: lane sub owns chunks sub, sub + 8
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (sub + 8 * q >= nch) continue;
    const int col = 64 * q + 8 * sub;
    if constexpr (EPI == SND_SPMM_PLAIN) {
      *reinterpret_cast<uint4*>(a.out + (long long)r * a.ldo + col) = to_bf16x8(acc[q]);
    } else {
      float* pp = a.pre + (long long)r * a.ldp + col;
      *reinterpret_cast<float4*>(pp) = make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
      *reinterpret_cast<float4*>(pp + 4) = make_float4(acc[q][4], acc[q][5], acc[q][6], acc[q][7]);
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = col + j;
        const float b1 = lrelu(acc[q][j]) * (a.g1[c] * kBnC) + a.b1[c];    // H2[:, :h1]
        g[j] = b1 * (a.ge[c] * kBnC) + a.be[c];                             // encoder_g BN
      }
      *reinterpret_cast<uint4*>(a.g + (long long)r * a.ldg + col) = to_bf16x8(g);
    }
  }
  if constexpr (EPI == SND_SPMM_GCN) {
    if (sub == 0) {   // concat X (model.py:109) -> encoder_g BN on those columns
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = a.width + j;
        g[j] = j < a.f ? a.x[(long long)r * a.ldx + j] * (a.ge[c] * kBnC) + a.be[c] : 0.f;
      }
      *reinterpret_cast<uint4*>(a.g + (long long)r * a.ldg + a.width) = to_bf16x8(g);
    }
  }
}

template <int NQ>
__device__ __forceinline__ void zero_acc(float (&acc)[NQ][8]) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
}

template <int EPI, int NQ>
__global__ void __launch_bounds__(NT) spmm_bf16_kernel(SpmmBfArgs a) {
  const int sub = threadIdx.x & (LPR - 1);
  const int r = row_of(a.row_order, xcd_rowblock(blockIdx.x, a.xcd_nbg), a.R);
  if (r >= a.R) return;            // whole 8-lane row groups leave together
  float acc[NQ][8];
  zero_acc(acc);
  // chunks past the width read the next row's bytes (or zeros past the end): never stored
  const __amdgpu_buffer_rsrc_t rs = rows_rsrc(a.h, (long long)a.R * a.ldh * 2);
  gather_rows16<NQ>(a.colidx, a.rowptr[r], a.rowptr[r + 1], rs, 2u * a.ldh, sub,
                    [&](int, const u32x4 (&v)[NQ], bool) {
#pragma unroll
                      for (int q = 0; q < NQ; ++q) acc8v(acc[q], v[q]);
                    });
  spmm_row_epilogue<EPI, NQ>(a, r, sub, acc);
}

// ---------------------------------------------------------------- bf16 SpMM over row tiles
// Persistent, software-pipelined SpMM over the row tiles of snd_row_tiles_t.
//  * A tile's distinct neighbour rows (its set; ascending ids, so mostly consecutive
//    128-byte lines) are read once from HBM/L2 and widened to fp32 in LDS, plus one
//    zero row at index ustride.
//  * Every row's 8-lane group walks its neighbours in colidx order, 16 per round
//    (local ids broadcast inside the group), LDS reads in flight, packed fp32 adds;
//    a round's trip count is the wavefront's longest row (rows sorted by degree in
//    the tile keep that close to each row's own), shorter rows read the zero row
//    (exact +0 adds).  Same fp32 sums in the same order as spmm_bf16_kernel:
//    bitwise-equal output.
//  * Each workgroup walks a run of tiles (one graph's tiles stay on one XCD).  While
//    it sums tile i from LDS, tile i+1's rows and first local ids are in flight into
//    registers and tile i+2's row metadata and set ids are read: every dependent
//    load chain (set ids -> rows, row pointers -> local ids) spans one tile of work.
// Bank-conflict-free reads: ds_read_b128 serves a wave in 16-lane groups holding
// four 4-lane pieces of four different rows ({0-3,12-15,20-23,24-27} ...); the
// piece of 8-lane group g, half h reads row quarter (2g + h + 2 r) mod 4 in read r,
// so the four pieces of every 16-lane group hit four distinct bank quarters for any
// four rows (fp32 rows are 256 B = 64 banks: the quarter is fixed by the column).
constexpr int TNT = 512;                   // 64 row groups of 8 lanes
constexpr int TG = TNT / LPR;
constexpr int TILE_CAP = 319;              // largest set: 320 fp32 image rows with the zero row
constexpr int TRPG = 2;                    // rows per 8-lane group (tile_rows <= 128)
constexpr int TPRE = 4;                    // local ids prefetched per lane and row (32 per row)
// LDS image bytes: 80 KB for 64-wide rows (two workgroups per CU), 160 KB for 128-wide
template <int NQ> constexpr int tile_lds_bytes() { return (TILE_CAP + 1) * 256 * NQ; }
// 16-byte bf16 chunks staged per thread and tile: (TILE_CAP + 1) * 8 NQ / TNT
template <int NQ> constexpr int tile_chunks() { return (TILE_CAP + 1) * 8 * NQ / TNT; }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));


// float4 chunk of a 64-column block read by this lane in read r (0, 1)
__device__ __forceinline__ int tile_chunk(int sub, int r) {
  const int g = (threadIdx.x >> 3) & 3;
  return 4 * ((2 * g + (sub >> 2) + 2 * r) & 3) + (sub & 3);
}

template <int NQ>
__device__ __forceinline__ void lds_round16(int id0, int id1, int n, const f32x4* img, const int (&chb)[2 * NQ],
                                            f32x2 (&acc)[2 * NQ][2]) {
  // n (wave-uniform) = the wave's longest row in this round; shorter rows read the
  // zero row there (exact +0 adds: bit-identical sums).  Ids become byte offsets
  // before the broadcast (one multiply per lane, not per neighbour).
  const int b0 = id0 * (256 * NQ), b1 = id1 * (256 * NQ);
  int c[16];
  c[0] = bcast8<0>(b0); c[1] = bcast8<1>(b0); c[2] = bcast8<2>(b0); c[3] = bcast8<3>(b0);
  c[4] = bcast8<4>(b0); c[5] = bcast8<5>(b0); c[6] = bcast8<6>(b0); c[7] = bcast8<7>(b0);
  c[8] = bcast8<0>(b1); c[9] = bcast8<1>(b1); c[10] = bcast8<2>(b1); c[11] = bcast8<3>(b1);
  c[12] = bcast8<4>(b1); c[13] = bcast8<5>(b1); c[14] = bcast8<6>(b1); c[15] = bcast8<7>(b1);
  const char* base = reinterpret_cast<const char*>(img);
  constexpr int IF = 8 / NQ;        // neighbours in flight: 64 VGPRs of LDS reads
#pragma unroll
  for (int u0 = 0; u0 < 16; u0 += IF) {
    if (u0 >= n) break;
    f32x4 v[IF][2 * NQ];
#pragma unroll
    for (int u = 0; u < IF; ++u)
#pragma unroll
      for (int i = 0; i < 2 * NQ; ++i) v[u][i] = *reinterpret_cast<const f32x4*>(base + c[u0 + u] + chb[i]);
#pragma unroll
    for (int u = 0; u < IF; ++u) {
      if (u0 + u >= n) break;
#pragma unroll
      for (int i = 0; i < 2 * NQ; ++i) {
        acc[i][0] += v[u][i].xy;
        acc[i][1] += v[u][i].zw;
      }
    }
  }
}

// Epilogue of a row finished in the tiled kernel: this lane holds the 4-column
// groups 4 ch[i] .. 4 ch[i] + 3 (tile_chunk order), acc[i] = {cols 0-1, cols 2-3}.
template <int EPI, int NQ>
__device__ __forceinline__ void spmm_tile_epilogue(const SpmmBfArgs& a, int r, const int (&ch)[2 * NQ],
                                                   const f32x2 (&acc)[2 * NQ][2]) {
#pragma unroll
  for (int i = 0; i < 2 * NQ; ++i) {
    const int col = 4 * ch[i];
    if (col >= a.width) continue;
    const float v[4] = {acc[i][0].x, acc[i][0].y, acc[i][1].x, acc[i][1].y};
    if constexpr (EPI == SND_SPMM_PLAIN) {
      bf16x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (__bf16)v[k];
      *reinterpret_cast<bf16x4*>(a.out + (long long)r * a.ldo + col) = o;
    } else {
      *reinterpret_cast<float4*>(a.pre + (long long)r * a.ldp + col) = make_float4(v[0], v[1], v[2], v[3]);
      bf16x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = col + k;
        const float b1 = lrelu(v[k]) * (a.g1[c] * kBnC) + a.b1[c];    // H2[:, :h1]
        o[k] = (__bf16)(b1 * (a.ge[c] * kBnC) + a.be[c]);             // encoder_g BN
      }
      *reinterpret_cast<bf16x4*>(a.g + (long long)r * a.ldg + col) = o;
    }
  }
  if constexpr (EPI == SND_SPMM_GCN) {
    if ((threadIdx.x & (LPR - 1)) == 0) {   // concat X (model.py:109) -> encoder_g BN on those columns
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = a.width + j;
        g[j] = j < a.f ? a.x[(long long)r * a.ldx + j] * (a.ge[c] * kBnC) + a.be[c] : 0.f;
      }
      *reinterpret_cast<uint4*>(a.g + (long long)r * a.ldg + a.width) = to_bf16x8(g);
    }
  }
}

// Tile run of workgroup b: tiles [lo, hi) of the XCD-major tile list.  With tpg
// tiles per graph and ngraphs % 8 == 0 (and the grid a multiple of 8), XCD x
// = b % 8 owns the graphs g = x (mod 8) and its workgroups split that list into
// contiguous runs; otherwise the tiles are split contiguously.
struct TileRun {
  int lo, hi, tpg, x;
  __device__ int tile(int i) const {
    if (tpg <= 0) return i;
    const int gi = i / tpg;
    return (x + 8 * gi) * tpg + (i - gi * tpg);
  }
};

__device__ __forceinline__ TileRun tile_run(int ntiles, int tpg, int ngraphs) {
  const int G = gridDim.x, b = blockIdx.x;
  if (tpg > 0 && ngraphs % 8 == 0 && G % 8 == 0 && ntiles == tpg * ngraphs) {
    const int x = b & 7, l = b >> 3, gx = G >> 3, tx = ntiles >> 3;
    return TileRun{(int)((long long)l * tx / gx), (int)((long long)(l + 1) * tx / gx), tpg, x};
  }
  return TileRun{(int)((long long)b * ntiles / G), (int)((long long)(b + 1) * ntiles / G), 0, 0};
}

template <int NQ, int RPG>
struct TileMeta {                 // stage 1: row slots and set ids of a tile
  int r[RPG], s[RPG], e[RPG];
  int uc[tile_chunks<NQ>()];
};
template <int NQ, int RPG>
struct TileRows {                 // stage 2: the tile's rows (bf16 chunks) and first local ids
  u32x4 raw[tile_chunks<NQ>()];
  int pre[RPG][TPRE];
};

// RPG rows per 8-lane group: 1 for tiles of <= 64 rows, 2 for <= 128.
// Image row 0 is the zero row, row 1 + u holds set entry u (lcol = 1 + u).
template <int EPI, int NQ, int RPG>
__global__ void __launch_bounds__(TNT) __attribute__((amdgpu_waves_per_eu(NQ == 1 ? 4 : 2)))
spmm_bf16_tiled_kernel(SpmmBfArgs a, int ntiles, int tpg) {
  extern __shared__ f32x4 img[];   // [ustride + 1][16 NQ float4]
  constexpr int CPR = 8 * NQ;      // 16-byte bf16 chunks per row in HBM
  constexpr int TSC = tile_chunks<NQ>();
  const int sub = threadIdx.x & (LPR - 1), grp = threadIdx.x / LPR;
  const int ust = a.t_ustride;
  const int nchunk = (ust + 1) * CPR;           // image chunks incl. the zero row
  const __amdgpu_buffer_rsrc_t rs = rows_rsrc(a.h, (long long)a.R * a.ldh * 2);
  const TileRun run = tile_run(ntiles, tpg, a.ngraphs);
  const int count = run.hi - run.lo;

  auto stage1 = [&](int t, TileMeta<NQ, RPG>& m) {
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
      const int ls = grp + j * TG, slot = t * a.t_rows + ls;
      const bool v = ls < a.t_rows && slot < a.R;
      m.r[j] = v ? a.t_rowid[slot] : -1;
      m.s[j] = v ? a.t_trp[slot] : 0;
      m.e[j] = v ? a.t_trp[slot + 1] : 0;
    }
#pragma unroll
    for (int c = 0; c < TSC; ++c) {
      const int u = (threadIdx.x + c * TNT) / CPR - 1;              // set entry (-1: zero row)
      m.uc[c] = (u >= 0 && u < ust) ? a.t_ucol[(long long)t * ust + u] : -1;   // -1: zeros
    }
  };
  auto stage2 = [&](const TileMeta<NQ, RPG>& m, TileRows<NQ, RPG>& w) {
#pragma unroll
    for (int c = 0; c < TSC; ++c) {
      const int ch = (threadIdx.x + c * TNT) % CPR;
      w.raw[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)m.uc[c] * (2u * a.ldh) + 16u * ch, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < RPG; ++j)
#pragma unroll
      for (int q = 0; q < TPRE; ++q) {
        const int k = m.s[j] + 8 * q + sub;
        w.pre[j][q] = k < m.e[j] ? (int)a.t_lcol[k] : 0;
      }
  };
  // exact bf16 -> fp32 widening of the staged rows into the image (the zero row
  // and the set's rows; set padding is skipped)
  auto write_image = [&](const TileMeta<NQ, RPG>& m, const TileRows<NQ, RPG>& w) {
#pragma unroll
    for (int c = 0; c < TSC; ++c) {
      const int cidx = threadIdx.x + c * TNT;
      if (cidx < nchunk && (cidx < CPR || m.uc[c] >= 0)) {
        const u32x4 v = w.raw[c];
        f32x4 lo, hi;
        lo.x = __uint_as_float(v[0] << 16); lo.y = __uint_as_float(v[0] & 0xFFFF0000u);
        lo.z = __uint_as_float(v[1] << 16); lo.w = __uint_as_float(v[1] & 0xFFFF0000u);
        hi.x = __uint_as_float(v[2] << 16); hi.y = __uint_as_float(v[2] & 0xFFFF0000u);
        hi.z = __uint_as_float(v[3] << 16); hi.w = __uint_as_float(v[3] & 0xFFFF0000u);
        img[2 * cidx] = lo;
        img[2 * cidx + 1] = hi;
      }
    }
  };

  int ch[2 * NQ], chb[2 * NQ];     // this lane's float4 chunks of a row, and their byte offsets
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    ch[2 * q] = 16 * q + tile_chunk(sub, 0);
    ch[2 * q + 1] = 16 * q + tile_chunk(sub, 1);
  }
#pragma unroll
  for (int i = 0; i < 2 * NQ; ++i) chb[i] = 16 * ch[i];
  TileMeta<NQ, RPG> m0, m1;        // m0: the tile in the image, m1: the next one
  TileRows<NQ, RPG> w;
  if (count > 0) {
    stage1(run.tile(run.lo), m0);
    stage2(m0, w);
    if (count > 1) stage1(run.tile(run.lo + 1), m1);
    write_image(m0, w);
  }
  __syncthreads();
  // the previous tile's sums: stored after the next loads are issued, so no wait for
  // a store stands between two tiles' loads
  int prr[RPG];
  f32x2 acc[RPG][2 * NQ][2];
#pragma unroll
  for (int j = 0; j < RPG; ++j) prr[j] = -1;
  // one tile: cur = its metadata (then reused for tile i+2's), nxt = tile i+1's.  The
  // loop runs two tiles per trip with the roles swapped, so no register copy of an
  // in-flight load forces a wait.
  auto body = [&](int i, TileMeta<NQ, RPG>& cur, TileMeta<NQ, RPG>& nxt) {
    int rr[RPG], s0[RPG], e0[RPG], pre[RPG][TPRE];
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
      rr[j] = cur.r[j]; s0[j] = cur.s[j]; e0[j] = cur.e[j];
#pragma unroll
      for (int q = 0; q < TPRE; ++q) pre[j][q] = w.pre[j][q];
    }
    if (i + 1 < count) stage2(nxt, w);             // tile i+1: rows + first local ids
#pragma unroll
    for (int j = 0; j < RPG; ++j)
      if (prr[j] >= 0) spmm_tile_epilogue<EPI, NQ>(a, prr[j], ch, acc[j]);
    if (i + 2 < count) stage1(run.tile(run.lo + i + 2), cur);   // tile i+2: slots + set ids
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
      prr[j] = rr[j];
#pragma unroll
      for (int q = 0; q < 2 * NQ; ++q) acc[j][q][0] = acc[j][q][1] = (f32x2){0.f, 0.f};
      if (j * TG >= a.t_rows) break;               // uniform: no slot of this pass in any tile
      const int s = s0[j], e = e0[j];
      // trip counts: a tile's rows are sorted by degree, so the wave's first row (lane 0)
      // is its longest; shorter and empty rows read the zero row
      const int dm = __builtin_amdgcn_readfirstlane(e - s);
      if (dm > 0) lds_round16<NQ>(pre[j][0], pre[j][1], min(16, dm), img, chb, acc[j]);
      if (dm > 16) lds_round16<NQ>(pre[j][2], pre[j][3], min(16, dm - 16), img, chb, acc[j]);
      for (int o = 8 * TPRE; o < dm; o += 16) {
        const int id0 = s + o + sub < e ? (int)a.t_lcol[s + o + sub] : 0;
        const int id1 = s + o + 8 + sub < e ? (int)a.t_lcol[s + o + 8 + sub] : 0;
        lds_round16<NQ>(id0, id1, min(16, dm - o), img, chb, acc[j]);
      }
    }
    __syncthreads();                               // every wave is done with this image
    if (i + 1 < count) write_image(nxt, w);        // the next tile (its loads ran during the sums)
    __syncthreads();
  };
  for (int i = 0; i < count; i += 2) {
    body(i, m0, m1);
    if (i + 1 < count) body(i + 1, m1, m0);
  }
#pragma unroll
  for (int j = 0; j < RPG; ++j)
    if (prr[j] >= 0) spmm_tile_epilogue<EPI, NQ>(a, prr[j], ch, acc[j]);
}

// ---------------------------------------------------------------- per-edge CE terms (bf16 z)
// For row i and each neighbour j (A_ij = 1), L = z_i . z_j:
//   loss += (pw - 1) softplus(L) - pw L ;  tp += (L > 0) ;  ej_i += ((pw - 1) sigmoid(L) - pw) z_j
// (optimizer.py:142-144 restricted to the A = 1 pairs; the dense kernel adds softplus(L)
// over all pairs).  8 lanes per row, one 16-byte z chunk per lane, 4 neighbours in flight.
template <int NQ>
__global__ void __launch_bounds__(NT) edge_bf16_kernel(EdgeBfArgs a) {
  __shared__ double sl[NT / 64];
  __shared__ unsigned st[NT / 64];
  const int sub = threadIdx.x & (LPR - 1);
  const int r = row_of(a.row_order, xcd_rowblock(blockIdx.x, a.xcd_nbg), a.R);
  const bool rv = r < a.R;
  const int nch = a.d >> 3;
  bool qv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) qv[q] = sub + 8 * q < nch;
  float lossr = 0.f;
  unsigned tp = 0;
  u32x4 zip[NQ];   // z_i packed (bf16 pairs): the dot2 operand
  float acc[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    zip[q] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  }
  if (rv)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (qv[q]) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(a.z + (long long)r * a.d + 64 * q + 8 * sub);
        zip[q] = __builtin_bit_cast(u32x4, v);
      }
  const float pw = a.pos_weight;
  const __amdgpu_buffer_rsrc_t rs = rows_rsrc(a.z, (long long)a.R * a.d * 2);
  gather_rows16<NQ>(a.colidx, rv ? a.rowptr[r] : 0, rv ? a.rowptr[r + 1] : 0, rs, 2u * a.d, sub,
                    [&](int, const u32x4 (&v)[NQ], bool valid) {
    float zj[NQ][8], dot = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const unsigned w = v[q][p];
        zj[q][2 * p] = qv[q] ? __uint_as_float(w << 16) : 0.f;
        zj[q][2 * p + 1] = qv[q] ? __uint_as_float(w & 0xFFFF0000u) : 0.f;
      }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (qv[q]) dot = dot8_bf16(zip[q], v[q], dot);   // as head_bwd_kernel
    const float L = row8_sum(dot);
    if (!valid) return;
    float coef;
    edge_ce_terms(L, pw, coef, lossr);
    lossr -= pw * L;
    tp += L > 0.f ? 1u : 0u;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[q][j] += coef * zj[q][j];
  });
  if (rv) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (qv[q]) {
        float* o = a.ej + (long long)r * a.d + 64 * q + 8 * sub;
        *reinterpret_cast<float4*>(o) = make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(acc[q][4], acc[q][5], acc[q][6], acc[q][7]);
      }
  }
  if (sub != 0 || !rv) { lossr = 0.f; tp = 0; }   // the row's 8 lanes hold the same sums
  const double l = wave_sum_d((double)lossr);
  const unsigned t = wave_sum_u(tp);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sl[w] = l; st[w] = t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tl = 0.0, tt = 0.0;
    for (int k = 0; k < NT / 64; ++k) { tl += sl[k]; tt += (double)st[k]; }
    a.part[2 * blockIdx.x] = tl;
    a.part[2 * blockIdx.x + 1] = tt;
  }
}

// ---------------------------------------------------------------- reparam backward
// dz = adj_scale (dJd + ej) + dz_dec;  dmu = dz + kl mu;  dlogstd = dz eps e^s + kl (e^2s - 1)
// (model.py:159, optimizer.py:193); bf16 output (next GEMM operand) and the
// per-column sums that give the bias gradient of the [mu | logstd] head.
__global__ void __launch_bounds__(NT) reparam_bwd_fast_kernel(ReparamBwdFastArgs a) {
  const int lpr = a.L >> 2, rpb = NT / lpr;
  const int c4 = threadIdx.x % lpr, rl = threadIdx.x / lpr;
  float sm[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = blockIdx.x * rpb + rl; r < a.R; r += gridDim.x * rpb) {
    const long long i = (long long)r * a.L + 4 * c4;
    const float4 mu = *reinterpret_cast<const float4*>(a.ms + (long long)r * a.ldms + 4 * c4);
    const float4 ls = *reinterpret_cast<const float4*>(a.ms + (long long)r * a.ldms + a.L + 4 * c4);
    const float4 ep = *reinterpret_cast<const float4*>(a.eps + i);
    float4 dj = *reinterpret_cast<const float4*>(a.dJd + i);
    for (int sx = 0; sx < a.nextra; ++sx) {   // zzt_split_sum_kernel's order
      const float4 e = *reinterpret_cast<const float4*>(a.dJd_extra + (long long)sx * a.R * a.L + i);
      dj.x += e.x; dj.y += e.y; dj.z += e.z; dj.w += e.w;
    }
    const float4 ej = *reinterpret_cast<const float4*>(a.ej + i);
    const float4 dd = *reinterpret_cast<const float4*>(a.dz_dec + i);
    const float m[4] = {mu.x, mu.y, mu.z, mu.w}, l[4] = {ls.x, ls.y, ls.z, ls.w};
    const float e4[4] = {ep.x, ep.y, ep.z, ep.w}, j4[4] = {dj.x, dj.y, dj.z, dj.w};
    const float q4[4] = {ej.x, ej.y, ej.z, ej.w}, d4[4] = {dd.x, dd.y, dd.z, dd.w};
    bf16x4 om, os;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float dm, dl;
      reparam_bwd_elem(m[t], l[t], e4[t], j4[t], q4[t], d4[t], a.adj_scale, a.kl_scale, dm, dl);
      om[t] = (__bf16)dm;
      os[t] = (__bf16)dl;
      sm[t] += dm;
      ss[t] += dl;
    }
    __bf16* o = a.dms + (long long)r * a.lddms;
    *reinterpret_cast<bf16x4*>(o + 4 * c4) = om;
    *reinterpret_cast<bf16x4*>(o + a.L + 4 * c4) = os;
  }
  __shared__ float red[NT][9];
#pragma unroll
  for (int t = 0; t < 4; ++t) { red[threadIdx.x][t] = sm[t]; red[threadIdx.x][4 + t] = ss[t]; }
  __syncthreads();
  if (threadIdx.x < lpr) {
    float tm[4] = {0.f, 0.f, 0.f, 0.f}, ts[4] = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < rpb; ++q)
#pragma unroll
      for (int t = 0; t < 4; ++t) { tm[t] += red[q * lpr + c4][t]; ts[t] += red[q * lpr + c4][4 + t]; }
    float* cp = a.colpart + (long long)blockIdx.x * 2 * a.L;
#pragma unroll
    for (int t = 0; t < 4; ++t) { cp[4 * c4 + t] = tm[t]; cp[a.L + 4 * c4 + t] = ts[t]; }
  }
}


// ---------------------------------------------------------------- per-edge terms + reparam backward
// edge_bf16_kernel and reparam_bwd_fast_kernel in one launch, for the node-latent fast
// encoder without the fused backward head (L = 128, C5): row r's 8 lanes gather its
// neighbours' z and keep e_r = sum_j coef_ij z_j in registers (edge_bf16_kernel's
// arithmetic, bit for bit), then apply the reparameterisation backward to their 8 (x NQ)
// columns of the row (reparam_bwd_fast_kernel's, bit for bit) -- no EJ round trip, one
// launch fewer, and the per-edge gather runs after zz^T instead of before it.  Partials:
// {loss, tp} per block (as edge_bf16_kernel) and the [mu | s] bias column sums per block
// (the block's 32 rows: shuffles over each wave's 8 rows, then the 4 waves in order).
template <int NQ>
__global__ void __launch_bounds__(NT) edge_reparam_bwd_kernel(EdgeBfArgs e, ReparamBwdFastArgs a) {
  __shared__ double sl[NT / 64];
  __shared__ unsigned st[NT / 64];
  __shared__ float bred[NT / 64][2 * 64 * NQ];
  const int sub = threadIdx.x & (LPR - 1), w = threadIdx.x >> 6;
  const int r = row_of(e.row_order, xcd_rowblock(blockIdx.x, e.xcd_nbg), e.R);
  const bool rv = r < e.R;
  const int L = a.L, nch = L >> 3;
  bool qv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) qv[q] = sub + 8 * q < nch;
  float lossr = 0.f;
  unsigned tp = 0;
  u32x4 zip[NQ];
  float acc[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    zip[q] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  }
  if (rv)
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (qv[q]) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(e.z + (long long)r * e.d + 64 * q + 8 * sub);
        zip[q] = __builtin_bit_cast(u32x4, v);
      }
  const float pw = e.pos_weight;
  const __amdgpu_buffer_rsrc_t rs = rows_rsrc(e.z, (long long)e.R * e.d * 2);
  gather_rows16<NQ>(e.colidx, rv ? e.rowptr[r] : 0, rv ? e.rowptr[r + 1] : 0, rs, 2u * e.d, sub,
                    [&](int, const u32x4 (&v)[NQ], bool valid) {
    float zj[NQ][8], dot = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const unsigned wv = v[q][p];
        zj[q][2 * p] = qv[q] ? __uint_as_float(wv << 16) : 0.f;
        zj[q][2 * p + 1] = qv[q] ? __uint_as_float(wv & 0xFFFF0000u) : 0.f;
      }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (qv[q]) dot = dot8_bf16(zip[q], v[q], dot);
    const float Lij = row8_sum(dot);
    if (!valid) return;
    float coef;
    edge_ce_terms(Lij, pw, coef, lossr);
    lossr -= pw * Lij;
    tp += Lij > 0.f ? 1u : 0u;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[q][j] += coef * zj[q][j];
  });
  // reparameterisation backward of the lane's columns (reparam_bwd_fast_kernel per element)
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float dm[8], dl[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { dm[j] = 0.f; dl[j] = 0.f; }
    const int c0 = 64 * q + 8 * sub;
    if (rv && qv[q]) {
      const float* msr = a.ms + (long long)r * a.ldms;
      const long long ie = (long long)r * L + c0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 mu = *reinterpret_cast<const float4*>(msr + c0 + 4 * h);
        const float4 ls = *reinterpret_cast<const float4*>(msr + L + c0 + 4 * h);
        const float4 ep = *reinterpret_cast<const float4*>(a.eps + ie + 4 * h);
        float4 dj = *reinterpret_cast<const float4*>(a.dJd + ie + 4 * h);
        for (int sx = 0; sx < a.nextra; ++sx) {   // zzt_split_sum_kernel's order
          const float4 x = *reinterpret_cast<const float4*>(a.dJd_extra + (long long)sx * e.R * L + ie + 4 * h);
          dj.x += x.x; dj.y += x.y; dj.z += x.z; dj.w += x.w;
        }
        const float4 dd = *reinterpret_cast<const float4*>(a.dz_dec + ie + 4 * h);
        const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, l4[4] = {ls.x, ls.y, ls.z, ls.w};
        const float e4[4] = {ep.x, ep.y, ep.z, ep.w}, j4[4] = {dj.x, dj.y, dj.z, dj.w};
        const float d4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
          reparam_bwd_elem(m4[u], l4[u], e4[u], j4[u], acc[q][4 * h + u], d4[u], a.adj_scale, a.kl_scale,
                           dm[4 * h + u], dl[4 * h + u]);
      }
      bf16x8 om, os;
#pragma unroll
      for (int j = 0; j < 8; ++j) { om[j] = (__bf16)dm[j]; os[j] = (__bf16)dl[j]; }
      *reinterpret_cast<bf16x8*>(a.dms + (long long)r * a.lddms + c0) = om;
      *reinterpret_cast<bf16x8*>(a.dms + (long long)r * a.lddms + L + c0) = os;
    }
    if (qv[q]) {   // bias sums over the wave's 8 rows (lanes sub, sub + 8, ..., sub + 56)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float sm = dm[j], ss = dl[j];
        sm += __shfl_xor(sm, 8, 64); sm += __shfl_xor(sm, 16, 64); sm += __shfl_xor(sm, 32, 64);
        ss += __shfl_xor(ss, 8, 64); ss += __shfl_xor(ss, 16, 64); ss += __shfl_xor(ss, 32, 64);
        if ((threadIdx.x & 63) < 8) { bred[w][c0 + j] = sm; bred[w][L + c0 + j] = ss; }
      }
    }
  }
  if (sub != 0 || !rv) { lossr = 0.f; tp = 0; }   // the row's 8 lanes hold the same sums
  const double l = wave_sum_d((double)lossr);
  const unsigned t = wave_sum_u(tp);
  if ((threadIdx.x & 63) == 0) { sl[w] = l; st[w] = t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tl = 0.0, tt = 0.0;
    for (int k = 0; k < NT / 64; ++k) { tl += sl[k]; tt += (double)st[k]; }
    e.part[2 * blockIdx.x] = tl;
    e.part[2 * blockIdx.x + 1] = tt;
  }
  for (int c = threadIdx.x; c < 2 * L; c += NT) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) v += bred[k][c];
    a.colpart[(long long)blockIdx.x * 2 * L + c] = v;
  }
}

// ---------------------------------------------------------------- reparam + zz^T staging
// z = mu + eps e^s (model.py:159) with the KL partial (optimizer.py:193), fused
// with the zz^T staging images: one block = 64 rows of one graph, writes z (fp32,
// edge terms), eps, z (bf16, decoder operand), z sqrt(log2 e) (bf16, K role),
// z^T (bf16, V role, through an LDS transpose) and the per-64-row column sums.
// (1024 threads: at DP = 128 a 256-thread block ran 8 dependent load -> store rounds per
// thread over its 64 rows, one workgroup per CU -- latency-bound; now 2)
constexpr int NTP = 1024;
template <int DP>
__global__ void __launch_bounds__(NTP) reparam_prep_kernel(ReparamPrepArgs a) {
  constexpr int NT = NTP;
  __shared__ float tile[64][DP + 1];
  __shared__ float stile[64][DP + 1];
  __shared__ double red[NT / 64];
  const int g = blockIdx.y, rb = blockIdx.x;
  const int L = a.L;                      // multiple of 4 (16 / 32 / 64 / 128)
  const unsigned off = a.step ? (unsigned)(*a.step) : 0u;
  if (a.stepn && g == 0 && rb == 0 && threadIdx.x == 0) *a.stepn = (int)off + 1;
  const float sc = 1.2011224087864498f;  // sqrt(log2 e)
  constexpr int Q = DP / 4;               // 4-column quads per row: one Philox block each
  double kl = 0.0;
  for (int idx = threadIdx.x; idx < 64 * Q; idx += NT) {
    const int rr = idx / Q, c = 4 * (idx - rr * Q);
    const int row = rb * 64 + rr;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (row < a.n && c < L) {
      const long long gr = (long long)g * a.n + row;
      const long long i = gr * L + c;
      const float4 m = *reinterpret_cast<const float4*>(a.ms + gr * a.ldms + c);
      if (a.stage_only) {
        z[0] = m.x; z[1] = m.y; z[2] = m.z; z[3] = m.w;
      } else {
        const float4 ls = *reinterpret_cast<const float4*>(a.ms + gr * a.ldms + L + c);
        const float4 ep = a.eps_in ? *reinterpret_cast<const float4*>(a.eps_in + i)
                                   : philox_normal4(a.seed, off, (a.eps_base + (unsigned long long)i) >> 2);
        const float mu[4] = {m.x, m.y, m.z, m.w}, s[4] = {ls.x, ls.y, ls.z, ls.w};
        const float e[4] = {ep.x, ep.y, ep.z, ep.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float es = __expf(s[t]);
          z[t] = mu[t] + e[t] * es;                                      // model.py:159
          kl += (double)kl_elem(s[t], mu[t]);    // optimizer.py:193
        }
        *reinterpret_cast<float4*>(a.z + i) = make_float4(z[0], z[1], z[2], z[3]);
        *reinterpret_cast<float4*>(a.eps_out + i) = ep;
      }
      bf16x4 zb;
#pragma unroll
      for (int t = 0; t < 4; ++t) zb[t] = (__bf16)z[t];
      *reinterpret_cast<bf16x4*>(a.zb + gr * L + c) = zb;
    }
    bf16x4 jb;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      tile[rr][c + t] = z[t];
      jb[t] = (__bf16)(z[t] * sc);
      stile[rr][c + t] = (float)jb[t];
    }
    *reinterpret_cast<bf16x4*>(a.jrow + ((long long)g * a.npad + row) * DP + c) = jb;
  }
  kl = wave_sum_d(kl);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = kl;
  __syncthreads();
  if (threadIdx.x == 0 && a.kl_part) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += red[k];
    a.kl_part[blockIdx.y * gridDim.x + blockIdx.x] = t;
  }
  if (threadIdx.x < DP) {
    float cs = 0.f;
    for (int rr = 0; rr < 64; ++rr) cs += stile[rr][threadIdx.x];
    a.colpart[((long long)g * (a.npad / 64) + rb) * DP + threadIdx.x] = cs;
  }
  // z^T image: 4 consecutive rows per lane (8-byte stores)
  for (int idx = threadIdx.x; idx < 16 * DP; idx += NT) {
    const int c = idx >> 4, r4 = 4 * (idx & 15);
    bf16x4 t;
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = (__bf16)tile[r4 + u][c];
    *reinterpret_cast<bf16x4*>(a.jt + ((long long)g * DP + c) * a.npad + rb * 64 + r4) = t;
  }
}

}  // namespace

int gcn0_blocks(int R) { return cdiv(R, RPB); }

int xcd_nbg(int npg, int ngraphs) {
  return (npg % RPB == 0 && ngraphs % 8 == 0) ? npg / RPB : 0;
}

int launch_gcn0(const Gcn0Args& a0, hipStream_t s) {
  if (a0.R <= 0) return 0;
  Gcn0Args a = a0;
  SND_CHECK_ARG(a.npack >= 0 && a.npack <= kMaxPack, "gcn0: at most %d packed images", kMaxPack);
  int pb = 0;
  for (int i = 0; i < a.npack; ++i) {
    const PackDesc& x = a.pack[i];
    SND_CHECK_ARG((x.kp == 32 || x.kp == 64 || x.kp == 128 || x.kp == 256) && x.np % 16 == 0 && x.np > 0 &&
                      x.T >= 1 && x.nsrc >= 1 && x.nsrc <= 2 && x.dst,
                  "gcn0: bad pack descriptor %d (kp %d np %d T %d)", i, x.kp, x.np, x.T);
    a.pack_blk[i] = pb;
    pb += cdiv(pack_chunks(x), NT);
  }
  a.pack_blk[a.npack] = pb;
  SND_CHECK_ARG(a.f >= 1 && a.f <= 4 && a.h0 % 8 == 0 && a.h0 <= 128 && a.ldh1 % 8 == 0 &&
                    a.ldh1 >= a.h0 + 8,
                "gcn0: f in 1..4, h0 %% 8 (<= 128), ldh1 >= h0 + 8");
  SND_CHECK_ARG(a.rowptr && a.x && a.w0 && a.g0 && a.b0 && a.h1 && a.ax && a.axb, "gcn0: null operand");
  hipLaunchKernelGGL(gcn0_kernel, dim3(gcn0_blocks(a.R) + pb), dim3(NT), 0, s, a);
  SND_LAUNCH_CHECK("gcn0_kernel");
  return 0;
}

template <typename K>
static int tile_lds_attr(K kern, int bytes) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                             bytes) == hipSuccess ? 0 : SND_ERR_HIP;
}

template <int EPI>
static int launch_spmm_bf16_epi(const SpmmBfArgs& a, bool two, hipStream_t s) {
  // The tiled kernel pays off through its pipeline (runs of tiles per workgroup)
  // and, for the plain epilogue, its LDS sums; a GraphConvolution epilogue over
  // ~1 tile per workgroup (the step's 8-graph batch, 512 tiles) is faster on the
  // register kernel, whose epilogue stores whole rows per 8-lane group
  // (16.6 vs 10.8 us at B = 8).  Up to 4 tiles per workgroup (B <= 32) the choice
  // is a wash: whole-step A/B with debug bit 2048 (tiles kept) at B = 8 / 16 / 32
  // measured 0.3407 / 0.5673 / 0.9867 ms (register) vs 0.3396 / 0.5670 / 0.9894 ms
  // (tiled), round 2; beyond that the tiled pipeline is used.
  const bool gcn_small = EPI == SND_SPMM_GCN && a.t_rows > 0 && cdiv(a.R, a.t_rows) <= 4 * 512 &&
                         !(debug_flags() & 2048);
  if (a.t_rows > 0 && a.t_ustride <= TILE_CAP && !gcn_small) {
    static const int attr = tile_lds_attr(spmm_bf16_tiled_kernel<EPI, 1, 1>, tile_lds_bytes<1>()) |
                            tile_lds_attr(spmm_bf16_tiled_kernel<EPI, 1, 2>, tile_lds_bytes<1>()) |
                            tile_lds_attr(spmm_bf16_tiled_kernel<EPI, 2, 1>, tile_lds_bytes<2>()) |
                            tile_lds_attr(spmm_bf16_tiled_kernel<EPI, 2, 2>, tile_lds_bytes<2>());
    if (attr) { set_error("spmm_bf16_tiled: hipFuncSetAttribute failed"); return SND_ERR_HIP; }
    const int ntiles = cdiv(a.R, a.t_rows);
    const size_t lds = (size_t)(a.t_ustride + 1) * 256 * (two ? 2 : 1);
    const int tpg = (a.npg > 0 && a.npg % a.t_rows == 0 && a.ngraphs % 8 == 0 &&
                     (long long)a.npg * a.ngraphs == a.R) ? a.npg / a.t_rows : 0;
    const int per_cu = std::max(1, std::min(2, (160 * 1024) / (int)std::max<size_t>(lds, 1)));
    const int grid = std::min(ntiles, 256 * per_cu);
    const bool one = a.t_rows <= TG;
#define SND_TILED(NQ, RPG) \
  hipLaunchKernelGGL((spmm_bf16_tiled_kernel<EPI, NQ, RPG>), dim3(grid), dim3(TNT), lds, s, a, ntiles, tpg)
    if (two) { if (one) SND_TILED(2, 1); else SND_TILED(2, 2); }
    else { if (one) SND_TILED(1, 1); else SND_TILED(1, 2); }
#undef SND_TILED
    return 0;
  }
  // no tiles, or a tile set beyond the LDS image: the register-gather kernel
  SND_CHECK_ARG(a.colidx || a.R == 0, "spmm_bf16: colidx");
  dim3 grid(cdiv(a.R, RPB));
  if (two) hipLaunchKernelGGL((spmm_bf16_kernel<EPI, 2>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((spmm_bf16_kernel<EPI, 1>), grid, dim3(NT), 0, s, a);
  return 0;
}

int launch_spmm_bf16(const SpmmBfArgs& a, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG(a.width % 8 == 0 && a.width <= 128 && a.ldh % 8 == 0, "spmm_bf16: width %% 8 <= 128, ldh %% 8");
  SND_CHECK_ARG((long long)a.R * a.ldh * 2 < (1ll << 31), "spmm_bf16: rows x ldh beyond the 2 GB buffer range");
  SND_CHECK_ARG(a.t_rows >= 0 && a.t_rows <= TRPG * TG, "spmm_bf16: tile_rows <= 128");
  SND_CHECK_ARG(a.t_rows == 0 || (a.t_rowid && a.t_trp && a.t_lcol && a.t_ucol && a.t_ustride >= 0 &&
                                  a.t_ustride <= 65535),
                "spmm_bf16: row tiles need rows, trp, lcol, ucol and 0 <= ustride <= 65535");
  const bool two = a.width > 64;
  if (a.epi == SND_SPMM_PLAIN) {
    SND_CHECK_ARG(a.out && a.ldo % 8 == 0, "spmm_bf16: out");
    SND_TRY(launch_spmm_bf16_epi<SND_SPMM_PLAIN>(a, two, s));
  } else {
    SND_CHECK_ARG(a.pre && a.g && a.g1 && a.b1 && a.ge && a.be && a.x && a.f <= 8 &&
                      a.ldp % 4 == 0 && a.ldg % 8 == 0 && a.ldg >= a.width + 8,
                  "spmm_bf16: GCN operands");
    SND_TRY(launch_spmm_bf16_epi<SND_SPMM_GCN>(a, two, s));
  }
  SND_LAUNCH_CHECK("spmm_bf16_kernel");
  return 0;
}

int edge_bf16_blocks(int R) { return cdiv(R, RPB); }

int launch_edge_bf16(const EdgeBfArgs& a, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG(a.d % 8 == 0 && a.d <= 128 && a.z && a.ej && a.part && a.rowptr, "edge_bf16: operands");
  SND_CHECK_ARG((long long)a.R * a.d * 2 < (1ll << 31), "edge_bf16: rows x d beyond the 2 GB buffer range");
  if (a.d > 64) hipLaunchKernelGGL(edge_bf16_kernel<2>, dim3(edge_bf16_blocks(a.R)), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(edge_bf16_kernel<1>, dim3(edge_bf16_blocks(a.R)), dim3(NT), 0, s, a);
  SND_LAUNCH_CHECK("edge_bf16_kernel");
  return 0;
}

int reparam_prep_blocks(int ngraphs, int npad) { return ngraphs * (npad / 64); }

int launch_reparam_prep(const ReparamPrepArgs& a, int dp, hipStream_t s) {
  if (a.ngraphs <= 0) return 0;
  SND_CHECK_ARG(a.npad % 64 == 0 && a.L <= dp && a.L % 4 == 0 && a.ldms % 4 == 0,
                "reparam_prep: npad %% 64, L <= dp, L and ldms %% 4");
  SND_CHECK_ARG(a.ms && a.zb && a.jrow && a.jt && a.colpart &&
                    (a.stage_only || (a.z && a.eps_out && a.kl_part)),
                "reparam_prep: null operand");
  dim3 grid(a.npad / 64, a.ngraphs);
  switch (dp) {
    case 32: hipLaunchKernelGGL((reparam_prep_kernel<32>), grid, dim3(NTP), 0, s, a); break;
    case 64: hipLaunchKernelGGL((reparam_prep_kernel<64>), grid, dim3(NTP), 0, s, a); break;
    case 128: hipLaunchKernelGGL((reparam_prep_kernel<128>), grid, dim3(NTP), 0, s, a); break;
    default: set_error("reparam_prep: dp %d", dp); return SND_ERR_ARG;
  }
  SND_LAUNCH_CHECK("reparam_prep_kernel");
  return 0;
}

int edge_reparam_blocks(int R) { return cdiv(R, RPB); }

int launch_edge_reparam_bwd(const EdgeBfArgs& e, const ReparamBwdFastArgs& a, hipStream_t s) {
  if (e.R <= 0) return 0;
  SND_CHECK_ARG(e.d == a.L && e.R == a.R && e.d % 8 == 0 && e.d <= 128 && e.z && e.part && e.rowptr,
                "edge_reparam_bwd: edge operands");
  SND_CHECK_ARG((a.L == 16 || a.L == 32 || a.L == 64 || a.L == 128) && a.ldms % 4 == 0 && a.lddms % 8 == 0,
                "edge_reparam_bwd: L / leading dims");
  SND_CHECK_ARG(a.dz_dec && a.dJd && a.eps && a.dms && a.colpart && a.ms, "edge_reparam_bwd: null operand");
  SND_CHECK_ARG((long long)e.R * e.d * 2 < (1ll << 31), "edge_reparam_bwd: rows x d beyond the 2 GB buffer range");
  if (a.L > 64) hipLaunchKernelGGL(edge_reparam_bwd_kernel<2>, dim3(edge_reparam_blocks(e.R)), dim3(NT), 0, s, e, a);
  else hipLaunchKernelGGL(edge_reparam_bwd_kernel<1>, dim3(edge_reparam_blocks(e.R)), dim3(NT), 0, s, e, a);
  SND_LAUNCH_CHECK("edge_reparam_bwd_kernel");
  return 0;
}

int reparam_bwd_fast_blocks(int R, int L) {
  const int rpb = NT / (L / 4);
  return std::min(cdiv(R, rpb), 512);
}

int launch_reparam_bwd_fast(const ReparamBwdFastArgs& a, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG((a.L == 16 || a.L == 32 || a.L == 64 || a.L == 128) && a.ldms % 4 == 0 && a.lddms % 4 == 0,
                "reparam_bwd_fast: L / leading dims");
  SND_CHECK_ARG(a.dz_dec && a.dJd && a.ej && a.eps && a.dms && a.colpart, "reparam_bwd_fast: null operand");
  hipLaunchKernelGGL(reparam_bwd_fast_kernel, dim3(reparam_bwd_fast_blocks(a.R, a.L)), dim3(NT), 0, s, a);
  SND_LAUNCH_CHECK("reparam_bwd_fast_kernel");
  return 0;
}

}  // namespace snd

using namespace snd;

extern "C" int snd_csr_spmm_bf16(const int* rowptr, const int* colidx, int n_rows, const void* h,
                                 int ldh, int width, void* out, int ldo, int n_per_graph,
                                 int n_graphs, const int* row_order, snd_stream_t stream) {
  SND_CHECK_ARG(rowptr && (colidx || n_rows == 0) && h && out && n_rows >= 0,
                "snd_csr_spmm_bf16: null operand");
  SpmmBfArgs a{rowptr, colidx, n_rows, reinterpret_cast<const __bf16*>(h), ldh, width,
               SND_SPMM_PLAIN, reinterpret_cast<__bf16*>(out), ldo};
  a.xcd_nbg = (n_per_graph > 0 && n_graphs > 0 && (long long)n_per_graph * n_graphs == n_rows)
                  ? xcd_nbg(n_per_graph, n_graphs) : 0;
  a.row_order = row_order;
  return launch_spmm_bf16(a, (hipStream_t)stream);
}

extern "C" int snd_csr_spmm_bf16_tiled(const int* rowptr, const int* colidx, int n_rows,
                                       const snd_row_tiles_t* tiles, const void* h, int ldh, int width,
                                       void* out, int ldo, int n_per_graph, int n_graphs,
                                       const int* row_order, snd_stream_t stream) {
  SND_CHECK_ARG(rowptr && (colidx || n_rows == 0) && h && out && n_rows >= 0 && tiles && tiles->tile_rows > 0,
                "snd_csr_spmm_bf16_tiled: null operand or no tiles");
  SpmmBfArgs a{rowptr, colidx, n_rows, reinterpret_cast<const __bf16*>(h), ldh, width,
               SND_SPMM_PLAIN, reinterpret_cast<__bf16*>(out), ldo};
  a.xcd_nbg = 0;
  a.row_order = row_order;
  a.t_rowid = tiles->rows; a.t_trp = tiles->trp; a.t_lcol = tiles->lcol; a.t_ucol = tiles->ucol;
  a.t_rows = tiles->tile_rows; a.t_ustride = tiles->ustride;
  a.npg = n_per_graph; a.ngraphs = n_graphs;
  return launch_spmm_bf16(a, (hipStream_t)stream);
}
