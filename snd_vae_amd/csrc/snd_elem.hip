// Element-wise and reduction kernels of the SND-VAE step: reparameterisation
// + KL, sigmoid/MSE heads, BN/lrelu backward with column partial sums,
// deterministic slab reduction, TF1 Adam, and the loss finalizer.
// All memory-bound; each reads its inputs once (HBM roofline).
#include "snd_elem.hpp"

#include <algorithm>
#include "snd_gemm.hpp"
#include "snd_tref.hpp"

namespace snd {
namespace {

template <typename T>
__device__ __forceinline__ T block_sum(T v) {
  __shared__ T sh[16];
  v = (sizeof(T) == 8) ? (T)wave_sum_d((double)v) : (T)wave_sum((float)v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  T t = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < nw; ++k) t += sh[k];
  return t;  // valid in thread 0
}

// ---------------------------------------------------------------- reparam
constexpr int kReparamGrid = 2048;

// thread -> (row, column) with a fixed column per thread: no per-element
// division; rows stride over the grid.  L <= 256.
__global__ void __launch_bounds__(256) reparam_fwd_kernel(ReparamFwdArgs a) {
  const unsigned off = a.step ? (unsigned)(*a.step) : 0u;
  if (a.stepn && blockIdx.x == 0 && threadIdx.x == 0) *a.stepn = (int)off + 1;
  const int rpb = 256 / a.L;                       // rows per block pass
  const int c = threadIdx.x % a.L, rl = threadIdx.x / a.L;
  double kl = 0.0;
  if (rl < rpb) {
    for (int r = blockIdx.x * rpb + rl; r < a.rows; r += gridDim.x * rpb) {
      const long long i = (long long)r * a.L + c;
      const float mu = a.ms[(long long)r * a.ldms + c];
      const float ls = a.ms[(long long)r * a.ldms + a.L + c];
      const float eps = a.eps_in ? a.eps_in[i] : philox_normal(a.seed, off, a.eps_base + (unsigned long long)i);
      const float es = __expf(ls);
      const float zv = mu + eps * es;       // model.py:159
      a.z[i] = zv;
      if (a.zb) a.zb[(long long)r * a.ldzb + c] = (__bf16)zv;
      if (a.eps_out) a.eps_out[i] = eps;
      kl += (double)kl_elem(ls, mu);   // optimizer.py:193
    }
  }
  const double t = block_sum(kl);
  if (threadIdx.x == 0) a.kl_part[blockIdx.x] = t;
}

__global__ void __launch_bounds__(256) reparam_bwd_kernel(ReparamBwdArgs a) {
  const int rpb = 256 / a.L;
  const int c = threadIdx.x % a.L, rl = threadIdx.x / a.L;
  if (rl >= rpb) return;
  for (int r = blockIdx.x * rpb + rl; r < a.rows; r += gridDim.x * rpb) {
    const long long i = (long long)r * a.L + c;
    const float mu = a.ms[(long long)r * a.ldms + c];
    const float ls = a.ms[(long long)r * a.ldms + a.L + c];
    const float es = __expf(ls);
    float dz = a.dJd ? a.adj_scale * (a.dJd[i] + a.ej[i]) : 0.f;
    if (a.dz_dec) dz += a.dz_dec[i];
    a.dms[(long long)r * a.lddms + c] = dz + a.kl_scale * mu;
    a.dms[(long long)r * a.lddms + a.L + c] = dz * a.eps[i] * es + a.kl_scale * (es * es - 1.f);
  }
}

// ---------------------------------------------------------------- graph-latent small heads
constexpr int kSHC = 8;        // latent columns per forward block (mu and logstd: 2 x 8 of Wms)
constexpr int kSHK = 128;      // gh limit
constexpr int kSHN = 64;       // columns of [mu || s] per backward block
constexpr int kSHD = 16;       // h columns per dh block
constexpr int kSHL2 = 256;     // 2L limit

__global__ void __launch_bounds__(256) small_head_fwd_kernel(SmallHeadFwdArgs a) {
  __shared__ float ws[kSHK][2 * kSHC];            // Wms columns c0.. (mu) and L + c0.. (logstd)
  __shared__ float hs[kSmallHeadRows][kSHK];
  const int c0 = blockIdx.x * kSHC, L2 = 2 * a.L, t = threadIdx.x;
  for (int i = t; i < a.gh * 2 * kSHC; i += 256) {
    const int k = i / (2 * kSHC), j = i - k * 2 * kSHC;
    const int c = c0 + (j & (kSHC - 1));
    ws[k][j] = c < a.L ? a.wms[k * L2 + (j < kSHC ? c : a.L + c)] : 0.f;
  }
  for (int i = t; i < a.rows * a.gh; i += 256) hs[i / a.gh][i % a.gh] = a.hh[i];
  __syncthreads();
  const unsigned off = a.step ? (unsigned)(*a.step) : 0u;
  if (a.stepn && blockIdx.x == 0 && t == 0) *a.stepn = (int)off + 1;
  const int b = t / kSHC, j = t - b * kSHC, c = c0 + j;
  double kl = 0.0;
  if (b < a.rows && c < a.L) {
    float mu = 0.f, ls = 0.f;
    for (int k = 0; k < a.gh; ++k) {
      mu = fmaf(hs[b][k], ws[k][j], mu);
      ls = fmaf(hs[b][k], ws[k][kSHC + j], ls);
    }
    mu += a.bms[c];
    ls += a.bms[a.L + c];
    a.ms[b * L2 + c] = mu;
    a.ms[b * L2 + a.L + c] = ls;
    const int i = b * a.L + c;
    const float eps = a.eps_in ? a.eps_in[i] : philox_normal(a.seed, off, a.eps_base + (unsigned long long)i);
    const float es = __expf(ls);
    a.z[i] = mu + eps * es;                // model.py:159
    if (a.eps_out) a.eps_out[i] = eps;
    kl = (double)kl_elem(ls, mu);   // optimizer.py:193
  }
  const double s = block_sum(kl);
  if (t == 0) a.kl_part[blockIdx.x] = s;
}

// d[mu || s] of the block's 64 columns for every row, then their Wms / bms slab columns
__global__ void __launch_bounds__(256) small_head_dms_kernel(SmallHeadBwdArgs a) {
  __shared__ float dm[kSmallHeadRows][kSHN];
  __shared__ float hs[kSmallHeadRows][kSHK];
  const int L2 = 2 * a.L, t = threadIdx.x, nl = t & (kSHN - 1), grp = t >> 6;
  const int n = blockIdx.x * kSHN + nl;
  for (int i = t; i < a.rows * a.gh; i += 256) hs[i / a.gh][i % a.gh] = a.hh[i];
  if (n < L2) {
    const int c = n < a.L ? n : n - a.L;
    for (int b = grp; b < a.rows; b += 4) {
      const float mu = a.ms[b * L2 + c], ls = a.ms[b * L2 + a.L + c];
      const float es = __expf(ls);
      const float dz = a.dz[b * a.L + c];
      const float v = n < a.L ? dz + a.kl_scale * mu : dz * a.eps[b * a.L + c] * es + a.kl_scale * (es * es - 1.f);
      a.dms[b * L2 + n] = v;
      dm[b][nl] = v;
    }
  }
  __syncthreads();
  if (n >= L2) return;
  for (int k = grp; k <= a.gh; k += 4) {
    float acc = 0.f;
    if (k < a.gh)
      for (int b = 0; b < a.rows; ++b) acc = fmaf(hs[b][k], dm[b][nl], acc);
    else
      for (int b = 0; b < a.rows; ++b) acc += dm[b][nl];
    a.slab[k * L2 + n] = acc;
  }
}

// dh[b][k] = sum_n d[mu || s][b][n] Wms[k][n] for the block's 16 h columns
__global__ void __launch_bounds__(256) small_head_dh_kernel(SmallHeadBwdArgs a) {
  __shared__ float dm[kSmallHeadRows][kSHL2 + 1];
  __shared__ float ws[kSHD][kSHL2 + 1];
  const int L2 = 2 * a.L, t = threadIdx.x, k0 = blockIdx.x * kSHD;
  for (int i = t; i < a.rows * L2; i += 256) dm[i / L2][i % L2] = a.dms[i];
  for (int i = t; i < kSHD * L2; i += 256) {
    const int kk = i / L2, n = i - kk * L2;
    ws[kk][n] = k0 + kk < a.gh ? a.wms[(k0 + kk) * L2 + n] : 0.f;
  }
  __syncthreads();
  const int b = t / kSHD, kk = t - b * kSHD, k = k0 + kk;
  if (b >= a.rows || k >= a.gh) return;
  float acc = 0.f;
  for (int n = 0; n < L2; ++n) acc = fmaf(dm[b][n], ws[kk][n], acc);
  a.dh[b * a.gh + k] = acc;
}

// ---------------------------------------------------------------- heads
constexpr int kHeadRows = 256;
constexpr int kHeadK = 64, kHeadO = 4;

struct HeadPack { HeadArgs h[2]; };
struct DecPack { DecBwdArgs d[2]; };

__global__ void __launch_bounds__(256) heads_kernel(HeadPack pk, int rows) {
  const HeadArgs& h = pk.h[blockIdx.y];
  __shared__ float su[kHeadRows][kHeadK + 1];
  __shared__ float sd[kHeadRows][kHeadO];
  const int r0 = blockIdx.x * kHeadRows;
  const int nrow = min(kHeadRows, rows - r0);
  // coalesced staging of the block's [rows x cin] input tile
  for (int idx = threadIdx.x; idx < kHeadRows * h.cin; idx += 256) {
    const int rr = idx / h.cin, k = idx - rr * h.cin;
    su[rr][k] = rr < nrow ? h.u[(long long)(r0 + rr) * h.ldu + k] : 0.f;
  }
  __syncthreads();
  const int rr = threadIdx.x, r = r0 + rr;
  double sse = 0.0;
  float dp[kHeadO];
#pragma unroll
  for (int o = 0; o < kHeadO; ++o) {
    dp[o] = 0.f;
    if (o < h.cout && rr < nrow) {
      float zo = h.b[o];
      for (int k = 0; k < h.cin; ++k) zo += su[rr][k] * h.w[k * h.cout + o];
      const float y = 1.f / (1.f + __expf(-zo));
      if (h.yhat) h.yhat[(long long)r * h.cout + o] = y;
      const float diff = y - (h.target ? h.target[(long long)r * h.ldt + o] : 0.f);
      sse += (double)diff * diff;
      dp[o] = 2.f * diff / h.count * y * (1.f - y);
    }
    sd[rr][o] = dp[o];
  }
  const double t = block_sum(sse);
  if (threadIdx.x == 0) h.sse_part[blockIdx.x] = t;
  __syncthreads();
  // du = dpre @ w^T, written coalesced from LDS
  for (int idx = threadIdx.x; idx < nrow * h.cin; idx += 256) {
    const int row = idx / h.cin, k = idx - row * h.cin;
    float du = 0.f;
#pragma unroll
    for (int o = 0; o < kHeadO; ++o)
      if (o < h.cout) du += sd[row][o] * h.w[k * h.cout + o];
    h.du[(long long)(r0 + row) * h.lddu + k] = du;
  }
  // dW, db partials of this block
  const int nw = h.cin * h.cout;
  for (int idx = threadIdx.x; idx < nw + h.cout; idx += 256) {
    float acc = 0.f;
    if (idx < nw) {
      const int k = idx / h.cout, o = idx - k * h.cout;
      for (int q = 0; q < kHeadRows; ++q) acc += su[q][k] * sd[q][o];
    } else {
      const int o = idx - nw;
      for (int q = 0; q < kHeadRows; ++q) acc += sd[q][o];
    }
    h.wpart[(long long)blockIdx.x * (nw + h.cout) + idx] = acc;
  }
}

// ---------------------------------------------------------------- BN/lrelu bwd
// Column-reduction kernels: block = kColRows rows x all columns; 256 threads in
// a (RP rows) x (CP columns) layout so every row read is coalesced; per-thread
// column sums are combined across the RP row lanes in LDS (fixed order).  At the
// widest layout (CP = 256, one row lane) a thread walks 64 rows: rows go in groups
// of 8 whose loads are all issued before the group's stores (one row in flight per
// thread left enc_bwd<256> at 59.5 us in the C5 step, one wave per SIMD).
template <int CP>
__device__ __forceinline__ float lane_rows_sum(float v, float* red) {
  constexpr int RP = 256 / CP;
  red[threadIdx.x] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x < CP)
    for (int k = 0; k < RP; ++k) t += red[k * CP + threadIdx.x];
  __syncthreads();
  return t;
}

template <int CP>
__global__ void __launch_bounds__(256) dec_bwd_kernel(DecPack pk, int rows) {
  constexpr int RP = 256 / CP;
  __shared__ float red[256];
  const DecBwdArgs& a = pk.d[blockIdx.y];
  const int c = threadIdx.x % CP, ty = threadIdx.x / CP;
  const bool on = c < a.ncols;
  const float gc = on ? a.gamma[c] * kBnC : 0.f, be = on ? a.beta[c] : 0.f;
  float sg = 0.f, sb = 0.f, sy = 0.f;
  const int r0 = blockIdx.x * kColRows, r1 = min(rows, r0 + kColRows);
  if (on) {
    constexpr int RG = 8;   // a group's loads before its stores (see enc_bwd_kernel)
    for (int rb = r0 + ty; rb < r1; rb += RG * RP) {
      float yv[RG], uv[RG];
#pragma unroll
      for (int k = 0; k < RG; ++k) {
        const int r = rb + k * RP;
        const bool rv = r < r1;
        yv[k] = rv ? a.y[(long long)r * a.ldy + c] : 0.f;
        uv[k] = rv ? a.du[(long long)r * a.lddu + c] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < RG; ++k) {
        const int r = rb + k * RP;
        if (r >= r1) break;
        const float y = yv[k];
        const float t = y * gc + be;
        const float dt = uv[k] * lrelu_grad(t);
        const float dy = dt * gc;
        a.dy[(long long)r * a.lddy + c] = dy;
        sg += dt * y;
        sb += dt;
        sy += dy;
      }
    }
  }
  sg = lane_rows_sum<CP>(sg, red);
  sb = lane_rows_sum<CP>(sb, red);
  sy = lane_rows_sum<CP>(sy, red);
  if (threadIdx.x < a.ncols) {
    float* p = a.part + (long long)blockIdx.x * 3 * a.ncols;
    p[c] = sg * kBnC;
    p[a.ncols + c] = sb;
    p[2 * a.ncols + c] = sy;
  }
}

template <int CP>
__global__ void __launch_bounds__(256) enc_bwd_kernel(EncBwdArgs a, int rows) {
  constexpr int RP = 256 / CP;
  __shared__ float red[256];
  const int c = threadIdx.x % CP, ty = threadIdx.x / CP;
  const int width = a.has_enc ? a.wenc : a.h;
  const bool on = c < width;
  const float gec = (on && a.has_enc) ? a.ge[c] * kBnC : 1.f;
  const float gc = c < a.h ? a.g[c] * kBnC : 0.f;
  float sge = 0.f, sbe = 0.f, sg = 0.f, sb = 0.f;
  const int r0 = blockIdx.x * kColRows, r1 = min(rows, r0 + kColRows);
  if (on) {
    // rows in groups of RG: every input of the group is loaded before the first
    // dp store (the store may alias the inputs as far as the compiler knows, so a
    // plain loop keeps one row's loads in flight per thread; same sums, same order)
    constexpr int RG = 8;
    const bool hc = c < a.h, he = a.has_enc != 0;
    for (int rb = r0 + ty; rb < r1; rb += RG * RP) {
      float dv[RG], hv[RG], pv[RG];
#pragma unroll
      for (int k = 0; k < RG; ++k) {
        const int r = rb + k * RP;
        const bool rv = r < r1;
        dv[k] = rv ? a.dg[(long long)r * a.lddg + c] : 0.f;
        hv[k] = (rv && he) ? a.h2[(long long)r * a.ldh2 + c] : 0.f;
        pv[k] = (rv && hc) ? a.p[(long long)r * a.ldp + c] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < RG; ++k) {
        const int r = rb + k * RP;
        if (r >= r1) break;
        float d = dv[k];
        if (he) {
          sge += d * hv[k];
          sbe += d;
          d *= gec;
        }
        if (hc) {
          sg += d * lrelu(pv[k]);
          sb += d;
          a.dp[(long long)r * a.lddp + c] = d * gc * lrelu_grad(pv[k]);
        }
      }
    }
  }
  if (a.has_enc) {
    sge = lane_rows_sum<CP>(sge, red);
    sbe = lane_rows_sum<CP>(sbe, red);
  }
  sg = lane_rows_sum<CP>(sg, red);
  sb = lane_rows_sum<CP>(sb, red);
  if (threadIdx.x < width) {
    const int stride = (a.has_enc ? 2 * a.wenc : 0) + 2 * a.h;
    float* pp = a.part + (long long)blockIdx.x * stride;
    int o = 0;
    if (a.has_enc) {
      pp[c] = sge * kBnC;
      pp[a.wenc + c] = sbe;
      o = 2 * a.wenc;
    }
    if (c < a.h) {
      pp[o + c] = sg * kBnC;
      pp[o + a.h + c] = sb;
    }
  }
}

// ---------------------------------------------------------------- reduce
#ifndef SND_RED_PL
#define SND_RED_PL 2   // part lanes of a >= 64-part slab of >= kRedWide items (round 5, C2 step on one
                       // box: 0.2220 ms at 2, 0.2228 at 4, 0.2226 at 1; another: 0.2210 at 4 vs 0.2236
                       // at 8, 0.2300 at 16)
#endif
#ifndef SND_RED_PLS
#define SND_RED_PLS 4  // part lanes of a < 64-part partial
#endif
#ifndef SND_RED_PLW
#define SND_RED_PLW 2  // part lanes of a < 64-part slab of >= kRedWide items (C5 and one-graph 32-chunk
                       // weight slabs; round 6: C5 0.3668-0.3694 -> 0.3635-0.3658 ms at 2, 1 alike,
                       // profiles/r06_ab_c5_pack_gcn0_reduce_lanes.txt)
#endif
constexpr long long kRedWide = 2048;
// part lanes of a descriptor (uniform per block): a thread sums nparts / PL parts in a
// dependent chain, so the many-part partials (C4's split-K head / projection slabs, ~1000
// parts) take wider lane groups and more blocks; a 64..255-part partial of few items
// (the per-tile column sums of the BN parameters) keeps 8 lanes, a wide weight slab 2
__host__ __device__ __forceinline__ int red_pl(int nparts, long long items) {
  return nparts >= 1024 ? 64
                        : (nparts >= 256 ? 32 : (nparts >= 64 ? (items >= kRedWide ? SND_RED_PL : 8) : (items >= kRedWide ? SND_RED_PLW : SND_RED_PLS)));
}
struct ReducePack {
  ReduceDesc d[kMaxReduce];
  int bstart[kMaxReduce + 1];   // first block of each descriptor (flattened 1-D grid)
};

template <int NTF> __device__ void finalize_block(const FinalizeArgs& a);

// fin: block 0 computes the loss terms (finalize) instead of a reduction block;
// ADAM: descriptors of ra.mask (this launch's bits) also take their TF1 Adam update
template <bool FIN, bool ADAM>
__global__ void __launch_bounds__(256) reduce_kernel(ReducePack pk, FinalizeArgs fin, ReduceAdam ra) {
  if constexpr (FIN) {
    if (blockIdx.x == 0) { finalize_block<256>(fin); return; }
  }
  const int bid = (int)blockIdx.x - (FIN ? 1 : 0);
  // descriptor of this block: the count of later starts <= bid (bstart is non-decreasing,
  // unused entries hold the total): independent scalar loads, no dependent search chain
  int di = 0;
#pragma unroll
  for (int i = 1; i < kMaxReduce; ++i) di += bid >= pk.bstart[i] ? 1 : 0;
  di = __builtin_amdgcn_readfirstlane(di);
  const ReduceDesc& d = pk.d[di];
  const int bx = bid - pk.bstart[di];
  // bias-corrected step size (snd_adam_tf1's arithmetic), while the slab loads are in flight
  const bool dad = ADAM && ((ra.mask >> di) & 1ull);   // uniform per block
  float lrt = 0.f;
  if (dad) {
    const int st = *ra.stepn;
    lrt = (float)((double)ra.lr * sqrt(1.0 - pow((double)ra.b2, st)) / (1.0 - pow((double)ra.b1, st)));
  }
  __shared__ double red[256];
  const int rows = d.rows > 0 ? d.rows : 1;
  const long long items = (long long)rows * d.len;
  const int PL = red_pl(d.nparts, items);        // part lanes
  const int IPB = 256 / PL;                      // items per block
  const int it = threadIdx.x % IPB, pl = threadIdx.x / IPB;
  const long long j = (long long)bx * IPB + it;
  int r = 0, i = 0;
  double acc = 0.0;
  // the Adam operands (and an accumulated destination) do not depend on the sums: the
  // item's owner lane loads them before the slab loads, one round trip for both
  float pi = 0.f, mi = 0.f, vi = 0.f, prev = 0.f;
  if (j < items) {
    r = (int)(j / d.len);
    i = (int)(j - (long long)r * d.len);
    if (pl == 0) {
      const float* dst = d.dst + (long long)r * d.dst_rs + i;
      if (d.accumulate) prev = *dst;
      if constexpr (ADAM) {
        if (dad) {
          const long long k = dst - ra.gbase;
          pi = ra.p[k]; mi = ra.m[k]; vi = ra.v[k];
        }
      }
    }
    const float* src = d.src + (long long)r * d.src_rs + i;
    int p = pl;
    // 8 loads in flight per round (the 64-part weight slabs at 8 part lanes: one round
    // trip instead of two); the adds stay in part order
    // (16 or 32 loads per round, i.e. 1-2 rounds per thread, measured no faster:
    // profiles/r06_ab_reduce_rounds.txt)
    for (; p + 7 * PL < d.nparts; p += 8 * PL) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(long long)(p + u * PL) * d.stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)v[u];
    }
    for (; p + 3 * PL < d.nparts; p += 4 * PL) {
      const float v0 = src[(long long)p * d.stride];
      const float v1 = src[(long long)(p + PL) * d.stride];
      const float v2 = src[(long long)(p + 2 * PL) * d.stride];
      const float v3 = src[(long long)(p + 3 * PL) * d.stride];
      acc += (double)v0;
      acc += (double)v1;
      acc += (double)v2;
      acc += (double)v3;
    }
    for (; p < d.nparts; p += PL) acc += (double)src[(long long)p * d.stride];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (pl == 0 && j < items) {
    double t = 0.0;
    for (int q = 0; q < PL; ++q) t += red[q * IPB + it];
    float* dst = d.dst + (long long)r * d.dst_rs + i;
    float v = (float)(t * (double)d.scale);
    if (d.accumulate) v += prev;
    *dst = v;
    if constexpr (ADAM) {
      if (dad) {
        const long long k = dst - ra.gbase;
        adam_elem(pi, mi, vi, __fmul_rn(v, 1.f), ra.b1, ra.b2, ra.eps, lrt);
        ra.m[k] = mi;
        ra.v[k] = vi;
        ra.p[k] = pi;
      }
    }
  }
}

// ---------------------------------------------------------------- finalize
// Loss terms from the per-block partials, in fixed order (one workgroup of NTF threads).
template <int NTF>
__device__ __forceinline__ void finalize_block(const FinalizeArgs& a) {
  double v[7] = {0, 0, 0, 0, 0, 0, 0};   // dl, dc, el, tp, kl, ss, sn
#pragma unroll 4
  for (int k = threadIdx.x; k < a.n_zzt; k += NTF) { v[0] += a.zzt_part[2 * k]; v[1] += a.zzt_part[2 * k + 1]; }
#pragma unroll 4
  for (int k = threadIdx.x; k < a.n_edge; k += NTF) { v[2] += a.edge_part[2 * k]; v[3] += a.edge_part[2 * k + 1]; }
#pragma unroll 4
  for (int k = threadIdx.x; k < a.n_kl; k += NTF) v[4] += a.kl_part[k];
#pragma unroll 4
  for (int k = threadIdx.x; k < a.n_s; k += NTF) { v[5] += a.sse_s[k]; v[6] += a.sse_n[k]; }
  __shared__ double sh[NTF / 64][7];
#pragma unroll
  for (int q = 0; q < 7; ++q) v[q] = wave_sum_d(v[q]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) sh[threadIdx.x >> 6][q] = v[q];
  __syncthreads();
  double dl = 0, dc = 0, el = 0, tp = 0, kl = 0, ss = 0, sn = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < NTF / 64; ++w) {
      dl += sh[w][0]; dc += sh[w][1]; el += sh[w][2]; tp += sh[w][3];
      kl += sh[w][4]; ss += sh[w][5]; sn += sh[w][6];
    }
  if (threadIdx.x != 0) return;
  const double rows = (double)a.ngraphs * a.n;
  const double pairs = rows * (double)a.n;
  const double nnz = (double)a.rowptr[(long long)a.ngraphs * a.n];
  const double adj_sum = (double)a.norm * (dl + el + rows * kSoftplusM1);
  const double adj_cost = adj_sum / pairs;                      // optimizer.py:144
  const double correct = pairs - nnz - dc + 2.0 * tp;           // main.py:334
  const double klm = -0.5 * kl / (a.kl_count > 0 ? a.kl_count : rows * a.L);   // optimizer.py:193
  const double spatial = ss / (rows * a.sdim);                  // optimizer.py:153
  const double node = sn / (rows * a.nfeat);                    // optimizer.py:149
  const double cost = adj_cost + node + spatial + (double)a.beta * klm;   // :157,194
  double* L = a.losses;
  L[0] = cost; L[1] = spatial; L[2] = adj_cost; L[3] = node; L[4] = klm;
  L[5] = correct / pairs; L[6] = adj_sum; L[7] = correct;
  if (a.grad_tail)
    for (int k = 0; k < 6; ++k) a.grad_tail[k] = (float)L[k];
  if (a.step) *a.step += 1;
}

constexpr int kFinT = 1024;
__global__ void __launch_bounds__(kFinT) finalize_kernel(FinalizeArgs a) { finalize_block<kFinT>(a); }

// ---------------------------------------------------------------- Adam
__global__ void __launch_bounds__(256) adam_kernel(float* p, const float* g, float* m, float* v,
                                                   long long n, float lr, float b1, float b2,
                                                   float eps, float gscale, const int* step) {
  const int t = *step;
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
  const float lrt = (float)lr_t;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    float pi = p[i], mi = m[i], vi = v[i];
    adam_elem(pi, mi, vi, __fmul_rn(g[i], gscale), b1, b2, eps, lrt);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

}  // namespace

int reparam_blocks(int rows, int L) {
  int b = cdiv((long long)rows * L, 256);
  return b < kReparamGrid ? (b < 1 ? 1 : b) : kReparamGrid;
}
int launch_reparam_fwd(const ReparamFwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(reparam_fwd_kernel, dim3(reparam_blocks(a.rows, a.L)), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("reparam_fwd_kernel");
  return 0;
}
int launch_reparam_bwd(const ReparamBwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3(reparam_blocks(a.rows, a.L)), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("reparam_bwd_kernel");
  return 0;
}

bool small_head_supported(int rows, int gh, int L) {
  return rows >= 1 && rows <= kSmallHeadRows && rows * kSHC <= 256 && gh >= 1 && gh <= kSHK && L >= 1 &&
         2 * L <= kSHL2 && rows * kSHD <= 256;
}
int small_head_fwd_blocks(int L) { return cdiv(L, kSHC); }
int launch_small_head_fwd(const SmallHeadFwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(small_head_supported(a.rows, a.gh, a.L), "small_head: rows <= 16, gh <= 128, 2L <= 256");
  SND_CHECK_ARG(a.hh && a.wms && a.bms && a.ms && a.z && a.kl_part, "small_head_fwd: operands");
  hipLaunchKernelGGL(small_head_fwd_kernel, dim3(small_head_fwd_blocks(a.L)), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("small_head_fwd_kernel");
  return 0;
}
int launch_small_head_bwd(const SmallHeadBwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(small_head_supported(a.rows, a.gh, a.L), "small_head: rows <= 16, gh <= 128, 2L <= 256");
  SND_CHECK_ARG(a.hh && a.wms && a.ms && a.eps && a.dz && a.dms && a.slab && a.dh, "small_head_bwd: operands");
  hipLaunchKernelGGL(small_head_dms_kernel, dim3(cdiv(2 * a.L, kSHN)), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("small_head_dms_kernel");
  hipLaunchKernelGGL(small_head_dh_kernel, dim3(cdiv(a.gh, kSHD)), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("small_head_dh_kernel");
  return 0;
}

int head_blocks(int rows) { return cdiv(rows, kHeadRows); }

int launch_heads(const HeadArgs* h, int nheads, int rows, hipStream_t s) {
  if (nheads < 1 || nheads > 2) { set_error("heads: 1 or 2 heads"); return SND_ERR_ARG; }
  HeadPack pk{};
  for (int i = 0; i < nheads; ++i) {
    if (h[i].cin > kHeadK || h[i].cout > kHeadO) {
      set_error("heads: cin <= %d, cout <= %d", kHeadK, kHeadO);
      return SND_ERR_ARG;
    }
    pk.h[i] = h[i];
  }
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(heads_kernel, dim3(head_blocks(rows), nheads), dim3(256), 0, s, pk, rows);
  SND_LAUNCH_CHECK("heads_kernel");
  return 0;
}

int col_blocks(int rows) { return cdiv(rows, kColRows); }

int launch_dec_bwd(const DecBwdArgs* a, int n, int rows, hipStream_t s) {
  if (n < 1 || n > 2) { set_error("dec_bwd: 1 or 2 descriptors"); return SND_ERR_ARG; }
  DecPack pk{};
  for (int i = 0; i < n; ++i) {
    if (a[i].ncols > 256) { set_error("dec_bwd: ncols %d > 256", a[i].ncols); return SND_ERR_ARG; }
    pk.d[i] = a[i];
  }
  if (rows <= 0) return 0;
  int w = a[0].ncols;
  if (n > 1 && a[1].ncols > w) w = a[1].ncols;
  dim3 grid(col_blocks(rows), n);
  if (w <= 16) hipLaunchKernelGGL(dec_bwd_kernel<16>, grid, dim3(256), 0, s, pk, rows);
  else if (w <= 32) hipLaunchKernelGGL(dec_bwd_kernel<32>, grid, dim3(256), 0, s, pk, rows);
  else if (w <= 64) hipLaunchKernelGGL(dec_bwd_kernel<64>, grid, dim3(256), 0, s, pk, rows);
  else if (w <= 128) hipLaunchKernelGGL(dec_bwd_kernel<128>, grid, dim3(256), 0, s, pk, rows);
  else hipLaunchKernelGGL(dec_bwd_kernel<256>, grid, dim3(256), 0, s, pk, rows);
  SND_LAUNCH_CHECK("dec_bwd_kernel");
  return 0;
}

int launch_enc_bwd(const EncBwdArgs& a, int rows, hipStream_t s) {
  const int width = a.has_enc ? a.wenc : a.h;
  if (width > 256) { set_error("enc_bwd: width %d > 256", width); return SND_ERR_ARG; }
  dim3 grid(col_blocks(rows));
  if (width <= 64) hipLaunchKernelGGL(enc_bwd_kernel<64>, grid, dim3(256), 0, s, a, rows);
  else if (width <= 128) hipLaunchKernelGGL(enc_bwd_kernel<128>, grid, dim3(256), 0, s, a, rows);
  else hipLaunchKernelGGL(enc_bwd_kernel<256>, grid, dim3(256), 0, s, a, rows);
  SND_LAUNCH_CHECK("enc_bwd_kernel");
  return 0;
}

int launch_reduce(const ReduceDesc* d, int n, hipStream_t s, const FinalizeArgs* fin,
                  const ReduceAdam* adam) {
  SND_CHECK_ARG(!adam || (n <= 64 && adam->gbase && adam->p && adam->m && adam->v && adam->stepn),
                "reduce: fused Adam needs <= 64 descriptors and its operands");
  for (int base = 0; base < n || (base == 0 && fin); base += kMaxReduce) {
    const bool last = base + kMaxReduce >= n;
    ReduceAdam ra{};
    if (adam) {
      ra = *adam;
      ra.mask = adam->mask >> base;
      if (n - base < 64) ra.mask &= (1ull << (n - base)) - 1;
    }
    const bool ad = ra.mask != 0;
    ReducePack pk{};
    const int cnt = n - base < kMaxReduce ? n - base : kMaxReduce;
    long long nb = 0;
    for (int i = 0; i < kMaxReduce; ++i) {
      pk.bstart[i] = (int)nb;
      if (i < cnt) {
        pk.d[i] = d[base + i];
        const long long items = (long long)(pk.d[i].rows > 0 ? pk.d[i].rows : 1) * pk.d[i].len;
        const int ipb = 256 / red_pl(pk.d[i].nparts, items);
        nb += (items + ipb - 1) / ipb;
      }
    }
    pk.bstart[kMaxReduce] = (int)nb;
    if (fin && last) {   // the loss terms ride in the last reduction launch
      if (ad) hipLaunchKernelGGL((reduce_kernel<true, true>), dim3((unsigned)nb + 1), dim3(256), 0, s, pk, *fin, ra);
      else hipLaunchKernelGGL((reduce_kernel<true, false>), dim3((unsigned)nb + 1), dim3(256), 0, s, pk, *fin, ra);
    } else {
      if (nb == 0) continue;
      if (ad) hipLaunchKernelGGL((reduce_kernel<false, true>), dim3((unsigned)nb), dim3(256), 0, s, pk, FinalizeArgs{}, ra);
      else hipLaunchKernelGGL((reduce_kernel<false, false>), dim3((unsigned)nb), dim3(256), 0, s, pk, FinalizeArgs{}, ra);
    }
    SND_LAUNCH_CHECK("reduce_kernel");
  }
  return 0;
}

int launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(kFinT), 0, s, a);
  SND_LAUNCH_CHECK("finalize_kernel");
  return 0;
}

}  // namespace snd

using namespace snd;

extern "C" int snd_reparam_kl_blocks(int rows, int latent) { return reparam_blocks(rows, latent); }
extern "C" int snd_sigmoid_mse_blocks(int rows) { return head_blocks(rows); }

extern "C" int snd_sigmoid_mse(const float* u, int ldu, int rows, int cin, const float* w,
                               const float* b, int cout, const float* target, int ldt,
                               double* sse, float* yhat, float* du, int lddu, float* dw,
                               float* db, void* workspace, size_t workspace_bytes,
                               snd_stream_t stream) {
  SND_CHECK_ARG(u && w && b && target && sse && du && dw && db, "snd_sigmoid_mse: null operand");
  const int nb = head_blocks(rows);
  const size_t need = (size_t)nb * (cin * cout + cout) * sizeof(float);
  SND_CHECK_ARG(workspace && workspace_bytes >= need, "snd_sigmoid_mse: workspace %zu < %zu",
                workspace_bytes, need);
  hipStream_t s = (hipStream_t)stream;
  HeadArgs h{u, ldu, cin, w, b, cout, target, ldt, (float)rows * cout, yhat, du, lddu,
             (float*)workspace, sse};
  SND_TRY(launch_heads(&h, 1, rows, s));
  const int stride = cin * cout + cout;
  ReduceDesc d[2] = {{(const float*)workspace, dw, nb, cin * cout, stride, 1.f, 1},
                     {(const float*)workspace + cin * cout, db, nb, cout, stride, 1.f, 1}};
  return launch_reduce(d, 2, s);
}

extern "C" int snd_reparam_kl(const float* ms, int ldms, int rows, int latent,
                              const float* eps, unsigned long long seed,
                              const int* step_counter, float* eps_out, float* z,
                              double* kl_sum, snd_stream_t stream) {
  SND_CHECK_ARG(ms && z && kl_sum && rows >= 0 && latent > 0 && latent <= 256,
                "snd_reparam_kl: bad args (latent in 1..256)");
  // kl_sum receives one partial per block; callers sum reparam_blocks() values.
  ReparamFwdArgs a{ms, ldms, rows, latent, eps, seed, step_counter, eps_out, z, kl_sum};
  return launch_reparam_fwd(a, (hipStream_t)stream);
}

extern "C" int snd_adam_tf1_ranges(float* param, const float* grad, float* m, float* v,
                                   const long long* offsets, const long long* counts, int n_ranges,
                                   float lr, float beta1, float beta2, float eps, float grad_scale,
                                   const int* step_counter, snd_stream_t stream) {
  SND_CHECK_ARG(param && grad && m && v && step_counter && offsets && counts && n_ranges >= 0,
                "snd_adam_tf1_ranges: bad args");
  if (n_ranges == 0) return 0;
  bool vec = n_ranges <= kAdamMaxRanges &&
             ((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
  for (int k = 0; k < n_ranges && vec; ++k) vec = offsets[k] % 4 == 0 && counts[k] % 4 == 0;
  if (vec)
    return launch_adam_ranges(param, grad, m, v, offsets, counts, n_ranges, lr, beta1,
                              beta2, eps, grad_scale, step_counter, (hipStream_t)stream);
  for (int k = 0; k < n_ranges; ++k)   // unaligned ranges: one launch each
    SND_TRY(snd_adam_tf1(param + offsets[k], grad + offsets[k], m + offsets[k], v + offsets[k], counts[k],
                         lr, beta1, beta2, eps, grad_scale, step_counter, stream));
  return 0;
}

extern "C" int snd_adam_tf1(float* param, const float* grad, float* m, float* v, long long n,
                            float lr, float beta1, float beta2, float eps, float grad_scale,
                            const int* step_counter, snd_stream_t stream) {
  SND_CHECK_ARG(param && grad && m && v && step_counter && n >= 0, "snd_adam_tf1: bad args");
  if (n % 4 == 0 && ((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0)
    return launch_adam_vec(param, grad, m, v, n, lr, beta1, beta2, eps, grad_scale, step_counter,
                           (hipStream_t)stream);
  int blocks = cdiv(n, 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, param, grad,
                     m, v, n, lr, beta1, beta2, eps, grad_scale, step_counter);
  SND_LAUNCH_CHECK("adam_kernel");
  return 0;
}
