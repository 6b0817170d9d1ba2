// bf16 GraphConvolution SpMM (layers.py:120-123, out = A @ h) streamed through a
// sliding window of h rows in LDS.
//
// Why a window.  Under the per-graph reverse Cuthill-McKee schedule
// (data.locality_order) a row's neighbours sit within +-beta schedule positions
// of it (beta ~ 180-260 at N = 4096, ~350 at N = 16384, SURVEY §8a RGGs).  A
// workgroup walks its graph's positions in steps of 128 rows and keeps the h rows
// of positions [p - beta, p + 127 + beta] in a 1096-row LDS ring (bf16, 137 KB at
// width 64): every h row enters the ring ONCE, by LDS-DMA, two steps before the
// first row that needs it.  HBM traffic is the compulsory bytes: h once, out once,
// the plan's per-position metadata and u16 ring slots (2 B per nonzero instead
// of the CSR's 4).  The register-gather kernel re-reads every neighbour row from
// L2 (15.5 x the output bytes) and the row-tile kernel re-stages each tile's
// neighbour set (3.4 rows per row).
//
// Plan (snd_vae_amd/data.py window_plan, built once per batch like the CSR):
//   meta[q]   position q's row: (start8 << 6) | degree, start8 = its slot list's
//             offset in 16-byte units (lists padded to 8 entries)
//   slots[]   u16 ring slot (neighbour position % 1096) of every neighbour, in
//             colidx order: the fp32 sums are the register kernel's, in the same
//             order, so the result is bitwise equal to snd_csr_spmm_bf16; each
//             list is padded with the zero row's slot (1096) to a multiple of 8
//             and to the largest degree of its wavefront's 8 rows (<= 32)
//   rows[q]   the row whose sums position q computes: inside every aligned
//             128-position block the rows (and their meta) are listed by degree,
//             descending, so the 8 rows of a wave have near-equal degrees and the
//             wave's neighbour loop stops at their common maximum
//   order[q]  the row at position q (the schedule: the h row the window holds
//             at ring slot q % 1096; outputs stay at their rows)
//
// Per step s (positions P0 + 128 s ..; wave w owns 8 rows, 8 lanes per row, a
// lane 8 columns).  Everything a step consumes arrives by LDS-DMA, issued in
// inline asm: hipcc tracks a builtin LDS-DMA as a pending LDS write and drains
// vmcnt(0) before the next ds_read (and __syncthreads()' fence drains it too),
// which would serialise the prefetch; here the only vector-memory waits are the
// counted ones below, before a raw s_barrier.  Per wave, in issue order:
//   b  ds_read: start8 of the rows of step s+1, row ids of this step's window piece
//   c  DMA index(s+3): meta / row id of the rows of step s+3, row ids of the
//      window piece of step s+3 (24 lanes x 4 B)
//   d  DMA slot lists of step s+1 (32 lanes x 16 B: 8 rows x 32 u16)
//   e  DMA window piece of step s: positions (hi(s+1), hi(s+2)], 8 rows x 128 B
//   f  vmcnt(5): slots(s) are in (issued at step s-1, followed by e(s-1), the
//      store of s-1 and c/d/e of s), and with them every older DMA: index(s+2)
//      and this step's window (e of step s-2)
//   barrier; sum from the ring; store; barrier (the next step's DMAs overwrite
//   what this step read).  With beta8 <= 288 the step is instead: vmcnt(2)
//   (slots(s)); barrier; b-e; sum; store -- one barrier per step.
// LDS (one array): ring 1096 rows x 128 B, two zero rows (the slots of list entries
// past a row's degree),
// 4 index blocks (16 waves x [meta 8 | row 8 | piece 8]), 2 slot-list buffers
// (16 waves x 512 B) = 163072 B.  The window of step s+1
// (e of step s-1) is in flight while step s sums, and e(s) overwrites ring rows
// 1096 below hi(s+2) + 8 x 15, which no later step reads while 2 beta < 712.
#include "snd_spmm.hpp"

#include <algorithm>

namespace snd {
int debug_flags();
namespace {

// neighbour reads issued before a chunk's adds (round 5, 256-graph batch, one box,
// alternating processes: GK 2 / 4 / 8 = 88.7-90.4 / 85.1-87.6 / 87.4-91.7 us)
constexpr int kWinGK = 4;
constexpr int WT = 1024;       // threads: 16 waves x 8 rows
constexpr int RR = 1096;       // ring rows
constexpr int STEP = 128;      // rows per step
constexpr int WIDTH = 64;      // bf16 columns (128-byte rows)
constexpr int ZROW = RR;       // the zero rows' slots: RR (even) and RR + 1 (odd, pair plans)
constexpr int OFF_IDX = (RR + 2) * WIDTH * 2;       // 4 x 1536 B index blocks
constexpr int OFF_SL = OFF_IDX + 4 * 16 * 96;       // 2 x 8192 B slot-list buffers
constexpr int LDS_BYTES = OFF_SL + 2 * 16 * 512;

typedef __attribute__((address_space(3))) void* lptr_t;

struct WinArgs {
  const int* meta;
  const unsigned short* slots;
  const int* rows;
  const int* order;
  const __bf16* h;
  int ldh;
  __bf16* out;
  int ldo;
  int n, spg, seg, beta8;
  int dbg;   // snd_debug_set >> 24.  A/B (both builds): 32 two barriers per step at any beta,
             // 64 wave w sums group w (no SIMD balancing).  Measurement build only
             // (MEAS, any of bits 1-4 set): 1 no sums, 2 no window DMA, 4 no slot DMA
};

// fp32 sums without unpacking: v_dot2c_f32_bf16 with (1, 0) / (0, 1) adds the low /
// high bf16 of a word to an fp32 accumulator (x * 1 and y * 0 are exact, one rounding),
// 8 VALU per neighbour instead of the 12 of shift / mask + add
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void acc8_dot(float (&f)[8], const uint4 d) {
  const unsigned v[4] = {d.x, d.y, d.z, d.w};
  // (1, 0) and (0, 1) through SGPRs: hipcc encodes the bf16 pair (1, 0) as the inline
  // constant 1.0, which the hardware reads as the fp32 word 0x3F800000 = (0, 1)
  unsigned lo1u, hi1u;
  asm volatile("s_mov_b32 %0, 0x3f80" : "=s"(lo1u));
  asm volatile("s_mov_b32 %0, 0x3f800000" : "=s"(hi1u));
  const bf16x2_t lo1 = __builtin_bit_cast(bf16x2_t, lo1u);
  const bf16x2_t hi1 = __builtin_bit_cast(bf16x2_t, hi1u);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x2_t x = __builtin_bit_cast(bf16x2_t, v[j]);
    f[2 * j] = __builtin_amdgcn_fdot2_f32_bf16(x, lo1, f[2 * j], false);
    f[2 * j + 1] = __builtin_amdgcn_fdot2_f32_bf16(x, hi1, f[2 * j + 1], false);
  }
}

// LDS byte address of ring slot (the low or high u16 of w) for a lane at column
// offset `base`: slot * 128 + base in one v_mad_u32_u16 (op_sel picks the half).
// Entries past a row's degree hold the zero row's slot (the plan pads every list
// to its wavefront group's largest degree), so no per-entry compare or select.
__device__ __forceinline__ unsigned slot_addr(unsigned w, int hi, unsigned base) {
  unsigned r;
  if (hi) asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(w), "s"(WIDTH * 2), "v"(base));
  else asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(w), "s"(WIDTH * 2), "v"(base));
  return r;
}

constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

// global -> LDS DMA of `bytes` (4 or 16) per active lane to the wave-uniform LDS
// address `dst` + 4/16 x lane (the compiler does not see it: vmcnt counted by hand)
template <int BYTES>
__device__ __forceinline__ void glds(const void* src, unsigned dst) {
  unsigned keep;
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int GK, bool MEAS>
__global__ void __launch_bounds__(WT) spmm_win_kernel(WinArgs a) {
  // the phase-skip bits exist in the measurement instantiation only
  const int skip = MEAS ? (a.dbg & 7) : 0;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const unsigned lds0 = (unsigned)(uintptr_t)(lptr_t)lds;   // LDS byte address of lds[0]
  const int g = blockIdx.x / a.spg, sg = blockIdx.x - g * a.spg;
  const int gb = g * a.n;                         // graph's first global position / row
  const int P0 = sg * a.seg, P1 = min(a.n, P0 + a.seg);
  if (P0 >= P1) return;                           // uniform per workgroup
  const int nsteps = (P1 - P0 + STEP - 1) / STEP;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r8 = lane >> 3, l8 = lane & 7;
  const int Q0 = max(0, P0 - a.beta8);            // first window position (8-aligned)
  const int Q1 = min(a.n, P1 + a.beta8);          // window end (exclusive)
  // last window position step s reads
  auto hi = [&](int s) { return min(P0 + STEP * s + STEP - 1 + a.beta8, Q1 - 1); };
  // the 8-row group this wave sums: groups are listed by degree (descending) inside
  // each step, and wave w runs on SIMD w % 4, so the snake {s, 7 - s, 8 + s, 15 - s}
  // gives every SIMD the same share of the step's neighbours (w % 4 = s; dbg 64: group w)
  const int sm = w & 3, wk = w >> 2;
  const int grp = (a.dbg & 64) ? w : (wk == 0 ? sm : wk == 1 ? 7 - sm : wk == 2 ? 8 + sm : 15 - sm);
  // graph-local position of row j (0..7) of this wave at step s (clamped: duplicates are benign)
  auto rpos = [&](int s, int j) { return min(P0 + STEP * s + 8 * grp + j, P1 - 1); };
  // first position of the 8-row piece this wave DMAs at step s (8-aligned; past the
  // window end it lands in dead ring rows)
  auto dpiece = [&](int s) { return ((hi(s + 1) + 8) & ~7) + 8 * w; };
  auto idx_blk = [&](int s) { return OFF_IDX + (s & 3) * (16 * 96) + 96 * w; };
  auto sl_buf = [&](int s) { return OFF_SL + (s & 1) * (16 * 512) + 512 * w; };

  // c: index(s) -> lanes 0-7 meta, 8-15 row id, 16-23 row id of the window piece of step s
  auto dma_index = [&](int s) {
    if (lane < 24) {
      const int j = lane & 7;
      const int* src = lane < 8    ? a.meta + gb + rpos(s, j)
                       : lane < 16 ? a.rows + gb + rpos(s, j)
                                   : a.order + gb + min(dpiece(s) + j, Q1 - 1);
      glds<4>(src, __builtin_amdgcn_readfirstlane(lds0 + idx_blk(s)));
    }
  };
  // d: slot lists of step s (start8 per row from index(s))
  auto dma_slots = [&](int s, int start8) {
    if (lane < 32) {
      const unsigned short* src = a.slots + (long long)start8 * 8 + 8 * (lane & 3);
      glds<16>(src, __builtin_amdgcn_readfirstlane(lds0 + sl_buf(s)));
    }
  };
  // e: one 8-row piece of the window (row ids from index(s))
  auto dma_piece = [&](int p0, int row) {
    const __bf16* src = a.h + (long long)row * a.ldh + 8 * l8;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + (p0 % RR) * (WIDTH * 2));
    // allocating loads: non-temporal window DMA measured within noise on the 256-graph
    // batch and 1.5-4 us slower in the C2 step, where h was just written and still sits
    // in L2 / the Infinity Cache (retired A/B)
    glds<16>(src, dst);
  };
  auto lds_i32 = [&](int off) { return *reinterpret_cast<const int*>(lds + off); };

  // ---- prologue: zero row, index(0..2), slots(0), window [Q0, hi(1)]
  if (tid < 2 * WIDTH * 2 / 16)
    reinterpret_cast<uint4*>(lds + RR * WIDTH * 2)[tid] = make_uint4(0u, 0u, 0u, 0u);
  dma_index(0);
  dma_index(1);
  dma_index(2);
  {
    const int np = (hi(1) - Q0) / 8 + 1;          // window pieces
    for (int j = w; j < np; j += WT / 64) {
      const int p0 = Q0 + 8 * j;
      dma_piece(p0, a.order[gb + min(p0 + r8, Q1 - 1)]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  dma_slots(0, lds_i32(idx_blk(0) + 4 * (lane >> 2)) >> 6);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  const unsigned base = (unsigned)(l8 * 16);
  // b-e: the step's reads of index(s) / index(s+1) and its DMAs
  auto issue = [&](int s) {
    const int st1 = lds_i32(idx_blk(s + 1) + 4 * (lane >> 2)) >> 6;
    const int prow = lds_i32(idx_blk(s) + 64 + 4 * r8);
    dma_index(s + 3);
    if (!(skip & 4)) dma_slots(s + 1, st1);
    if (!(skip & 2)) dma_piece(dpiece(s), prow);
  };
  // One barrier per step when the window leaves room: the DMAs of step s are issued
  // after its barrier (every wave has finished step s-1, the last reader of the
  // index block, slot buffer and ring rows they overwrite; the ring rows e(s)
  // overwrites lie below every position step s reads while 2 beta8 < 592).
  const bool one = a.beta8 <= 288 && !(a.dbg & 32);
  for (int s = 0; s < nsteps; ++s) {
    if (one) {
      // slots(s) (d of step s-1, followed by e(s-1) and the store of s-1) and every
      // older DMA are in
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(2));
      raw_barrier();
      issue(s);
    } else {
      issue(s);
      // f: slots(s), index(s+2) and this step's window are in
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(5));
      raw_barrier();
    }

    {
    // sum the row's neighbours from the ring (colidx order, fp32).  The wave's 8 rows
      // are one degree-sorted group and every list is padded with the zero row to the
      // group's largest degree (exact +0 adds past a row's own degree): a chunk of GK
      // reads is issued before the first add; the wave leaves the loop after the
      // group's largest degree.  (Reads of the next chunk issued before the adds of
      // the current one measured slower: 101 vs 96 us.)
      const int m0 = lds_i32(idx_blk(s) + 4 * r8);
      const int row0 = lds_i32(idx_blk(s) + 32 + 4 * r8);
      const int deg = m0 & 63;
      const uint4* slp = reinterpret_cast<const uint4*>(lds + sl_buf(s) + 64 * r8);
      const uint4 sl[4] = {slp[0], slp[1], slp[2], slp[3]};
      const unsigned sv[16] = {sl[0].x, sl[0].y, sl[0].z, sl[0].w, sl[1].x, sl[1].y, sl[1].z, sl[1].w,
                               sl[2].x, sl[2].y, sl[2].z, sl[2].w, sl[3].x, sl[3].y, sl[3].z, sl[3].w};
      float f[8];
  #pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
  #pragma unroll
      for (int k0 = 0; k0 < 32; k0 += GK) {
        if (!__builtin_amdgcn_ballot_w64(deg > k0) || (skip & 1)) break;
        uint4 d[GK];
  #pragma unroll
        for (int j = 0; j < GK; ++j) {
          const int k = k0 + j;
          d[j] = *reinterpret_cast<const uint4*>(lds + slot_addr(sv[k >> 1], k & 1, base));
        }
  #pragma unroll
        for (int j = 0; j < GK; ++j) {
          acc8_dot(f, d[j]);
        }
      }
      if (__builtin_amdgcn_ballot_w64(deg > 32)) {   // rows past 32 neighbours (rare)
        const int k0 = (m0 >> 6) * 8;
        for (int k = 32; k < deg; ++k) {
          const unsigned slot = a.slots[k0 + k];
          const uint4 dv = *reinterpret_cast<const uint4*>(lds + slot * (WIDTH * 2) + base);
          acc8_dot(f, dv);
        }
      }
      bf16x8 o;
  #pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (__bf16)f[j];
      // (non-temporal output stores measured no faster: retired A/B)
      *reinterpret_cast<bf16x8*>(a.out + (long long)row0 * a.ldo + 8 * l8) = o;
    }

    // every wave's LDS reads of this step are done (their values were consumed)
    // before any wave's next DMA overwrites ring rows, index blocks or slot lists
    if (!one) raw_barrier();
  }
}

}  // namespace

int spmm_win_max_beta() { return 352; }   // 8-aligned, 2 beta < RR - 3 STEP (712)

}  // namespace snd

using namespace snd;

namespace snd {
int launch_spmm_window(const SpmmWinArgs& w, hipStream_t st) {
  SND_CHECK_ARG(w.meta && w.slots && w.rows && w.order && w.h && w.out, "snd_csr_spmm_bf16_window: null operand");
  SND_CHECK_ARG(w.width == WIDTH, "snd_csr_spmm_bf16_window: width %d (the ring holds 64-column rows)", w.width);
  SND_CHECK_ARG(w.n_per_graph > 0 && w.n_graphs > 0 && (long long)w.n_per_graph * w.n_graphs == w.n_rows,
                "snd_csr_spmm_bf16_window: n_rows != n_per_graph * n_graphs");
  SND_CHECK_ARG(w.ldh % 8 == 0 && w.ldo % 8 == 0 && w.ldh >= w.width && w.ldo >= w.width,
                "snd_csr_spmm_bf16_window: ldh / ldo must be multiples of 8 >= width");
  const int beta8 = (w.beta + 7) & ~7;
  SND_CHECK_ARG(w.beta >= 0 && beta8 <= spmm_win_max_beta() && (long long)w.n_rows < (1LL << 31),
                "snd_csr_spmm_bf16_window: beta %d exceeds the ring (<= %d)", w.beta, spmm_win_max_beta());
  // segments: about 256 workgroups in all, at least one step each
  const int steps = cdiv(w.n_per_graph, STEP);
  const int spg = std::max(1, std::min(steps, cdiv(256, w.n_graphs)));
  const int seg = cdiv(steps, spg) * STEP;
  WinArgs a{w.meta, w.slots, w.rows, w.order, reinterpret_cast<const __bf16*>(w.h), w.ldh,
            reinterpret_cast<__bf16*>(w.out), w.ldo, w.n_per_graph, cdiv(w.n_per_graph, seg), seg, beta8,
            debug_flags() >> 24};
  if (a.dbg & 7) hipLaunchKernelGGL((spmm_win_kernel<kWinGK, true>), dim3(w.n_graphs * a.spg), dim3(WT), 0, st, a);
  else hipLaunchKernelGGL((spmm_win_kernel<kWinGK, false>), dim3(w.n_graphs * a.spg), dim3(WT), 0, st, a);
  SND_LAUNCH_CHECK("spmm_win_kernel");
  return 0;
}
}  // namespace snd

extern "C" int snd_csr_spmm_bf16_window(const int* meta, const uint16_t* slots, const int* rows,
                                        const int* order,
                                        int n_rows, int n_per_graph, int n_graphs, int beta,
                                        const void* h, int ldh, int width, void* out, int ldo,
                                        snd_stream_t stream) {
  SpmmWinArgs w{meta, slots, rows, order, beta, n_rows, n_per_graph, n_graphs, h, ldh, width, out, ldo};
  return launch_spmm_window(w, (hipStream_t)stream);
}
