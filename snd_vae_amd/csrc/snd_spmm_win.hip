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
// past a row's degree; the pair plans pad the odd side with the second),
// 4 index blocks (16 waves x [meta 8 | row 8 | piece 8]), 2 slot-list buffers
// (16 waves x 512 B) = 163072 B.  The window of step s+1
// (e of step s-1) is in flight while step s sums, and e(s) overwrites ring rows
// 1096 below hi(s+2) + 8 x 15, which no later step reads while 2 beta < 712.
#include "snd_spmm.hpp"

#include <algorithm>

namespace snd {
int debug_flags();
namespace {

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
  int dbg;   // measurement only (snd_debug_set >> 16): 1 no sums, 2 no window DMA, 4 no slot DMA,
             // 8 neighbour groups of 8 (default 4), 16 shift/and unpack + packed adds (default dot2),
             // 32 two barriers per step at any beta, 64 the MFMA sums (default: VALU, 8 lanes per row)
};

__device__ __forceinline__ void acc8(float (&f)[8], const uint4 d) {
  const unsigned v[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] += __uint_as_float(v[j] << 16);
    f[2 * j + 1] += __uint_as_float(v[j] & 0xFFFF0000u);
  }
}

// the same fp32 sums without unpacking: v_dot2c_f32_bf16 with (1, 0) / (0, 1) adds
// the low / high bf16 of a word to an fp32 accumulator (x * 1 and y * 0 are exact,
// one rounding: the add of acc8), 8 VALU per neighbour instead of 12
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

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

// MF: the sums on MFMA (see the MF block of the step loop); the ring rows are then
// stored with their 32-byte segments XORed by (slot >> 1) & 3.  Measured slower than
// the VALU sums (105.6 vs 94.0 us on the 256-graph batch, 1 of 67 M outputs 1 bf16 ulp
// apart): twice the LDS instructions (8-byte transposed reads), bank conflicts 40 % of
// LDS-active cycles (a 32-lane half's 8 ring rows fall on 8 segment positions at
// random), and ~10 VALU per MFMA of address arithmetic.  Kept behind debug bit 64 << 16.
template <int GK, bool DOT, bool MF, bool PR = false>
__global__ void __launch_bounds__(WT) spmm_win_kernel(WinArgs a) {
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
  // graph-local position of row j (0..7) of this wave at step s (clamped: duplicates are benign)
  auto rpos = [&](int s, int j) { return min(P0 + STEP * s + 8 * w + j, P1 - 1); };
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
    // MF: ring slot p0 % RR + r8 holds its segment sigma at sigma ^ ((slot >> 1) & 3)
    const int ch16 = MF ? (l8 ^ ((((p0 % RR) + r8) >> 1 & 3) << 1)) : l8;
    const __bf16* src = a.h + (long long)row * a.ldh + 8 * ch16;
    glds<16>(src, __builtin_amdgcn_readfirstlane(lds0 + (p0 % RR) * (WIDTH * 2)));
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
  // MF: lane (gq, li) holds B[k = 8 gq + e][n = li] = 1 iff k >> 1 == n (k = 2 n + t)
  bf16x8 bsel;
  {
    const int dd = (lane & 15) - 4 * (lane >> 4);
    const unsigned one2 = 0x3F803F80u;
    const uint4 bw = make_uint4(dd == 0 ? one2 : 0u, dd == 1 ? one2 : 0u, dd == 2 ? one2 : 0u, dd == 3 ? one2 : 0u);
    bsel = __builtin_bit_cast(bf16x8, bw);
  }
  // b-e: the step's reads of index(s) / index(s+1) and its DMAs
  auto issue = [&](int s) {
    const int st1 = lds_i32(idx_blk(s + 1) + 4 * (lane >> 2)) >> 6;
    const int prow = lds_i32(idx_blk(s) + 64 + 4 * r8);
    dma_index(s + 3);
    if (!(a.dbg & 4)) dma_slots(s + 1, st1);
    if (!(a.dbg & 2)) dma_piece(dpiece(s), prow);
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

    if constexpr (PR) {
      // Pair sums (plan: data.window_plan_pairs).  The wave sums its 8 rows two at a
      // time, each row over rounds of 4 neighbours: 32-lane half h takes the round's
      // pair h = (A, B) (an even and an odd ring slot where the row allows: the two
      // 128-byte rows cover the 64 banks once), its 16-lane group g1 columns
      // 32 g1 .. 32 g1 + 31.  ds_read_b64_tr_b16: lane quad qd supplies row A or B
      // (qd & 1) at column piece (qd >> 1) + 2 g1; lane i of the group receives
      // (A[c], B[c]) and (A[c + 16], B[c + 16]), c = 32 g1 + i, and one v_dot2c with
      // (1, 1) adds both neighbours: 3 VALU (1 address + 2 dot2c) per 4 neighbours x
      // 64 columns.  The halves' partial sums meet in one v_permlane32_swap.
      const int hh = lane >> 5, g1 = (lane >> 4) & 1, qd = (lane >> 2) & 3;
      const int cls = 2 * hh + (qd & 1);
      const unsigned K = 32u * (unsigned)((qd >> 1) + 2 * g1) + 8u * (unsigned)(lane & 3);
      const int col = 32 * g1 + 16 * hh + (lane & 15);
      unsigned one2u;
      asm volatile("s_mov_b32 %0, 0x3f803f80" : "=s"(one2u));
      auto tr = [&](unsigned off) {
        const v4s_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(lds + off));
        return __builtin_bit_cast(uint2, v);
      };
      // VOP3P v_dot2_f32_bf16 (untied accumulator): the builtin picks v_dot2c, whose
      // tied accumulator cost one v_mov per add at every round-chunk join
      auto add2 = [&](float& c0, float& c1, uint2 v) {
        asm("v_dot2_f32_bf16 %0, %1, %2, %3" : "=v"(c0) : "v"(v.x), "s"(one2u), "v"(c0));
        asm("v_dot2_f32_bf16 %0, %1, %2, %3" : "=v"(c1) : "v"(v.y), "s"(one2u), "v"(c1));
      };
      // The wave's 8 rows go through the rounds together (rows are listed by degree,
      // descending, so row 0 bounds the round count; past a row's own rounds its
      // block holds zero rows), two rounds per chunk: 16 transposed reads in flight.
      const int blk = idx_blk(s);
      const int deg0 = __builtin_amdgcn_readfirstlane(lds_i32(blk)) & 63;
      const int nr = (a.dbg & 1) ? 0 : min((deg0 + 3) >> 2, 8);
      unsigned wv[8][4];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4 t = *reinterpret_cast<const uint4*>(lds + sl_buf(s) + 64 * j + 16 * cls);
        wv[j][0] = t.x; wv[j][1] = t.y; wv[j][2] = t.z; wv[j][3] = t.w;
      }
      // all 32 slot words in registers before the rounds (no LDS round trip per chunk)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(wv[j][0]), "v"(wv[j][1]), "v"(wv[j][2]), "v"(wv[j][3]));
      float c0[8], c1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { c0[j] = 0.f; c1[j] = 0.f; }
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        if (r < nr) {
          uint2 x[8], y[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            x[j] = tr(slot_addr(wv[j][r >> 1], 0, K));
            y[j] = tr(slot_addr(wv[j][r >> 1], 1, K));
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) add2(c0[j], c1[j], x[j]);
#pragma unroll
          for (int j = 0; j < 8; ++j) add2(c0[j], c1[j], y[j]);
        }
      }
      // rounds past 8 (degree > 32, rare): entries 32 + 4 (r - 8) + class, from HBM
      if (deg0 > 32 && !(a.dbg & 1)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int mj = __builtin_amdgcn_readfirstlane(lds_i32(blk + 4 * j));
          const int nrj = ((mj & 63) + 3) >> 2;
          const unsigned short* e = a.slots + (long long)(mj >> 6) * 8 + 32 + cls;
          for (int r = 8; r < nrj; ++r) add2(c0[j], c1[j], tr(e[4 * (r - 8)] * (WIDTH * 2) + K));
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const auto f = __builtin_amdgcn_permlane32_swap(__float_as_uint(c0[j]), __float_as_uint(c1[j]), false, false);
        const int row = lds_i32(blk + 32 + 4 * j);
        a.out[(long long)row * a.ldo + col] = (__bf16)(__uint_as_float(f[0]) + __uint_as_float(f[1]));
      }
    } else if constexpr (MF) {
      // Sums on v_mfma_f32_16x16x32_bf16 (wave = 16 degree-sorted rows x 32 columns):
      //   D[m = column][n = row] += A[m][k] B[k][n],  k = 2 n + t (neighbour 2 j + t of row n)
      // A: ds_read_b64_tr_b16 delivers to lane (gq, li) column li of four ring rows whose
      //    addresses lanes 4 q + p of its 16-lane group supply -- two reads give the 8 k of
      //    k-block gq: neighbours 2 j, 2 j + 1 of rows 4 gq + 0..3 of the group
      // B: the constant 0/1 segment matrix (k -> its row), held in registers
      // The plan pads every list (zero row) to the group's largest degree, so all 16
      // rows run the same rounds; D accumulates over rounds in fp32 (products exact).
      const int rg = w >> 1, chh = w & 1;
      const int gq = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3, par = q & 1;
      const int r1 = 16 * rg + 4 * gq + (q >> 1);           // step-local rows of the two reads
      auto slw = [&](int r) {
        return reinterpret_cast<const uint4*>(lds + OFF_SL + (s & 1) * (16 * 512) + 512 * (r >> 3) + 64 * (r & 7));
      };
      const uint4* s1p = slw(r1);
      const uint4* s2p = slw(r1 + 2);
      const uint4 u0 = s1p[0], u1 = s1p[1], u2 = s1p[2], u3 = s1p[3];
      const uint4 v0 = s2p[0], v1 = s2p[1], v2 = s2p[2], v3 = s2p[3];
      const unsigned w1[16] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w,
                               u2.x, u2.y, u2.z, u2.w, u3.x, u3.y, u3.z, u3.w};
      const unsigned w2[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                               v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
      const int blk = OFF_IDX + (s & 3) * (16 * 96);
      const int gdeg = __builtin_amdgcn_readfirstlane(lds_i32(blk + 96 * (2 * rg)) & 63);
      const int nr = (a.dbg & 1) ? 0 : (min(gdeg, 32) + 1) >> 1;
      const unsigned K = ((unsigned)chh << 6) | ((unsigned)p4 << 3);
      const unsigned sh = 16u * (unsigned)par;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      auto addr = [&](unsigned sl) { return (sl << 7) | (((sl << 4) & 0x60u) ^ K); };
      auto tr = [&](unsigned off) {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(lds + off));
      };
      auto round = [&](unsigned sa, unsigned sb) {
        const unsigned a0 = addr(sa), b0 = addr(sb);
        const v4s_t ra0 = tr(a0), rb0 = tr(b0), ra1 = tr(a0 ^ 32u), rb1 = tr(b0 ^ 32u);
        const bf16x8 A0 = __builtin_bit_cast(bf16x8, (v8s_t)__builtin_shufflevector(ra0, rb0, 0, 1, 2, 3, 4, 5, 6, 7));
        const bf16x8 A1 = __builtin_bit_cast(bf16x8, (v8s_t)__builtin_shufflevector(ra1, rb1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, bsel, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, bsel, acc1, 0, 0, 0);
      };
      // rounds in pairs (lists are padded to 8 entries = 4 rounds): one uniform branch
      // per pair, the pair's 8 transposed reads issued before its 4 MFMAs
#pragma unroll
      for (int jr = 0; jr < 16; jr += 2) {
        if (jr < nr) {
          round(__builtin_amdgcn_ubfe(w1[jr], sh, 16), __builtin_amdgcn_ubfe(w2[jr], sh, 16));
          round(__builtin_amdgcn_ubfe(w1[jr + 1], sh, 16), __builtin_amdgcn_ubfe(w2[jr + 1], sh, 16));
        }
      }
      if (gdeg > 32) {   // rows past 32 neighbours (rare): entries from the plan in HBM
        const int m1 = lds_i32(blk + 96 * (r1 >> 3) + 4 * (r1 & 7));
        const int m2 = lds_i32(blk + 96 * ((r1 + 2) >> 3) + 4 * ((r1 + 2) & 7));
        for (int jr = 16; 2 * jr < gdeg; ++jr) {
          const int k = 2 * jr + par;
          const unsigned sa = k < (m1 & 63) ? (unsigned)a.slots[(long long)(m1 >> 6) * 8 + k] : (unsigned)ZROW;
          const unsigned sb = k < (m2 & 63) ? (unsigned)a.slots[(long long)(m2 >> 6) * 8 + k] : (unsigned)ZROW;
          round(sa, sb);
        }
      }
      // lane (gq, li): columns 32 chh + 16 cb + 4 gq + 0..3 of the group's row li
      const int orow = lds_i32(blk + 96 * (2 * rg + (li >> 3)) + 32 + 4 * (li & 7));
      __bf16* op = a.out + (long long)orow * a.ldo + 32 * chh + 4 * gq;
      bf16x4 o0, o1;
#pragma unroll
      for (int e = 0; e < 4; ++e) { o0[e] = (__bf16)acc0[e]; o1[e] = (__bf16)acc1[e]; }
      *reinterpret_cast<bf16x4*>(op) = o0;
      *reinterpret_cast<bf16x4*>(op + 16) = o1;
    } else {
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
        if (!__builtin_amdgcn_ballot_w64(deg > k0) || (a.dbg & 1)) break;
        uint4 d[GK];
  #pragma unroll
        for (int j = 0; j < GK; ++j) {
          const int k = k0 + j;
          d[j] = *reinterpret_cast<const uint4*>(lds + slot_addr(sv[k >> 1], k & 1, base));
        }
  #pragma unroll
        for (int j = 0; j < GK; ++j) {
          if constexpr (DOT) acc8_dot(f, d[j]);
          else acc8(f, d[j]);
        }
      }
      if (__builtin_amdgcn_ballot_w64(deg > 32)) {   // rows past 32 neighbours (rare)
        const int k0 = (m0 >> 6) * 8;
        for (int k = 32; k < deg; ++k) {
          const unsigned slot = a.slots[k0 + k];
          const uint4 dv = *reinterpret_cast<const uint4*>(lds + slot * (WIDTH * 2) + base);
          if constexpr (DOT) acc8_dot(f, dv);
          else acc8(f, dv);
        }
      }
      bf16x8 o;
  #pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (__bf16)f[j];
      *reinterpret_cast<bf16x8*>(a.out + (long long)row0 * a.ldo + 8 * l8) = o;    }

    // every wave's LDS reads of this step are done (their values were consumed)
    // before any wave's next DMA overwrites ring rows, index blocks or slot lists
    if (!one) raw_barrier();
  }
}

}  // namespace

int spmm_win_max_beta() { return 352; }   // 8-aligned, 2 beta < RR - 3 STEP (712)

}  // namespace snd

using namespace snd;

namespace {
int window_launch(bool pairs, const int* meta, const uint16_t* slots, const int* rows, const int* order,
                  int n_rows, int n_per_graph, int n_graphs, int beta, const void* h, int ldh, int width,
                  void* out, int ldo, snd_stream_t stream) {
  SND_CHECK_ARG(meta && slots && rows && order && h && out, "snd_csr_spmm_bf16_window: null operand");
  SND_CHECK_ARG(width == WIDTH, "snd_csr_spmm_bf16_window: width %d (the ring holds 64-column rows)", width);
  SND_CHECK_ARG(n_per_graph > 0 && n_graphs > 0 && (long long)n_per_graph * n_graphs == n_rows,
                "snd_csr_spmm_bf16_window: n_rows != n_per_graph * n_graphs");
  SND_CHECK_ARG(ldh % 8 == 0 && ldo % 8 == 0 && ldh >= width && ldo >= width,
                "snd_csr_spmm_bf16_window: ldh / ldo must be multiples of 8 >= width");
  const int beta8 = (beta + 7) & ~7;
  SND_CHECK_ARG(beta >= 0 && beta8 <= spmm_win_max_beta() && (long long)n_rows < (1LL << 31),
                "snd_csr_spmm_bf16_window: beta %d exceeds the ring (<= %d)", beta, spmm_win_max_beta());
  // segments: about 256 workgroups in all, at least one step each
  const int steps = cdiv(n_per_graph, STEP);
  const int spg = std::max(1, std::min(steps, cdiv(256, n_graphs)));
  const int seg = cdiv(steps, spg) * STEP;
  WinArgs a{meta, slots, rows, order, reinterpret_cast<const __bf16*>(h), ldh,
            reinterpret_cast<__bf16*>(out), ldo, n_per_graph, cdiv(n_per_graph, seg), seg, beta8,
            debug_flags() >> 16};
  const dim3 grid(n_graphs * a.spg);
  const hipStream_t st = (hipStream_t)stream;
  if (pairs) {
    hipLaunchKernelGGL((spmm_win_kernel<4, true, false, true>), grid, dim3(WT), 0, st, a);
  } else if (a.dbg & 64) {
    hipLaunchKernelGGL((spmm_win_kernel<4, true, true>), grid, dim3(WT), 0, st, a);
  } else if (a.dbg & 8) {
    if (a.dbg & 16) hipLaunchKernelGGL((spmm_win_kernel<8, false, false>), grid, dim3(WT), 0, st, a);
    else hipLaunchKernelGGL((spmm_win_kernel<8, true, false>), grid, dim3(WT), 0, st, a);
  } else {
    if (a.dbg & 16) hipLaunchKernelGGL((spmm_win_kernel<4, false, false>), grid, dim3(WT), 0, st, a);
    else hipLaunchKernelGGL((spmm_win_kernel<4, true, false>), grid, dim3(WT), 0, st, a);
  }
  SND_LAUNCH_CHECK("spmm_win_kernel");
  return 0;
}
}  // namespace

extern "C" int snd_csr_spmm_bf16_window(const int* meta, const uint16_t* slots, const int* rows,
                                        const int* order,
                                        int n_rows, int n_per_graph, int n_graphs, int beta,
                                        const void* h, int ldh, int width, void* out, int ldo,
                                        snd_stream_t stream) {
  return window_launch(false, meta, slots, rows, order, n_rows, n_per_graph, n_graphs, beta, h, ldh, width,
                       out, ldo, stream);
}

extern "C" int snd_csr_spmm_bf16_window_pairs(const int* meta, const uint16_t* slots, const int* rows,
                                              const int* order,
                                              int n_rows, int n_per_graph, int n_graphs, int beta,
                                              const void* h, int ldh, int width, void* out, int ldo,
                                              snd_stream_t stream) {
  return window_launch(true, meta, slots, rows, order, n_rows, n_per_graph, n_graphs, beta, h, ldh, width,
                       out, ldo, stream);
}
