// bf16 fast path of the train step: packed bf16 weight images, the row-tile
// conv/linear engine (halo rows staged once in LDS, fused epilogues) and the
// weight-gradient engine (LDS transpose reads).  The f32 parity mode keeps
// the generic GEMM engine of snd_gemm.hip.
#pragma once
#include "snd_common.hpp"

namespace snd {

// Two-part column layout of a logical [a | b] tensor: part A at physical
// columns [0, a), part B at [offb, offb + b) (offb = round_up(a, 8) keeps
// part B 16-byte aligned in bf16).  b == 0: plain layout.  The decoder's
// fused [s | n] branches use it so one launch serves both.
struct ColMap {
  int a, b, offb;
  __host__ __device__ int phys() const { return b ? offb + b : a; }
  __host__ __device__ bool valid(int c) const { return c < a || (b && c >= offb && c < offb + b); }
  __host__ __device__ int logical(int c) const { return c < a ? c : c - offb + a; }
};
inline ColMap colmap_plain(int n) { return {n, 0, n}; }
inline ColMap colmap_split(int a, int b) { return {a, b, (int)round_up(a, 8)}; }

// ---- packed weight images ------------------------------------------------
// dst[t][n][k] (bf16, np x kp per tap, 16-byte chunks of k XOR-swizzled per
// row n -- the LDS image the row engine reads with ds_read_b128).
// Source window W[T][A][B] (fp32, row-major) placed at (n_off, k_off):
//   mode 0 (forward):  n = b - b0 + n_off, k = a - a0 + k_off, tap t
//   mode 1 (data grad): n = a - a0 + n_off, k = b - b0 + k_off, tap T-1-t
struct PackSrc {
  const float* w;
  int A, B;
  int a0, a1, b0, b1;
  int n_off, k_off;
  int mode;                   // 0: w[t][k][n] -> (n, k); 1: transposed, taps flipped; 2: identity
};
struct PackDesc {
  __bf16* dst;
  int T, kp, np;
  int nsrc;
  PackSrc s[2];
};
constexpr int kMaxPack = 16;
int launch_pack(const PackDesc* d, int n, hipStream_t s);
size_t pack_bytes(int T, int kp, int np);

// ---- row engine -----------------------------------------------------------
// out[r][n] = epi( sum_t sum_k x[r + t - H][k] * Wt[t][k][n] ), H = (T-1)/2,
// rows r + t - H outside r's graph read as zero (TF SAME padding per graph).
enum RcEpi {
  RC_LIN = 0,     // (+bias) -> out; optional colpart q0 = sum out
  RC_FWD = 1,     // y = acc + bias -> y; out = lrelu(y*gamma*c + beta)
  RC_DECBWD = 2,  // du = acc; t = y*gamma*c + beta; dt = du*lrelu'(t); out = dy = dt*gamma*c;
                  // colpart {sum dt*y, sum dt, sum dy}
  RC_ENC1 = 3,    // dG = acc (cols [0, h) = B1 part, [h, h+f) = X part); see snd_fast.hip
  RC_ENC0 = 4,    // dB0 = acc; P0 recomputed from AX, W0; see snd_fast.hip
};
struct RcArgs {
  const void* x; int ldx; int K; int x_bf16;
  int R, npg, T;
  const __bf16* wpk; int kp, np;
  int N;                        // physical output columns
  ColMap cols;                  // physical -> logical (per-column parameters)
  const float* bias; const float* gamma; const float* beta;
  // part-B parameter vectors of a split layout (nullptr: one logical vector)
  const float* bias_b; const float* gamma_b; const float* beta_b;
  float* y; int ldy;            // RC_FWD out / RC_DECBWD in (fp32)
  void* out; int ldo; int out_bf16;
  float* colpart; int ncp;      // [gridDim.x][ncp][N] (nullptr: none)
  // encoder epilogues
  const float* p; int ldp;      // ENC1: P1 [R][h]; ENC0: AX [R][f]
  const float* xf; int ldxf; int f;   // ENC1: X
  const float* w0;              // ENC0: W0 [f][h]
  const float* g2; const float* b2;   // ENC1: bn1 gamma/beta (gamma/beta = bne)
  int h;                        // ENC1: h1
  const void* zero;             // >= 16 zero bytes in device memory (LDS-DMA fill source)
  int dbg;                      // measurement only: bits skip phases (see snd_debug_set)
  // RC_LIN / RC_FWD: x columns [K, K + ktail) (bf16, ktail <= 4) beyond the image enter in
  // the epilogue: acc[r][n] += sum_j x[r][K + j] * wtail[j * ldwt + n] (a [B | X] input one
  // feature column wider than 128)
  int ktail; const float* wtail; int ldwt;
  int npb;                      // image columns per workgroup (set by launch_rowconv: np, or a
                                // 16-multiple window when the whole image exceeds the LDS budget;
                                // blockIdx.y selects the window)
  // RC_ENC0 with T = 1 and a CSR (round 5): the x rows are A @ x, gathered into the LDS
  // image by the workgroup itself (the register-gather SpMM's fp32 sums in colidx order,
  // bitwise its output) and also stored to gout [R][ldgo] (bf16) for the weight gradient:
  // the separate A @ dP1 SpMM launch and its output's re-read disappear
  const int* g_rowptr; const int* g_colidx; void* gout; int ldgo;
};
constexpr int kRcRows = 128;    // rows per workgroup tile
constexpr size_t kRcLdsLimit = 136 * 1024;   // dynamic LDS (static partials use the rest)
int rc_blocks(int R);
size_t rc_lds_bytes(int T, int kp, int np);
// columns per workgroup for an image: np if it fits kRcLdsLimit, else the widest
// 16-multiple window that does (0: none does)
int rc_cols_per_block(int T, int kp, int np);
int launch_rowconv(const RcArgs& a, int epi, hipStream_t s);

// ---- weight-gradient engine ----------------------------------------------
// slab[wg][t][k][n] = sum over the workgroup's rows r of x[r + t - H][k] * dy[r][n]
// (same per-graph zero padding), k < K, n < N; slab rows are padded to
// n4 = round_up(N, 4) floats (wgrad_n4).  Deterministic partials.
struct WgArgs {
  const void* x; int ldx; int K; int x_bf16;
  const void* dy; int lddy; int N; int dy_bf16;
  int R, npg, T;
  int rows_per_wg;              // multiple of kRcRows
  int pairs_per_wg;             // (tap, 16-column k block) pairs per workgroup (<= 20)
  float* slab;
  const void* zero;             // >= 16 zero bytes in device memory
  int dbg;
  // slab geometry of the whole weight when this descriptor is a (k, n) window of it
  // (launch_wgrad_multi's LDS split): rows sK, padded width sn4, window origin
  // (wk0, wn0); 0 = the descriptor's own K / n4(N) at origin 0
  int sK, sn4, wk0, wn0;
  unsigned* stamps;             // measurement only (debug bit 1 << 21): 12 words per workgroup
  long long stamp_words;        // capacity of stamps in words (checked by launch_wgrad_multi)
};
struct WgGeom { int rows_per_wg, pairs_per_wg, gx, gy; };
// chunks > 0: that many row chunks per weight (the step's multi-segment launch);
// 0: about 256 workgroups per weight (one launch each)
WgGeom wgrad_geom(int R, int T, int K, int N, int chunks = 0);
inline int wgrad_n4(int N) { return (N + 3) & ~3; }
int launch_wgrad(const WgArgs& a, hipStream_t s);
// n independent weight gradients (each its own geometry and slab) in one launch
constexpr int kMaxWgMulti = 32;   // segments after the column-window split (C5: 29)
int launch_wgrad_multi(const WgArgs* a, int n, hipStream_t s);

// ---- fused sigmoid head + MSE + backward + BN/lrelu backward of the head's
// input layer (model_joint.py:115-121,138-144; optimizer.py:149,153).
// One thread per row.  part[block] = {dW [cin][cout], db [cout],
// sum dt*y [cin], sum dt [cin], sum dy [cin]}.
struct HeadFastArgs {
  const void* u; int ldu; int u_bf16;     // head input U = lrelu(BN(y))
  const float* y; int ldy;               // U's pre-activation
  const float* gamma; const float* beta;  // U's BN
  int cin;
  const float* w; const float* b; int cout;
  const float* target; int ldt;
  float count;                            // rows * cout (mean denominator)
  float* yhat;                            // optional [R][cout]
  __bf16* dy; int lddy;                   // gradient wrt y (bf16)
  float* part;
  double* sse;                            // [blocks]
};
constexpr int kHeadFastRows = 256;
int heads_fast_blocks(int R);
bool heads_fast_supported(int cin, int cout);   // built (cin, cout) pairs
int heads_fast_parts(int cin, int cout);
int launch_heads_fast(const HeadFastArgs* h, int n, int R, hipStream_t s);

// ---- encoder (snd_fast_enc.hip) ------------------------------------------
// GraphConvolution 0 as (A X) W0: AX (fp32 [R][4], bf16 [R][8]) and
// H1 = [BN0(lrelu(AX W0)) | X] (bf16 [R][ldh1]).
struct Gcn0Args {
  const int* rowptr; const int* colidx; int R;
  const float* x; int ldx; int f;
  const float* w0; const float* g0; const float* b0; int h0;
  __bf16* h1; int ldh1;
  float* ax; __bf16* axb;
  int xcd_nbg;                // xcd_nbg(): row blocks per graph for the XCD-aware order
  const int* row_order;       // optional processing order of the rows (locality schedule)
  // the step's packed weight images, built by extra workgroups of the same launch (as
  // enc_front does) when npack > 0; pack_blk is filled by launch_gcn0
  PackDesc pack[kMaxPack]; int pack_blk[kMaxPack + 1]; int npack;
};
int xcd_nbg(int npg, int ngraphs);
int gcn0_blocks(int R);
int launch_gcn0(const Gcn0Args& a, hipStream_t s);

// bf16-input CSR SpMM: PLAIN (bf16 out) or GCN (pre-activation fp32 and
// G = BNe([BN1(lrelu(P)) | X]) bf16).
struct SpmmBfArgs {
  const int* rowptr; const int* colidx; int R;
  const __bf16* h; int ldh; int width; int epi;
  __bf16* out; int ldo;
  float* pre; int ldp;
  const float* g1; const float* b1;
  const float* x; int ldx; int f;
  const float* ge; const float* be;
  __bf16* g; int ldg;
  int xcd_nbg;
  const int* row_order;       // optional processing order of the rows (locality schedule)
  // optional row tiles (snd_row_tiles_t over row_order): tile_rows > 0 selects the LDS-staged kernel
  const int* t_rowid = nullptr; const int* t_trp = nullptr; const uint16_t* t_lcol = nullptr;
  const int* t_ucol = nullptr; int t_rows = 0; int t_ustride = 0;
  int npg = 0; int ngraphs = 0;  // graph shape for the XCD-aware tile order (0: natural)
};
int launch_spmm_bf16(const SpmmBfArgs& a, hipStream_t s);

// reparameterisation backward with bf16 [dmu | dlogstd] and per-block column sums
struct ReparamBwdFastArgs {
  const float* ms; int ldms; int R; int L;
  const float* eps; const float* dz_dec; const float* dJd; const float* ej;
  float adj_scale, kl_scale;
  __bf16* dms; int lddms;
  float* colpart;             // [blocks][2L]
  // zz^T column-split partials [nextra][R][L] added to dJd here (launch_zzt_dense defer_split)
  const float* dJd_extra = nullptr; int nextra = 0;
};
int reparam_bwd_fast_blocks(int R, int L);
// edge_bf16 + reparam_bwd_fast in one launch (e.ej unused): partials {loss, tp} into e.part
// and [mu | s] bias sums into a.colpart, edge_reparam_blocks(R) blocks each
int edge_reparam_blocks(int R);

// reparameterisation + KL fused with the zz^T staging images (snd_zzt.hpp ZztStage)
struct ReparamPrepArgs {
  const float* ms; int ldms; int n, npad, ngraphs, L;
  const float* eps_in; unsigned long long seed; const int* step;
  float* z; float* eps_out; __bf16* zb;
  __bf16* jrow; __bf16* jt; float* colpart;
  double* kl_part;            // [ngraphs * npad / 64]
  int stage_only;             // 1: ms is J itself (T-ref projection output); no eps / KL
  unsigned long long eps_base = 0;   // Philox element index of row 0 (data parallel: rank * rows * L)
  int* stepn = nullptr;        // optional: *step + 1 published for the fused-Adam reduction (ReduceAdam)
};
int reparam_prep_blocks(int ngraphs, int npad);

// per-edge CE terms from the bf16 z copy (snd_spmm.hpp EdgeArgs semantics)
struct EdgeBfArgs {
  const int* rowptr; const int* colidx; int R;
  const __bf16* z; int d;
  float pos_weight;
  float* ej;                  // [R][d]
  double* part;               // [blocks][2] = {loss, tp}
  int xcd_nbg;
  const int* row_order;       // optional processing order of the rows (locality schedule)
};
int edge_bf16_blocks(int R);
int launch_edge_bf16(const EdgeBfArgs& a, hipStream_t s);
int launch_reparam_prep(const ReparamPrepArgs& a, int dp, hipStream_t s);
int launch_reparam_bwd_fast(const ReparamBwdFastArgs& a, hipStream_t s);
int launch_edge_reparam_bwd(const EdgeBfArgs& e, const ReparamBwdFastArgs& a, hipStream_t s);

int fast_init_attributes();
int debug_flags();

}  // namespace snd
