// Fused encoder heads of the node-latent bf16 fast path (snd_head.hip): the row-local
// chains on either side of zz^T collapsed into one launch each.
#pragma once
#include "snd_fast.hpp"

namespace snd {

// GraphConvolution 1 gather + its epilogue (layers.py:122-123, model.py:107-112),
// h = G Wh + bh, [mu | s] = h Wms + bms (model.py:113-115), z = mu + eps e^s
// (model.py:159) with the KL partials (optimizer.py:193) and the zz^T staging images
// (reparam_prep semantics).  One workgroup = 128 rows of one graph.
struct HeadFwdArgs {
  const int* rowptr; const int* colidx;
  int R, npg, ngraphs, npad;
  const __bf16* xw1; int h1;                  // XW1 [R][h1] (bf16, the gathered operand)
  const float* g1; const float* b1;           // BN1
  const float* x; int ldx; int f;             // node features (concat X)
  const float* ge; const float* be;           // encoder_g BN
  float* p1;                                  // P1 [R][h1] fp32 (pre-activation)
  __bf16* g; int ldg;                         // G [R][ldg] bf16
  const __bf16* wh_img; int kp1, np1, gh;     // packed Wh image [np1][kp1]
  const float* bh;
  __bf16* hh;                                 // h [R][gh] bf16
  const __bf16* wms_img; int kp2, np2;        // packed Wms image [np2][kp2], np2 = 2L
  const float* bms;
  float* ms;                                  // [mu | s] [R][2L] fp32
  int L;
  const float* eps_in; unsigned long long seed; const int* step; unsigned long long eps_base;
  float* z; float* eps_out; __bf16* zb;       // z fp32 / bf16 [R][L], eps [R][L]
  __bf16* jrow; __bf16* jt; float* colpart;   // zz^T staging (zzt_stage), DP == L
  double* kl_part;                            // [ngraphs * npad / 64]
  int dbg;
  int* stepn = nullptr;                       // optional: *step + 1 for the fused-Adam reduction
};
bool head_fwd_supported(int h1, int f, int gh, int L, int kp1, int np1, int kp2, int np2);
int launch_head_fwd(const HeadFwdArgs& a, hipStream_t s);

// Per-edge CE terms (the A = 1 pairs, optimizer.py:142-144) + the reparameterisation /
// KL backward (model.py:159, optimizer.py:193) + dh = d[mu | s] Wms^T (model.py:114-115)
// + dG = dh Wh^T with the encoder BN / lrelu backward down to dP1 (model.py:107-113):
// edge_bf16 + reparam_bwd_fast + two row-engine launches in one.  One workgroup = 128
// rows (the row engine's tiles: its column partials keep their layout and order).
struct HeadBwdArgs {
  const int* rowptr; const int* colidx; int R;
  const __bf16* zb; int L; float pos_weight;   // z (bf16) [R][L]
  double* edge_part;                           // [tiles][2] = {loss, tp}
  const float* ms; const float* eps; const float* dz_dec; const float* dJd;
  const float* dJd_extra; int nextra;          // zz^T column-split partials, added in order
  float adj_scale, kl_scale;
  __bf16* dms; float* bms_part;                // d[mu | s] [R][2L] bf16; [tiles][2L]
  const __bf16* wmsb_img; int kp1, np1, gh;    // Wms^T image [np1][kp1 = 2L]
  __bf16* dh; float* bh_part;                  // dh [R][gh] bf16; [tiles][gh]
  const __bf16* whb_img; int kp2, np2;         // Wh^T image [np2][kp2]
  int W, h1;
  const float* ge; const float* g1; const float* b1;   // BNe gamma; BN1 gamma, beta
  const float* p1; const float* x; int ldx;            // P1 [R][h1] fp32, X [R][ldx]
  __bf16* dp1; float* enc1_part;               // dP1 [R][h1] bf16; [tiles][4][W]
  int npg, ngraphs;                            // XCD-aware tile order (npg % 128, ngraphs % 8)
  int dbg;
};
bool head_bwd_supported(int L, int gh, int W, int h1, int kp1, int np1, int kp2, int np2);
// rows per backward-head tile: 128, or 64 when 128-row tiles would leave more than half
// the CUs idle (fewer than kHeadBwdSmall tiles: one or two graphs of 4096 rows, the C3
// per-rank step).  At the full batch 64-row tiles measured head_bwd 25.4 vs 25.7 us with
// no step change (round 5), so the batch keeps 128.
constexpr int kHeadBwdRows = 128;
#ifndef SND_HB_SMALL
#define SND_HB_SMALL 128
#endif
constexpr int kHeadBwdSmall = SND_HB_SMALL;
// 32-row tiles when even 64-row tiles stay under kHeadBwdTiny (one N = 4096 graph)
#ifndef SND_HB_TINY
#define SND_HB_TINY 128
#endif
#ifndef SND_HB_TINY_ROWS
#define SND_HB_TINY_ROWS 32
#endif
constexpr int kHeadBwdTinyRows = SND_HB_TINY_ROWS;
constexpr int kHeadBwdTiny = SND_HB_TINY;
int head_bwd_rows(int R);
int head_tiles(int R);   // backward-head tiles (head_bwd_rows(R) rows each)
int launch_head_bwd(const HeadBwdArgs& a, hipStream_t s);

// GraphConvolution 0 as (A X) W0 (gcn0 semantics: AX, H1 = [BN0(lrelu(AX W0)) | X]) and
// XW1 = H1 W1 (layers.py:121, the first product of GraphConvolution 1) in one 128-row
// tile pass; the step's packed weight images ride in the same launch as extra workgroups.
struct FrontArgs {
  const int* rowptr; const int* colidx; int R;
  const float* x; int ldx; int f;
  const float* w0; const float* g0; const float* b0; int h0;
  __bf16* h1; int ldh1; float* ax; __bf16* axb;
  const float* w1; int n1; int kp1, np1;     // W1 [h0 + f][n1] fp32; its image geometry
  __bf16* xw1;                               // [R][n1]
  PackDesc pack[kMaxPack]; int npack;        // weight images built by the extra workgroups
  int pack_wg[kMaxPack + 1];                 // workgroup prefix per image
  int dbg;
};
bool front_supported(int f, int h0, int n1, int kp1, int np1);
int launch_front(FrontArgs& a, const PackDesc* pack, int npack, hipStream_t s);

int head_init_attributes();

}  // namespace snd
