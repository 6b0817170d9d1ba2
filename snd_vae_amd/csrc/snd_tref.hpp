#pragma once
#include "snd_common.hpp"

namespace snd {

// Graph-latent (T-ref) heads and decoder projection: the skinny, weight-streaming
// linears of model.py:113-115 and model_joint.py:97.  Up to kTrefMaxB graphs
// per launch; every kernel reads its weight matrix exactly once (HBM-bound).
constexpr int kTrefMaxB = 8;

// TF1 Adam applied where a weight gradient is produced complete (1 GPU: no
// all-reduce between gradient and update).  The step counter is read before the
// step's finalize advances it, so the update uses t = *step + 1 (optimizer.py:125).
struct AdamFuse {
  float* p; float* m; float* v;   // block base of params / Adam state (same layout)
  float lr, b1, b2, eps;
  const int* step;
};

// h[b, j] = sum_k G[b, k] Wh[k, j] (+ bh[j] in block 0): split-K partial slab
// [blocks][B][gh]; reduce over blocks gives h.  G [B, K] contiguous per graph
// (the row-major tf.reshape of [N, W] node rows, model.py:113).
struct TrefHeadFwdArgs {
  const float* g; long long K; int B;
  const float* wh; int gh; const float* bh;
  float* slab;
  // bf16 G of the fast encoder instead of g: node rows of width W at leading dim ldg
  // (flat index k = n * W + c -> gb[(b * npg + n) * ldg + c])
  const __bf16* gb; int ldg; int W; int npg;
};
int tref_head_fwd_blocks(long long K, int gh);
int launch_tref_head_fwd(const TrefHeadFwdArgs& a, hipStream_t s);

// dWh[k, j] = sum_b G[b, k] dh[b, j]   (written, complete: no reduction)
// dG[b, k]  = sum_j dh[b, j] Wh[k, j]
struct TrefHeadBwdArgs {
  const float* g; long long K; int B;
  const float* wh; int gh;
  const float* dh;            // [B, gh]
  float* dwh;                 // [K, gh]
  float* dg;                  // [B, K]   (or, with gb, bf16 rows dgb[(b * npg + n) * ldg + c])
  const __bf16* gb; int ldg; int W; int npg; __bf16* dgb;
  AdamFuse adam;              // adam.p != null: update Wh in place instead of writing dwh
};
int launch_tref_head_bwd(const TrefHeadBwdArgs& a, hipStream_t s);

// J[b, c] = sum_l z[b, l] Wp[l, c] + bp[c]   (c < Cp = N * node_h)
struct TrefProjFwdArgs {
  const float* z; int B; int L;
  const float* wp; const float* bp; long long Cp;
  float* j;                   // [B, Cp]
};
int launch_tref_proj_fwd(const TrefProjFwdArgs& a, hipStream_t s);

// dJ = dz_dec + adj_scale (dJd + ej)      (combined on the fly, [B, Cp] each)
// dWp[l, c] = sum_b z[b, l] dJ[b, c]; dbp[c] = sum_b dJ[b, c]   (written, complete)
// dz partial slab [blocks][B][L] = sum_c dJ[b, c] Wp[l, c]
struct TrefProjBwdArgs {
  const float* z; int B; int L;
  const float* wp; long long Cp;
  const float* dz_dec; const float* dJd; const float* ej; float adj_scale;
  float* dwp; float* dbp;
  float* slab;
  AdamFuse adam;              // adam.p != null: update Wp in place instead of writing dwp
  AdamFuse adam_b{};          // adam_b.p != null: update bp in place instead of writing dbp
};
int tref_proj_bwd_blocks(long long Cp);
int launch_tref_proj_bwd(const TrefProjBwdArgs& a, hipStream_t s);

// Vectorised TF1 Adam (float4 streams; n % 4 == 0, 16-byte aligned buffers)
int launch_adam_vec(float* p, const float* g, float* m, float* v, long long n, float lr,
                    float b1, float b2, float eps, float gscale, const int* step, hipStream_t s);
// the same update over up to kAdamMaxRanges disjoint [off, off + cnt) ranges (multiples of 4)
constexpr int kAdamMaxRanges = 16;
int launch_adam_ranges(float* p, const float* g, float* m, float* v, const long long* off,
                       const long long* cnt, int n, float lr, float b1, float b2, float eps, float gscale,
                       const int* step, hipStream_t s);

}  // namespace snd
