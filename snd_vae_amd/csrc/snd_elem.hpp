#pragma once
#include "snd_common.hpp"

namespace snd {

// ---- reparameterisation (model.py:153-161) + KL (optimizer.py:193)
struct ReparamFwdArgs {
  const float* ms; int ldms; int rows; int L;
  const float* eps_in; unsigned long long seed; const int* step;
  float* eps_out; float* z;
  double* kl_part;            // [blocks]
  __bf16* zb; int ldzb;       // optional bf16 copy of z (fast-path MFMA operand)
  unsigned long long eps_base = 0;   // Philox element index of row 0 (data parallel: rank * rows * L)
  int* stepn = nullptr;        // optional: *step + 1 published for the fused-Adam reduction (ReduceAdam)
};
int reparam_blocks(int rows, int L);
int launch_reparam_fwd(const ReparamFwdArgs& a, hipStream_t s);

// Graph-latent heads on <= kSmallHeadRows rows (B graphs): [mu || s] = h Wms + bms fused
// with the reparameterisation + KL (model.py:114-115,153-161; optimizer.py:193), and the
// backward as two launches: d[mu || s] (reparam/KL backward) with the Wms / bms slab of
// one split ([gh + 1][2L], bias row last, as the generic split-K wgrad writes it), then
// dh = d[mu || s] Wms^T.  Each block stages its operand slice in LDS first, so no thread
// walks a chain of dependent global loads (the generic GEMMs ran ~6 us apiece here).
constexpr int kSmallHeadRows = 32;
struct SmallHeadFwdArgs {
  const float* hh; int rows; int gh;          // [rows][gh]
  const float* wms; const float* bms; int L;  // [gh][2L], [2L]
  float* ms;                                  // [rows][2L] out
  const float* eps_in; unsigned long long seed; const int* step; unsigned long long eps_base;
  float* eps_out; float* z;                   // [rows][L]
  double* kl_part;                            // [small_head_fwd_blocks(L)]
  int* stepn = nullptr;        // optional: *step + 1 published for the fused-Adam reduction (ReduceAdam)
};
struct SmallHeadBwdArgs {
  const float* hh; int rows; int gh;
  const float* wms; int L;
  const float* ms; const float* eps; const float* dz;   // dz: [rows][L]
  float kl_scale;
  float* dms;                                 // [rows][2L]
  float* slab;                                // [gh + 1][2L]
  float* dh;                                  // [rows][gh]
};
bool small_head_supported(int rows, int gh, int L);
int small_head_fwd_blocks(int L);
int launch_small_head_fwd(const SmallHeadFwdArgs& a, hipStream_t s);
int launch_small_head_bwd(const SmallHeadBwdArgs& a, hipStream_t s);

struct ReparamBwdArgs {
  const float* ms; int ldms; int rows; int L;
  const float* eps;
  const float* dz_dec;        // [rows, L] gradient from the conv decoders (may be null)
  const float* dJd; const float* ej;   // zz^T terms, combined as adj_scale*(dJd + ej); may be null
  float adj_scale;            // norm / (B N^2)
  float kl_scale;             // beta / (rows * L)
  float* dms; int lddms;      // [rows, 2L] = [dmu || dlogstd]
};
int launch_reparam_bwd(const ReparamBwdArgs& a, hipStream_t s);

// ---- sigmoid output heads + MSE (model_joint.py:121,144; optimizer.py:149,153)
struct HeadArgs {
  const float* u; int ldu; int cin;
  const float* w; const float* b; int cout;
  const float* target; int ldt;
  float count;                // denominator of the mean: rows * cout
  float* yhat;                // optional [rows, cout]
  float* du; int lddu;        // [rows, cin]
  float* wpart;               // [blocks][cin*cout + cout] (dW then db)
  double* sse_part;           // [blocks]
};
int head_blocks(int rows);
int launch_heads(const HeadArgs* h, int nheads, int rows, hipStream_t s);

// ---- decoder BN + lrelu backward (BN then lrelu: model_joint.py:115-116)
struct DecBwdArgs {
  const float* du; int lddu;
  const float* y; int ldy;    // conv output incl. bias (BN input)
  const float* gamma; const float* beta; int ncols;
  float* dy; int lddy;        // gradient wrt conv output
  float* part;                // [blocks][3*ncols] = {dgamma, dbeta, dbias}
};
int col_blocks(int rows);
int launch_dec_bwd(const DecBwdArgs* a, int n, int rows, hipStream_t s);

// ---- encoder lrelu + BN (+ encoder_g BN) backward (model.py:107-112)
struct EncBwdArgs {
  const float* dg; int lddg;   // gradient wrt layer output (G if has_enc else H)
  const float* h2; int ldh2;   // [BN(lrelu P) || X] (has_enc only)
  const float* ge;             // encoder_g gamma (has_enc only)
  int wenc;                    // width of G (has_enc only)
  const float* p; int ldp;     // pre-activation A @ XW
  const float* g;              // layer BN gamma
  int h;                       // layer width
  float* dp; int lddp;         // gradient wrt pre-activation
  float* part;                 // [blocks][2*wenc (if enc) + 2*h]
  int has_enc;
};
int launch_enc_bwd(const EncBwdArgs& a, int rows, hipStream_t s);

// ---- finalize: losses, step counter (main.py:331-334, optimizer.py:203)
struct FinalizeArgs {
  const double* zzt_part; int n_zzt;
  const double* edge_part; int n_edge;
  const double* kl_part; int n_kl;
  const double* sse_s; const double* sse_n; int n_s;
  const int* rowptr; int ngraphs; int n; int L; int sdim; int nfeat;
  float beta; float norm;
  double* losses; float* grad_tail; int* step;
  double kl_count;            // elements of mu (0: ngraphs * n * L, node latent)
};
int launch_finalize(const FinalizeArgs& a, hipStream_t s);

}  // namespace snd
