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
};
int reparam_blocks(int rows, int L);
int launch_reparam_fwd(const ReparamFwdArgs& a, hipStream_t s);

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
