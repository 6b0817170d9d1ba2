// Fused bf16 decoder of the train step (model_joint.py:112-145; optimizer.py:149,153).
// Two launches replace the row engine's seven decoder launches (snd_dec.hip).
#pragma once
#include "snd_fast.hpp"

namespace snd {

constexpr int kDecRows = 128;   // own rows per tile (one workgroup per tile, tiles never span graphs)
// 64-row tiles when 128-row tiles would leave more than half the CUs idle (fewer than
// kDecSmall tiles: one or two graphs of 4096 rows, the C3 per-rank step)
constexpr int kDecRowsSmall = 64;
#ifndef SND_DEC_SMALL
#define SND_DEC_SMALL 128
#endif
constexpr int kDecSmall = SND_DEC_SMALL;
// 32-row tiles when even 64-row tiles stay under kDecTiny (one N = 4096 graph: 0.1210 ->
// 0.1157 ms together with head_bwd's 32-row tiles)
#ifndef SND_DEC_TINY_ROWS
#define SND_DEC_TINY_ROWS 32
#endif
constexpr int kDecRowsTiny = SND_DEC_TINY_ROWS;
#ifndef SND_DEC_TINY
#define SND_DEC_TINY 128
#endif
constexpr int kDecTiny = SND_DEC_TINY;

// Packed weight image in the workspace (pack_kernel layout [tap][n][k], T = 5)
struct DecImg { const __bf16* w; int kp, np; };

struct DecChainFwdArgs {
  const __bf16* zb; int ldz; int dj;          // J [R][dj]
  int R, npg, ngraphs;
  DecImg k1, k2, k3;                          // conv1 (dj -> w1), conv2 (w1 -> w2), conv3 (s2 -> s3)
  ColMap m1, m2; int s3;
  const float *b1, *g1, *be1;                 // conv1 logical [s1 + n1] vectors
  const float *b2s, *g2s, *be2s, *b2n, *g2n, *be2n;
  const float *b3, *g3, *be3;
  float* y1; int ldy1; __bf16* u1;            // own rows: Y1 fp32, U1 bf16 (same ld)
  float* y2; int ldy2; __bf16* u2;            // own rows: Y2 fp32, U2 bf16
  // sigmoid heads (model_joint.py:121,144) + MSE + backward (HeadFastArgs semantics)
  const float *ws, *bs; int sd; const float* s_truth; float cnt_s; float* shat;
  const float *wn, *bn; int nf; const float* x_truth; float cnt_n; float* xhat;
  __bf16* dy3; int lddy3;                     // dY3 [R][lddy3]
  __bf16* dy2; int lddy2;                     // dY2 [R][lddy2]; the head writes the n part at m2.offb
  float* phs; float* phn;                     // [tiles][dec_head_parts]
  double* sse_s; double* sse_n;               // [tiles]
  const void* zero;
  int dbg;                                    // measurement only (snd_debug_set): phase-skip bits
};

struct DecChainBwdArgs {
  int R, npg, ngraphs, dj;
  DecImg k3t, k2t, k1t;                       // conv3^T (s3 -> s2), conv2^T (w2 -> w1), conv1^T (w1 -> dj)
  ColMap m1, m2; int s3;
  const float *g1, *be1;                      // conv1 BN (logical)
  const float *g2s, *be2s;                    // conv2 s-branch BN
  const float* y1; int ldy1;                  // Y1 fp32 (BN input of conv1)
  const float* y2; int ldy2;                  // Y2 fp32
  __bf16* dy3; int lddy3;                     // dY3 (in)
  __bf16* dy2; int lddy2;                     // dY2: n part in (heads), s part out (own rows)
  __bf16* dy1; int lddy1;                     // dY1 out (own rows)
  float* dz; int lddz;                        // d cost / dJ of the decoders, own rows
  float* pc2s;                                // [tiles][3 s2]  {sum dt y, sum dt, sum dy}
  float* pc1;                                 // [tiles][3 w1]
  const void* zero;
  int dbg;
};

int dec_rows(int ngraphs, int npg, int dj);    // kDecRows, kDecRowsSmall or kDecRowsTiny (dj > 64: small)
int dec_tiles(int ngraphs, int npg, int dj);
int dec_head_parts(int cin, int cout);        // == heads_fast_parts
bool dec_fused_supported(int dj, const ColMap& m1, const ColMap& m2, int s3, int sd, int nf,
                         const DecImg& k1, const DecImg& k2, const DecImg& k3, const DecImg& k3t,
                         const DecImg& k2t, const DecImg& k1t);
int launch_dec_chain_fwd(const DecChainFwdArgs& a, hipStream_t s);
int launch_dec_chain_bwd(const DecChainBwdArgs& a, hipStream_t s);
int dec_init_attributes();

}  // namespace snd
