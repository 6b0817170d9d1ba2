/*
 * snd_vae.h -- C ABI of the MI355X (gfx950) SND-VAE training hot path.
 *
 * One shared library, libsndvae.so, built by hipcc for gfx950.  Every entry
 * point takes caller-owned DEVICE pointers plus sizes and a HIP stream (passed
 * as an opaque pointer so FFI bindings need no HIP headers), launches
 * stream-ordered work, never allocates or synchronises (graph-capturable), and
 * returns 0 or a negative SND_ERR_* code; snd_last_error() gives the
 * thread-local message.  Layouts are row-major fp32 unless stated.  A batch of
 * B graphs with N nodes each is one block-diagonal CSR (int32 rowptr [B*N+1],
 * sorted int32 colidx with global column ids b*N+j) plus row-major node data
 * [B*N, width].
 *
 * Each function names the reference interface it replaces (file:line in
 * xguo7/SND-VAE, TensorFlow 1.x).  The reference is a TF graph-construction
 * API, not an FFI; INTEGRATION.md shows the ctypes binding a maintainer adds.
 */
#ifndef SND_VAE_H
#define SND_VAE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* snd_stream_t; /* hipStream_t */

enum {
  SND_OK = 0,
  SND_ERR_ARG = -1,         /* bad shape/pointer/enum */
  SND_ERR_HIP = -2,         /* HIP launch/runtime error */
  SND_ERR_UNSUPPORTED = -3  /* configuration not built for gfx950 path */
};

enum { SND_F32 = 0, SND_BF16 = 1 }; /* MFMA operand dtype; accumulation always fp32 */

const char* snd_last_error(void);
/* the ABI this header describes; snd_abi_version() returns it */
#define SND_ABI_VERSION 17
int snd_abi_version(void);

/* ---- a1: adjacency ingest ------------------------------------------------
 * Replaces the dense adj_truth feed (main.py:257, input_data.py:62-72):
 * converts B dense [N,N] float 0/1 matrices (diagonal ignored) into the
 * block-diagonal CSR, entries in np.where row-major order (bit-exact vs
 * scipy.sparse.csr_matrix).  *nnz_out (device int) receives the total.
 * Fails with SND_ERR_ARG (message set) via *nnz_out = -1 when colidx_cap is
 * too small.  workspace: snd_dense_to_csr_workspace() bytes. */
size_t snd_dense_to_csr_workspace(int n_graphs, int n);
int snd_dense_to_csr(const float* adj, int n_graphs, int n, int* rowptr,
                     int* colidx, long long colidx_cap, int* nnz_out,
                     void* workspace, size_t workspace_bytes, snd_stream_t stream);

/* ---- a2/a3/a4: CSR SpMM with GraphConvolution epilogue -------------------
 * Replaces tf.matmul(adj, new_x) + lrelu (layers.py:122-123) and the BN /
 * concat that follow it (model.py:107-112).
 *   acc = A @ h                      (A symmetric: also the backward A^T @ dy)
 *   epilogue SND_SPMM_PLAIN: out = acc
 *   epilogue SND_SPMM_GCN:   preact = acc;
 *       y = lrelu(acc) * gamma/sqrt(1.001) + beta        -> out[:, :width]
 *       out[:, width:width+fx] = concat_x                 (model.py:109)
 *       if out2: out2 = [y || concat_x] * g2/sqrt(1.001) + b2 (encoder_g BN) */
enum { SND_SPMM_PLAIN = 0, SND_SPMM_GCN = 1 };
int snd_csr_spmm(const int* rowptr, const int* colidx, int n_rows,
                 const float* h, int ldh, int width, float* out, int ldo,
                 int epilogue, const float* bn_gamma, const float* bn_beta,
                 float* preact, int ldp, const float* concat_x, int ldx, int fx,
                 const float* bn2_gamma, const float* bn2_beta, float* out2,
                 int ldo2, snd_stream_t stream);

/* a2 in the bf16 throughput mode (the SpMM of the fast path, layers.py:122 and
 * its backward): out = A @ h over bf16 rows with fp32 accumulation, rounded to
 * bf16.  width % 8 == 0 and <= 128; ldh, ldo % 8 == 0 (16-byte rows).  When
 * n_per_graph % 32 == 0 and n_graphs % 8 == 0 the row blocks are ordered so one
 * graph's rows stay on one XCD (its gathered rows then hit that XCD's L2);
 * otherwise natural order.  row_order (optional, NULL = 0..n_rows-1) is the
 * order rows are processed in, a permutation of 0..n_rows-1 that keeps each
 * graph's rows inside its own slot range (snd_vae_amd/data.py locality_order:
 * per-graph reverse Cuthill-McKee, so a workgroup's neighbour rows overlap in
 * L1); the result does not depend on it.  h and out are bf16 device buffers. */
int snd_csr_spmm_bf16(const int* rowptr, const int* colidx, int n_rows,
                      const void* h, int ldh, int width, void* out, int ldo,
                      int n_per_graph, int n_graphs, const int* row_order,
                      snd_stream_t stream);

/* Row tiles of a CSR (ABI 5): a per-batch companion format of the bf16 SpMM
 * that stages neighbour rows in LDS.  The schedule (row_order, or natural
 * order) is cut into tiles of tile_rows consecutive slots.  Per tile:
 *   rows[slot]   the tile's rows, by degree (descending, ties by schedule
 *                order), so a wavefront's rows have similar lengths;
 *   trp[slot]    row pointers in slot order into lcol ([n_rows+1]);
 *   lcol[k]      1 + each neighbour's index in its tile's set, every
 *                row's entries in colidx order (u16; 0 is never used);
 *   ucol[t*ustride + u]  the tile's set: ascending distinct neighbour rows,
 *                padded with -1 to ustride = the largest set.
 * The adjacency is static across training steps, so the tiles are built
 * once per batch, on the HOST (plain C++ over host arrays): call
 * snd_spmm_tile_plan with rows/trp/lcol/ucol NULL to size (*ustride), then
 * with them to fill; it returns the ucol length n_tiles*ustride (>= 0) or a
 * negative error.  A tile set of 65535 rows or more is an error.  The
 * SpMM relies on the degree order: a wavefront's first row is its longest. */
typedef struct snd_row_tiles {
  const int* rows;              /* [n_rows] device */
  const int* trp;               /* [n_rows+1] device */
  const uint16_t* lcol;         /* [nnz] device */
  const int* ucol;              /* [n_tiles*ustride] device */
  int tile_rows;                /* rows per tile (<= 128); 0 = no tiles */
  int ustride;                  /* largest tile set */
} snd_row_tiles_t;
long long snd_spmm_tile_plan(const int* rowptr, const int* colidx, int n_rows,
                             const int* row_order, int tile_rows, int* rows,
                             int* trp, uint16_t* lcol, int* ucol, int* ustride);
/* snd_csr_spmm_bf16 over row tiles: a persistent, software-pipelined kernel.
 * Each workgroup walks its tiles; while it sums tile i from LDS, the rows of
 * tile i+1 are in flight into registers and the set of tile i+2 is read.
 * A tile's rows are widened to fp32 in LDS once; every row accumulates its
 * neighbours from LDS in colidx order (the same fp32 sums as
 * snd_csr_spmm_bf16, bit for bit).  If ustride exceeds the LDS image
 * (319 rows) the launch runs snd_csr_spmm_bf16's kernel instead. */
int snd_csr_spmm_bf16_tiled(const int* rowptr, const int* colidx, int n_rows,
                            const snd_row_tiles_t* tiles, const void* h, int ldh,
                            int width, void* out, int ldo, int n_per_graph,
                            int n_graphs, const int* row_order, snd_stream_t stream);
/* snd_csr_spmm_bf16 streamed through a sliding window (ABI 7): out = A @ h,
 * width 64, bf16 rows, fp32 sums in colidx order (accumulated by
 * v_dot2c_f32_bf16: within one fp32 ulp per add of snd_csr_spmm_bf16, bitwise
 * equal on every tested batch).  A workgroup walks one graph's schedule positions (e.g.
 * the per-graph RCM order) in steps of 128 rows and keeps the h rows of
 * positions [p - beta, p + 127 + beta] in a 1096-row LDS ring, filled by
 * LDS-DMA two steps ahead: every h row is read from HBM once.  The plan
 * (snd_vae_amd/data.py window_plan, host-built once per batch):
 *   meta[q]  = (start8 << 6) | degree of the row at position q (degree <= 63)
 *   slots[]  = u16 ring slot (neighbour position % 1096) per neighbour, each
 *              row's list at 8 * start8, padded with the zero row's slot 1096
 *              to a multiple of 8 and to the largest degree (<= 32) of its
 *              wavefront group (8 consecutive rows of the listing below); the
 *              kernel reads 32 entries from every list start, so the array holds
 *              24 entries past the end of the last list
 *   rows[q]  = the row whose sums position q computes, and meta[q] its meta:
 *              inside each aligned 128-position block listed by degree,
 *              descending (a wave's 8 rows then share their neighbour count)
 *   order[q] = the row at position q (the h row held at ring slot q % 1096)
 * beta = max |neighbour position - row position|; ceil8(beta) <= 352, else
 * SND_ERR_ARG (use snd_csr_spmm_bf16_tiled).  Replaces layers.py:122 (tf.matmul
 * of the dense adjacency). */
int snd_csr_spmm_bf16_window(const int* meta, const uint16_t* slots, const int* rows,
                             const int* order,
                             int n_rows, int n_per_graph, int n_graphs, int beta,
                             const void* h, int ldh, int width, void* out, int ldo,
                             snd_stream_t stream);
/* ---- a5: linear / dense GEMM on MFMA ---------------------------------------
 * Replaces linear() (layers.py:566-576) and the X@w of GraphConvolution
 * (layers.py:120-121; the tile() copy is not needed):
 *   C[m,n] = sum_k op(A)[m,k] op(B)[k,n] (+ bias[n])
 * op(A) = A (trans_a=0, A is [m,k] lda) or A^T (A is [k,m]); same for B. */
int snd_gemm(int trans_a, int trans_b, int m, int n, int k, const float* a,
             int lda, const float* b, int ldb, float* c, int ldc,
             const float* bias, int dtype, snd_stream_t stream);

/* ---- a8/a9: conv1d k=5 SAME over the node axis of each graph --------------
 * Replaces tf.layers.conv1d(k=5, stride 1, padding='SAME') + BN + lrelu
 * (model_joint.py:115-116, 138-139).  w is TF layout [5][cin][cout].
 *   fwd:  y_pre = conv(x) + bias;  out = lrelu(y_pre*g/sqrt(1.001) + b)
 *         (gamma == NULL: out = y_pre, no BN/lrelu)
 *   bwd_data:   dx = conv^T(dy)   (flipped taps, transposed channels)
 *   bwd_weight: dw[t,c,o] = sum_rows x[r+t-2,c] dy[r,o]  (deterministic
 *               split-K; workspace snd_conv1d_bwd_weight_workspace()).
 * rows = B*N, n_per_graph = N: taps never cross graph boundaries. */
int snd_conv1d_same_fwd(const float* x, int ldx, int rows, int n_per_graph,
                        int cin, const float* w, int cout, const float* bias,
                        const float* bn_gamma, const float* bn_beta,
                        float* y_pre, int ldy, float* out, int ldo, int dtype,
                        snd_stream_t stream);
int snd_conv1d_same_bwd_data(const float* dy, int lddy, int rows,
                             int n_per_graph, int cout, const float* w,
                             int cin, float* dx, int lddx, int dtype,
                             snd_stream_t stream);
size_t snd_conv1d_bwd_weight_workspace(int rows, int cin, int cout);
int snd_conv1d_same_bwd_weight(const float* x, int ldx, const float* dy,
                               int lddy, int rows, int n_per_graph, int cin,
                               int cout, float* dw, void* workspace,
                               size_t workspace_bytes, int dtype,
                               snd_stream_t stream);

/* ---- a6/a12: reparameterisation + KL --------------------------------------
 * Replaces get_z (model.py:153-161) and the KL term (optimizer.py:193).
 * ms = [mu || logstd] rows of width 2L (ld).  eps: injected [rows, L] or NULL
 * for the device Philox4x32-10 stream (seed, offset = *step_counter).
 *   z = mu + eps*exp(s)  -> z [rows, L]; eps written to eps_out if non-NULL.
 *   kl_part: snd_reparam_kl_blocks(rows, L) device doubles whose (fixed-order)
 *   sum is sum(1 + 2s - mu^2 - exp(s)^2). */
int snd_reparam_kl_blocks(int rows, int latent);
int snd_reparam_kl(const float* ms, int ldms, int rows, int latent,
                   const float* eps, unsigned long long seed,
                   const int* step_counter, float* eps_out, float* z,
                   double* kl_part, snd_stream_t stream);

/* ---- a7/a10: fused inner-product decoder + 2-class CE ----------------------
 * Replaces InnerProductDecoder (layers.py:407-409), the diagonal rule
 * (model.py:185,205-207), argmax (model.py:208), accuracy (main.py:334) and
 * softmax_cross_entropy (optimizer.py:142-144).  Logits never reach HBM.
 * For each graph b (z [B*N, d], d in {16,32,64,128}):
 *   L = z z^T; per off-diagonal pair CE = softplus(L) - A L (pos_weight,
 *   norm generalise to the weighted BCE of SURVEY §8 decision ii);
 *   diagonal pairs contribute softplus(-1) and no gradient.
 * Outputs (device): stats[0] = sum CE over all B*N*N pairs (double),
 *   stats[1] = number of pairs with argmax == A (as double),
 *   dz [B*N, d] = d(sum CE)/dz (unscaled; divide by B*N*N for the mean).
 * workspace: snd_zzt_ce_workspace() bytes. */
size_t snd_zzt_ce_workspace(int n_graphs, int n, int d, int dtype);
int snd_zzt_ce(const float* z, int n_graphs, int n, int d,
               const int* rowptr, const int* colidx, float pos_weight,
               float norm, double* stats, float* dz, void* workspace,
               size_t workspace_bytes, int dtype, snd_stream_t stream);

/* ---- a7/a10 row-sharded (SURVEY §8e "beyond DP": one N = 16384 graph over ranks) --
 * The same CE and gradient for the rows [row0, row1) of ONE graph against all N
 * columns (layers.py:407-409, optimizer.py:142-144 restricted to a row block):
 *   z       [n, d] the whole graph's latent (all-gathered by the caller);
 *   rowptr  [row1 - row0 + 1] the range's CSR row pointers (a slice of the graph's
 *           CSR is fine: offsets index colidx), colidx global column ids;
 *   stats[0] = sum CE over the range's rows x N pairs, stats[1] = #correct there;
 *   dz [row1 - row0, d] = d(sum CE over ALL pairs)/dz for the range's rows -- L is
 *   symmetric, so a rank's rows need no reduction across ranks.
 * row0 % 128 == 0 and (row1 % 128 == 0 or row1 == n).  Summing stats over a
 * partition of [0, n) gives snd_zzt_ce's stats for the graph. */
size_t snd_zzt_ce_rows_workspace(int n, int d, int row0, int row1, int dtype);
int snd_zzt_ce_rows(const float* z, int n, int d, int row0, int row1,
                    const int* rowptr, const int* colidx, float pos_weight, float norm,
                    double* stats, float* dz, void* workspace, size_t workspace_bytes,
                    int dtype, snd_stream_t stream);

/* ---- a11: sigmoid head + MSE ----------------------------------------------
 * Replaces tf.nn.sigmoid(linear(...)) (model_joint.py:121,144) and the
 * squared-difference means (optimizer.py:149,153) with their gradients:
 *   yhat = sigmoid(u @ w + b);  sse += sum (yhat - y)^2  (device double)
 *   du = dpre @ w^T with dpre = 2 (yhat - y)/count * yhat (1 - yhat),
 *   count = rows*cout (the mean's denominator).  dw/db accumulate (+=).
 *   sse: snd_sigmoid_mse_blocks(rows) device doubles (per-block partials).
 *   workspace: blocks * (cin*cout + cout) floats. */
int snd_sigmoid_mse_blocks(int rows);
int snd_sigmoid_mse(const float* u, int ldu, int rows, int cin,
                    const float* w, const float* b, int cout,
                    const float* target, int ldt, double* sse, float* yhat,
                    float* du, int lddu, float* dw, float* db, void* workspace,
                    size_t workspace_bytes, snd_stream_t stream);

/* ---- a13: TF1 Adam over a flat buffer --------------------------------------
 * Replaces tf.train.AdamOptimizer(lr).minimize (optimizer.py:125,197):
 *   t = *step_counter (1-based, already advanced for this step)
 *   g = grad*grad_scale; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2
 *   param -= lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps) */
int snd_adam_tf1(float* param, const float* grad, float* m, float* v,
                 long long n, float lr, float beta1, float beta2, float eps,
                 float grad_scale, const int* step_counter,
                 snd_stream_t stream);
/* The same update over n_ranges disjoint [offsets[k], offsets[k] + counts[k]) element
 * ranges of the same flat buffers in one launch (ABI 14; host arrays, read at call
 * time): the blocks a fused in-step update (snd_plan_fuse_adam) leaves to the caller
 * are not contiguous (C4: three ranges).  Offsets and counts that are multiples of 4
 * on 16-byte aligned buffers take one float4 launch for up to 16 ranges; anything
 * else falls back to one snd_adam_tf1 per range.  Same arithmetic either way. */
int snd_adam_tf1_ranges(float* param, const float* grad, float* m, float* v,
                        const long long* offsets, const long long* counts, int n_ranges,
                        float lr, float beta1, float beta2, float eps, float grad_scale,
                        const int* step_counter, snd_stream_t stream);

/* ---- SpatialGraphConvolution (layers.py:143-198) and the model_joint
 * spatial-graph encoder layer s' = lrelu(BN(SGConv(adj, s, rel)))
 * (model_joint.py:77-80), factorised to O(nnz (h0 + deg)) + row GEMMs (see
 * snd_sg.hip).  adj must be symmetric (spanning trees and adj_truth are;
 * input_data.py:31-37,67) with rel_dim 1 (Matrix1 has 3F+3 rows).
 * Per-layer parameter buffer (fp32, snd_sg_param_count floats), row-major:
 *   Matrix1 [3F+3][h0] (rows: x_i | x_j | x_k | rel_ij | rel_jk | dis_ik), bias1 [h0],
 *   Matrix2 [2F+1+h0][h1] (x_i | x_j | rel_ij | m3_sum), bias2 [h1],
 *   Matrix3 [F+h1][h2] (x | m2_sum), bias3 [h2], BN gamma [h2], BN beta [h2].
 * Gradients use the same layout (written, not accumulated). */
typedef struct snd_sg_graph {
  const int* rowptr;   /* [R+1] symmetric CSR, block-diagonal, sorted global ids */
  const int* colidx;   /* [nnz] */
  int n_rows;          /* R = B * n_per_graph */
  int n_per_graph;
  float* edge_lr;      /* [nnz] lrelu(rel_ij)                      (snd_sg_prep) */
  float* edge_q;       /* [nnz] sum_{k in N(j)} lrelu(rel_ik)      (snd_sg_prep) */
  int* edge_rev;       /* [nnz] index of the reverse edge (j, i)   (snd_sg_prep) */
  float* node_deg;     /* [R] degree                               (snd_sg_prep) */
  float* node_e;       /* [R] sum_{j in N(i)} lrelu(rel_ij)        (snd_sg_prep) */
} snd_sg_graph_t;
/* Edge / node scalars of a batch from rel [B, N, N] (the 'rel' feed, main.py:262,
 * /600 at load); *n_unmatched (device int) = edges without a reverse edge (must be 0). */
int snd_sg_prep(const snd_sg_graph_t* g, const float* rel, int* n_unmatched,
                snd_stream_t stream);
long long snd_sg_param_count(int f, int h0, int h1, int h2);
size_t snd_sg_workspace(int n_rows, int f, int h0, int h1, int h2);
/* y [R, h2] = SGConv(adj, x, rel); bn_act: out = lrelu(BN(y)) (frozen Keras BN).
 * The workspace keeps what snd_sg_layer_bwd needs: pass the same one. */
int snd_sg_layer_fwd(const snd_sg_graph_t* g, const float* x, int ldx, int f, int h0, int h1,
                     int h2, const float* params, int bn_act, float* y, float* out,
                     void* workspace, snd_stream_t stream);
/* dout = dL/d(out) (bn_act) or dL/dy; writes grads (param layout) and, if dx is
 * not NULL, dL/dx [R, f]. */
int snd_sg_layer_bwd(const snd_sg_graph_t* g, const float* x, int ldx, int f, int h0, int h1,
                     int h2, const float* params, int bn_act, const float* y,
                     const float* dout, float* dx, int lddx, float* grads, void* workspace,
                     snd_stream_t stream);

/* ---- §8f rank 4: disentangled-model pieces (ABI 8; not on the benchmarked path) -
 * e2e edge-to-edge filter of the structure decoder (layers.py:431-450), fp32:
 *   out[b,i,j,o] = 2 b1[o] + sum_t sum_c w1[t,c,o] (x[b,i,j+t-p,c] + x[b,i+t-p,j,c])
 * x [B, N, N, C] (NHWC), w1 [K, C, O] (the reference's [1, K, C, O] kernel; conv2
 * uses its transpose [K, 1, C, O]: the same taps), TF SAME padding p = (K-1)/2;
 * the decoder uses K = N (model.py:196).  Deterministic fixed-order sums. */
int snd_e2e_fwd(const float* x, int n_graphs, int n, int c, const float* w1, const float* b1,
                int k, int o, float* out, snd_stream_t stream);
/* dx [B, N, N, C], dw1 [K, C, O], db1 [O] of sum(out * dout). */
int snd_e2e_bwd(const float* x, int n_graphs, int n, int c, const float* w1, int k, int o,
                const float* dout, float* dx, float* dw1, float* db1, snd_stream_t stream);
/* The e2e structure decoder around the filters (model.py:193-208), fp32, frozen
 * Keras BN (y' = gamma y / sqrt(1.001) + beta) then relu:
 *   snd_e2e_pair_fwd: x0[b,i,j,:] = relu(BN0([z_i | z_j]))  (z [B, N, D] -> x0 [B, N, N, 2D])
 *   snd_bn_relu_fwd:  x = relu(BN(y)), y [rows, c]           (between e2e layers)
 *   snd_e2e_head_ce:  logits = relu(BN_adj(y)) W + b (d_e_lin2, W [c][2]), the diagonal
 *                     set to (1, 0) (model.py:200-203), CE against [1 - A, A] summed
 *                     over B N^2 (optimizer.py:142-144) into out[0], argmax == A count
 *                     (main.py:334) into out[1]; gradients of the MEAN CE: dy, dW, db,
 *                     dgamma, dbeta (c <= 32; adj dense [B, N, N] 0/1 floats)
 *   snd_bn_relu_bwd / snd_e2e_pair_bwd: the matching backward passes (per-channel
 *                     gamma / beta gradients in fixed order; the pair backward needs
 *                     snd_e2e_pair_bwd_workspace bytes). */
int snd_e2e_pair_fwd(const float* z, int n_graphs, int n, int d, const float* gamma, const float* beta,
                     float* x, snd_stream_t stream);
size_t snd_e2e_pair_bwd_workspace(int n_graphs, int n, int d);
int snd_e2e_pair_bwd(const float* dx0, const float* z, int n_graphs, int n, int d, const float* gamma,
                     const float* beta, float* dz, float* dgamma, float* dbeta, void* workspace,
                     snd_stream_t stream);
int snd_bn_relu_fwd(const float* y, long long rows, int c, const float* gamma, const float* beta, float* x,
                    snd_stream_t stream);
int snd_bn_relu_bwd(const float* dx, const float* y, long long rows, int c, const float* gamma,
                    const float* beta, float* dy, float* dgamma, float* dbeta, snd_stream_t stream);
int snd_e2e_head_ce(const float* y, const float* adj, int n_graphs, int n, int c, const float* gamma,
                    const float* beta, const float* w, const float* b, float* dy, float* dw, float* db,
                    float* dgamma, float* dbeta, double* out, snd_stream_t stream);
/* Frozen Keras BN (y' = gamma y / sqrt(1.001) + beta, model.py:41) with an activation
 * (ABI 12): act 0 identity, 1 relu, 2 lrelu(0.2) (layers.py:112-113); act_first = 1:
 * x = BN(act(y)) (GraphConvolution then BN, model.py:107), 0: x = act(BN(y)) (the
 * spatial encoder's relu after BN, model.py:123-124; identity for the disentangled
 * decoders' conv + BN, model.py:190,214).  Strided rows (ld >= c).  The backward
 * writes dy and, when non-NULL, the per-channel dgamma / dbeta (fixed-order sums). */
int snd_bn_act_fwd(const float* y, int ldy, long long rows, int c, const float* gamma,
                   const float* beta, int act, int act_first, float* x, int ldx, snd_stream_t stream);
int snd_bn_act_bwd(const float* dx, int lddx, const float* y, int ldy, long long rows, int c,
                   const float* gamma, const float* beta, int act, int act_first, float* dy, int lddy,
                   float* dgamma, float* dbeta, snd_stream_t stream);
/* Reparameterisation backward (model.py:155-159): dms = [dz + add_mu || dz eps e^s +
 * add_logstd] over ms = [mu || logstd] rows (dz / add_* may be NULL: zero). */
int snd_reparam_bwd(const float* ms, int ldms, int rows, int latent, const float* eps, const float* dz,
                    const float* add_mu, const float* add_logstd, float* dms, int lddms,
                    snd_stream_t stream);
/* y[r, c] += alpha x[r, c] over a strided [rows, cols] block: gradients of one tensor
 * reaching it along several branches (the disentangled decoders' concat inputs). */
int snd_add_strided(long long rows, int cols, float alpha, const float* x, int ldx, float* y, int ldy,
                    snd_stream_t stream);
/* Latent regularisers of one latent group (optimizer.py:7-58,159-190), mu / logstd /
 * z [batch, latent] fp32:
 *   term = w_kl kl  (cap_gamma > 0: cap_gamma relu(kl - cap_c), 'disentangled_C')
 *        + w_dip DIP(mu; lambda_od, lambda_d) + w_tc TC(z, mu, logstd)
 * kl = -0.5 mean(1 + 2s - mu^2 - e^{2s}) (optimizer.py:160); DIP optimizer.py:7-21;
 * TC the minibatch estimate of optimizer.py:29-58 (logvar = 2 logstd).  Writes
 * dmu / dlogstd = d term / d (mu, logstd) including the path through
 * z = mu + eps e^{logstd} (model.py:155-159), and out[4] (double) =
 * {kl, term, DIP, TC}.  One workgroup: sized for the reference's batches (<= a few
 * hundred latents).  workspace >= snd_latent_reg_workspace(batch, latent) bytes
 * when w_dip or w_tc is nonzero. */
typedef struct {
  float w_kl, cap_gamma, cap_c, w_dip, lambda_od, lambda_d, w_tc;
} snd_latent_reg_t;
size_t snd_latent_reg_workspace(int batch, int latent);
int snd_latent_reg(const float* mu, const float* logstd, const float* z, int batch, int latent,
                   const snd_latent_reg_t* w, float* dmu, float* dlogstd, double* out,
                   void* workspace, snd_stream_t stream);

/* ---- a14: the whole train step (main.py:315-334) ---------------------------
 * A plan fixes shapes; the step runs forward + backward of the SND-VAE
 * (SURVEY §8 "Composed step") for one batch in either decoder-input topology:
 *   SND_TSCALE  node latent: heads per node row, mu/logstd [B*N, L], J = z;
 *   SND_TREF    graph latent (model.py:113-115, model_joint.py:87-97):
 *               h = flat(G) Wh + bh per graph, z [B, L],
 *               J = reshape(z Wp + bp, [B, N, node_h]); at most 8 graphs
 *               per plan (the weight-streaming kernels keep B in registers);
 *   SND_SGJOINT the SND-VAE spatial-graph encoder (ABI 11; model_joint.py:72-85,
 *               model.py:134-151,172-180): two SpatialGraphConvolution layers
 *               (snd_sg_layer_fwd, BN + lrelu) over the B * sampling_num
 *               spanning-tree copies (batch tree_rowptr / tree_colidx / rel,
 *               features tiled per copy), flat heads per copy, z [B*S, L],
 *               J_b = mean_s reshape(z_{b,s} Wp + bp, [N, node_h]), then the
 *               graph-latent decoders; f_in = num_feature, h0/h1 unused, fp32
 *               generic engine (either dtype for the GEMM operands).
 * It writes the flat
 * gradient (same layout as params), advances *step_counter and writes
 * losses[0..7] = {cost, spatial_cost, adj_cost, node_cost, kl, acc,
 *                 adj_sum, correct} (device doubles; main.py:331-334
 * overall_loss order, optimizer.py:203).  It also writes the first six as
 * floats to grads[param_count .. +6) so one all-reduce averages them. */
typedef struct snd_config {
  int n_nodes;      /* N */
  int f_in;         /* encoder input width (num_feature + spatial_dim) */
  int num_feature;  /* node feature targets */
  int spatial_dim;  /* coordinate targets */
  int h0, h1;       /* g_conv_hidden */
  int g_hidden;     /* g_hidden_size */
  int latent;       /* L (g_latent_size) */
  int s1, s2, s3;   /* s_d_channel */
  int n1, n2;       /* n_d_channel[:2] */
  float beta;       /* KL weight */
  float pos_weight; /* 1 == reference */
  float norm;       /* 1 == reference */
  int dtype;        /* SND_F32 (parity) or SND_BF16 (throughput) */
  int topology;     /* SND_TSCALE or SND_TREF (ABI version 2) */
  int node_h;       /* width of J (node_h_size); == latent for SND_TSCALE */
  int sampling_num; /* SND_SGJOINT: spanning trees per graph (main.py:100) */
  int sg_h[6];      /* SND_SGJOINT: sg_conv_hidden [[h0,h1,h2],[h0,h1,h2]] (main.py:193) */
} snd_config_t;
enum { SND_TSCALE = 0, SND_TREF = 1, SND_SGJOINT = 2 };

/* The window SpMM's plan on the device (ABI 10; data.py window_plan, see
 * snd_csr_spmm_bf16_window): with it, the step's bf16 GraphConvolution backward
 * SpMM (A @ dP1, width 64) runs the window kernel.  meta NULL = none. */
typedef struct snd_window_plan {
  const int* meta;              /* [n_rows] */
  const uint16_t* slots;
  const int* rows;              /* [n_rows] */
  const int* order;             /* [n_rows] */
  int beta;
} snd_window_plan_t;

typedef struct snd_batch {
  const int* rowptr;           /* [B*N+1] */
  const int* colidx;           /* [nnz]   */
  const float* features;       /* [B*N, f_in] */
  const float* feature_truth;  /* [B*N, num_feature] */
  const float* spatial_truth;  /* [B*N, spatial_dim] */
  const int* row_order;        /* optional [B*N] locality schedule of the gather
                                  kernels (see snd_csr_spmm_bf16); NULL = natural */
  snd_row_tiles_t tiles;       /* optional row tiles over row_order (ABI 5; all
                                  zero = none): the bf16 encoder SpMMs stage
                                  neighbour rows in LDS */
  snd_window_plan_t window;    /* optional window SpMM plan over row_order (ABI 10) */
  /* SND_SGJOINT (ABI 11): the spanning trees of the B graphs, copy c = b * S + s of
   * graph b (input_data.py:76-83), one symmetric block-diagonal CSR over B*S*N rows;
   * rel [B*S, N, N] of each copy (the 'rel' feed / 600, input_data.py:59); features
   * are then [B*S*N, num_feature] (graph b's features in each of its copies) */
  const int* tree_rowptr;
  const int* tree_colidx;
  const float* rel;
} snd_batch_t;

typedef struct snd_plan snd_plan_t;

int snd_plan_create(const snd_config_t* cfg, int n_graphs, snd_plan_t** out);
void snd_plan_destroy(snd_plan_t* plan);
long long snd_plan_param_count(const snd_plan_t* plan);
int snd_plan_num_blocks(const snd_plan_t* plan);
int snd_plan_param_block(const snd_plan_t* plan, int idx, const char** name,
                         long long* offset, long long* numel);
size_t snd_plan_workspace_bytes(const snd_plan_t* plan);
/* Fused TF1 Adam (1 GPU: no all-reduce between gradient and update).  With m and
 * v set (flat buffers in the parameter layout), snd_train_step applies the Adam
 * update of optimizer.py:125,197 in place, through the params pointer, to the blocks
 * snd_plan_block_fused() reports nonzero; the caller's snd_adam_tf1 then covers the
 * other blocks (none on the node-latent plans).  m = v = NULL turns it off (default).
 * lr/betas/eps as snd_adam_tf1; grad_scale is 1.
 * snd_plan_block_fused (ABI 16): 0 = updated by the caller; 1 = updated inside the
 * weight-gradient stream that produces the gradient complete (graph-latent head weight,
 * d_sg_lin1 weight and bias) -- its gradient is NOT written; 2 = updated by the step's final
 * slab reduction, which writes the gradient and applies Adam to it in the same launch
 * (every block that launch writes complete), the gradient is written as usual.
 * The reduction reads the step index t = *step_counter + 1 that the step's
 * reparameterisation kernel publishes in the workspace, since the same launch's
 * finalize workgroup advances *step_counter. */
int snd_plan_fuse_adam(snd_plan_t* plan, float* m, float* v, float lr, float beta1,
                       float beta2, float eps);
int snd_plan_block_fused(const snd_plan_t* plan, int idx);
/* Bucketed data parallel (ABI 13).  Registers `event` (a hipEvent_t created by the
 * caller) to be recorded on the step's stream right after the kernel that writes
 * block idx's gradient complete, so the caller can start that bucket's collective on
 * another stream while the backward pass goes on (DP of optimizer.py:125,197 with
 * main.py:331's single update): the graph-latent d_sg_lin1 weight and
 * bias complete after the projection backward, the graph-latent head weight after
 * the head backward.  Returns k > 0, the block's completion point (blocks with the
 * same k complete together and share one event; points are reached in increasing k),
 * when it has one (the event is kept for every later snd_train_step; NULL unregisters
 * it), 0 when the block's gradient is completed by the step's final reduction
 * (nothing kept), <0 on a bad index. */
int snd_plan_grad_event(snd_plan_t* plan, int idx, void* event);
/* ABI 17: the event currently registered for block idx (NULL when none) in *event;
 * returns the block's completion point as snd_plan_grad_event does.  Lets a host
 * binding check that a freed optimizer did not unregister a newer one's events. */
int snd_plan_grad_event_get(const snd_plan_t* plan, int idx, void** event);
/* Data parallel (ABI 6): the device Philox normals of this plan's head rows start at
 * global head row `head_row_offset` (rank * n_graphs for SND_TREF, rank * n_graphs *
 * n_nodes for SND_TSCALE), so every rank of a sharded global batch draws exactly the
 * eps a single device would draw for those rows (model.py:155-159).  Default 0. */
int snd_plan_set_rng_offset(snd_plan_t* plan, long long head_row_offset);
/* Named intermediate buffers inside the workspace (tests / inspection). */
int snd_plan_buffer(const snd_plan_t* plan, const char* name,
                    long long* byte_offset, long long* numel);
int snd_train_step(const snd_plan_t* plan, const snd_batch_t* batch,
                   const float* params, float* grads, void* workspace,
                   const float* eps, unsigned long long seed,
                   int* step_counter, double* losses, snd_stream_t stream);
/* Forward-only evaluation / sampling on the plan's shapes and dtype, generic
 * kernels (main.py:358-469 generate_new / generate_new_train; model.py:163-169
 * get_random_z).  mode:
 *   SND_GEN_SAMPLE  encode `batch`, z = mu + eps exp(s) (eps_or_z = eps [RH, L]
 *                   or NULL: device Philox at (seed, *step_counter)), as in training
 *   SND_GEN_MEAN    encode `batch`, z = mu (z_mean_*, main.py:361,367)
 *   SND_GEN_PRIOR   z ~ N(0, 1) (eps_or_z = eps or NULL: Philox); batch unused
 *   SND_GEN_GIVEN   z = eps_or_z [RH, L]; batch unused
 * RH = n_graphs (SND_TREF) or n_graphs * n_nodes (SND_TSCALE).  Results stay in
 * the workspace (snd_plan_buffer): "MS" [mu || s], "Z" (node latent z / decoder
 * input J), "ZL" (graph latent z), "SHAT" generated_spatial, "XHAT"
 * generated_node_feat.  gen_adj (optional, uint8 [B, N, N]) receives
 * generated_adj: 1 iff i != j and (J J^T)_ij > 0 (argmax of the 2-class logits,
 * first index on ties, model.py:205-208).  Stream-ordered, no allocation;
 * *step_counter is read, not advanced. */
enum { SND_GEN_SAMPLE = 0, SND_GEN_MEAN = 1, SND_GEN_PRIOR = 2, SND_GEN_GIVEN = 3 };
int snd_generate(const snd_plan_t* plan, const snd_batch_t* batch, const float* params,
                 void* workspace, int mode, const float* eps_or_z, unsigned long long seed,
                 const int* step_counter, unsigned char* gen_adj, snd_stream_t stream);
/* Re-launch one kernel of the step on the workspace state left by the last
 * snd_train_step (measurement/profiling): "zzt_dense" (fused zz^T + CE),
 * "spmm_dxw1" (plain fp32 CSR SpMM, width h1; generic-engine plans),
 * "spmm_bf16" (the bf16 path's A @ dP1), "pack" / "dec:<k>" (bf16 weight
 * packing / k-th bf16 decoder kernel, k = 0..10), and on SND_TREF plans
 * "tref_head_fwd" / "tref_head_bwd" / "tref_proj_fwd" / "tref_proj_bwd"
 * (the weight-streaming heads and projection). */
int snd_plan_launch(const snd_plan_t* plan, const snd_batch_t* batch,
                    void* workspace, const char* kernel, snd_stream_t stream);
/* Measurement only: bits that make the bf16 decoder kernels skip phases
 * (1 weight staging, 2 row staging, 4 MFMA, 8 stores, 16 column params,
 * 32 epilogue prefetch) and, read by snd_plan_create, 256 = generic-engine
 * plan, 512 = generic encoder; read by snd_train_step, 1024 = run the edge
 * terms and weight gradients on a side stream.  0 (default) = normal. */
int snd_debug_set(int flags);

/* Plan options (round 4).  "conc_decoder": 1 = run the fused decoder on a side stream
 * beside the zz^T kernel (whose column splits then leave the decoder's tiles their CUs),
 * 0 = serial, -1 = auto (the default: on for graphs of N >= 2048 with at most 64
 * decoder tiles -- one or two N = 4096 graphs, C3's per-rank batch -- where neither
 * kernel fills the chip).  The
 * side stream is created by the first non-capturing step.
 * "reduce_adam" (ABI 16): 1 (default) = with snd_plan_fuse_adam set, the blocks the
 * final reduction completes take their Adam update in that launch (snd_plan_block_fused
 * 2); 0 = they are left to the caller's snd_adam_tf1 (kind 0).  Set it before
 * snd_plan_fuse_adam / the optimizer reads the kinds.
 * Returns 1 when the option is in effect for this plan, 0 when the plan cannot use it,
 * SND_ERR_ARG for an unknown option. */
int snd_plan_set_option(snd_plan_t* plan, const char* name, int value);

#ifdef __cplusplus
}
#endif
#endif /* SND_VAE_H */
