#pragma once
#include "snd_common.hpp"

namespace snd {

struct ZztArgs {
  const void* jrow;      // [B][npad][DP] z * sqrt(log2 e)   (bf16 or f32)
  const void* jt;        // [B][DP][npad] z^T                (bf16 or f32)
  int n, npad, ngraphs, d;
  float* dJd;            // [B*n][d]  sum_{j != i} sigmoid(L_ij) z_j
  double* part;          // [blocks][2] = {sum softplus over valid pairs, #{L > 0}}
  const float* colpart;  // [B][npad/64][DP] column sums of jrow (bf16 values), per 64 rows
  int variant;           // bf16 kernel: 0 = default (v4 for d <= 64, v7 for d = 128), 1 = v1
                         // (the bench's previous variant); >= 256 the measurement build of the
                         // default (phase-skip / stamp bits variant >> 8, tools/zzt_stamps.py)
  float* dJd_extra;      // v3 column splits 1.. (zzt_tsplit > 1): [(tsplit-1)][B*n][d] scratch
  int rb0 = 0;           // first 128-row block of the launch (row-sharded zz^T, snd_zzt_ce_rows)
  int nrb = 0;           // row blocks of the launch; 0 = every row block
  int tsplit = 0;        // column splits of the default bf16 kernel; 0 = zzt_tsplit's choice
};

// Staging buffers carved from one workspace region.
struct ZztStage {
  void* jrow;
  void* jt;
  float* colpart;
};

int zzt_dp(int d);
int zzt_npad(int n);
// Small batches (fewer row blocks than CUs) split the column range of every row
// block over zzt_tsplit() workgroups (bf16 only); their partial dJ rows are summed
// in fixed order by launch_zzt_dense.  Loss partials: zzt_dense_blocks() entries.
int zzt_tsplit(int ngraphs, int n, int dtype);
int zzt_tsplit_blocks(int row_blocks, int n, int dtype);   // the same for a row-block count
int zzt_dense_blocks(int ngraphs, int n, int d, int dtype);
int zzt_wpb(int d, int dtype);   // loss partials per 128-row block and split (v9: 2)
size_t zzt_staging_bytes(int ngraphs, int n, int d, int dtype);
ZztStage zzt_stage(void* base, int ngraphs, int n, int d, int dtype);
int zzt_init_attributes();
int launch_zzt_prep(const float* z, int ngraphs, int n, int d, int dtype, const ZztStage& st,
                    hipStream_t s);
// defer_split: column splits (zzt_tsplit > 1) leave their partial dJ in dJd_extra for
// the consumer to add (head_bwd_kernel, in the same fixed order) instead of launching
// zzt_split_sum_kernel
int launch_zzt_dense(const ZztArgs& a, int dtype, hipStream_t s, bool defer_split = false);

}  // namespace snd
