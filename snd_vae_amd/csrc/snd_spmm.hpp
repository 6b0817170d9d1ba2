#pragma once
#include "snd_common.hpp"

namespace snd {

struct SpmmArgs {
  const int* rowptr; const int* colidx; int n_rows;
  const float* h; int ldh; int width;
  float* out; int ldo;
  int epilogue;
  const float* gamma; const float* beta; float* pre; int ldp;
  const float* x; int ldx; int fx;
  const float* gamma2; const float* beta2; float* out2; int ldo2;
};
int launch_spmm(const SpmmArgs& a, hipStream_t s);

struct EdgeArgs {
  const int* rowptr; const int* colidx; int n_rows;
  const float* z; int d;        // row-major [n_rows, d]
  float pos_weight;
  float* ej;                    // [n_rows, d]
  double* part;                 // [blocks][2] = {loss, tp}
  int row0 = 0;                 // z row of local row 0 (row-sharded zz^T): z_i = z[row0 + r]
};
int edge_blocks(int n_rows, int d);
int launch_edge(const EdgeArgs& a, hipStream_t s);

}  // namespace snd

namespace snd {
// the sliding-window bf16 SpMM (snd_spmm_win.hip; plan: data.window_plan)
struct SpmmWinArgs {
  const int* meta; const uint16_t* slots; const int* rows; const int* order; int beta;
  int n_rows, n_per_graph, n_graphs;
  const void* h; int ldh; int width;
  void* out; int ldo;
};
int launch_spmm_window(const SpmmWinArgs& w, hipStream_t s);
int spmm_win_max_beta();
}  // namespace snd
