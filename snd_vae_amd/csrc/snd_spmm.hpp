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
};
int edge_blocks(int n_rows, int d);
int launch_edge(const EdgeArgs& a, hipStream_t s);

}  // namespace snd
