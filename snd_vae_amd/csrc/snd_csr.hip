// Adjacency ingest: dense [B,N,N] 0/1 float (the reference's adj_truth feed,
// main.py:257; built in input_data.py:62-67) -> block-diagonal CSR.
// Entry order is np.where / sparse_to_tuple row-major order (input_data.py:72,
// preprocessing.py:7-13): rows ascending, columns ascending.  Diagonal entries
// are dropped (input_data.py:65).  Three stream-ordered passes:
//   count (one block per row, HBM streaming of N floats)
//   exclusive scan of the B*N counts (single block)
//   fill  (one block per row, ballot + popcount stream compaction in order)
// HBM-bound: each dense row is read twice (count and fill).
#include "snd_common.hpp"

#include <algorithm>
#include <vector>

namespace snd {
namespace {

constexpr int NT = 256;

__global__ void __launch_bounds__(NT) csr_count_kernel(const float* adj, int n, int* counts) {
  const long long r = blockIdx.x;               // global row b*N + i
  const int i = (int)(r % n);
  const float* row = adj + r * (long long)n;
  unsigned c = 0;
  for (int j = threadIdx.x; j < n; j += NT) c += (row[j] != 0.f && j != i) ? 1u : 0u;
  c = wave_sum_u(c);
  __shared__ unsigned sh[NT / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[r] = (int)(sh[0] + sh[1] + sh[2] + sh[3]);
}

// exclusive scan of counts[0..total) into rowptr[0..total]; one block of 1024
__global__ void __launch_bounds__(1024) csr_scan_kernel(const int* counts, long long total,
                                                        int* rowptr, long long cap, int* nnz_out) {
  __shared__ long long part[1024];
  const long long chunk = (total + 1023) / 1024;
  const long long lo = threadIdx.x * chunk, hi = lo + chunk < total ? lo + chunk : total;
  long long s = 0;
  for (long long k = lo; k < hi; ++k) s += counts[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {     // Hillis-Steele inclusive scan
    long long v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  long long run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (long long k = lo; k < hi; ++k) {
    rowptr[k] = (int)run;
    run += counts[k];
  }
  if (threadIdx.x == 1023) {
    rowptr[total] = (int)part[1023];
    *nnz_out = (part[1023] > cap || part[1023] >= (1ll << 31)) ? -1 : (int)part[1023];
  }
}

__global__ void __launch_bounds__(NT) csr_fill_kernel(const float* adj, int n, const int* rowptr,
                                                      int* colidx, long long cap) {
  const long long r = blockIdx.x;
  const int i = (int)(r % n);
  const long long gbase = r - i;                 // b*N: column ids are global
  const float* row = adj + r * (long long)n;
  __shared__ int wsum[NT / 64];
  long long out = rowptr[r];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int j0 = 0; j0 < n; j0 += NT) {
    const int j = j0 + threadIdx.x;
    const bool f = j < n && row[j] != 0.f && j != i;
    const unsigned long long m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int woff = 0, tot = 0;
    for (int k = 0; k < NT / 64; ++k) {
      if (k < w) woff += wsum[k];
      tot += wsum[k];
    }
    const long long pos = out + woff + before;
    if (f && pos < cap) colidx[pos] = (int)(gbase + j);
    out += tot;
    __syncthreads();
  }
}

}  // namespace
}  // namespace snd

using namespace snd;

extern "C" size_t snd_dense_to_csr_workspace(int n_graphs, int n) {
  return (size_t)n_graphs * n * sizeof(int);
}

extern "C" int snd_dense_to_csr(const float* adj, int n_graphs, int n, int* rowptr, int* colidx,
                                long long colidx_cap, int* nnz_out, void* ws, size_t ws_bytes,
                                snd_stream_t stream) {
  SND_CHECK_ARG(adj && rowptr && nnz_out && n > 0 && n_graphs > 0, "snd_dense_to_csr: bad args");
  SND_CHECK_ARG(colidx || colidx_cap == 0, "snd_dense_to_csr: null colidx");
  SND_CHECK_ARG(ws && ws_bytes >= snd_dense_to_csr_workspace(n_graphs, n),
                "snd_dense_to_csr: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const long long rows = (long long)n_graphs * n;
  SND_CHECK_ARG(rows < (1ll << 31), "snd_dense_to_csr: too many rows");
  int* counts = (int*)ws;
  hipLaunchKernelGGL(csr_count_kernel, dim3((unsigned)rows), dim3(NT), 0, s, adj, n, counts);
  SND_LAUNCH_CHECK("csr_count_kernel");
  hipLaunchKernelGGL(csr_scan_kernel, dim3(1), dim3(1024), 0, s, counts, rows, rowptr,
                     colidx_cap, nnz_out);
  SND_LAUNCH_CHECK("csr_scan_kernel");
  if (colidx_cap > 0) {
    hipLaunchKernelGGL(csr_fill_kernel, dim3((unsigned)rows), dim3(NT), 0, s, adj, n, rowptr,
                       colidx, colidx_cap);
    SND_LAUNCH_CHECK("csr_fill_kernel");
  }
  return 0;
}

// Row tiles of the bf16 SpMM (snd_row_tiles_t; host code, once per batch).
// Tile t = schedule slots [t*tile_rows, (t+1)*tile_rows) of row_order (or the
// natural order), its rows sorted by degree (descending, stable); its set is the
// ascending distinct colidx values of those rows, and lcol maps every entry, in
// slot order, to 1 + its position in that set (0 is the kernel's zero row).
extern "C" long long snd_spmm_tile_plan(const int* rowptr, const int* colidx, int n_rows,
                                        const int* row_order, int tile_rows, int* rows, int* trp,
                                        uint16_t* lcol, int* ucol, int* ustride) {
  SND_CHECK_ARG(rowptr && n_rows >= 0 && tile_rows > 0 && ustride, "snd_spmm_tile_plan: bad args");
  const bool fill = rows || trp || lcol || ucol;
  SND_CHECK_ARG(!fill || (rows && trp && lcol && ucol), "snd_spmm_tile_plan: rows, trp, lcol, ucol go together");
  const long long nnz = rowptr[n_rows];
  SND_CHECK_ARG(colidx || nnz == 0, "snd_spmm_tile_plan: null colidx");
  const int ntiles = (n_rows + tile_rows - 1) / tile_rows;
  std::vector<int> cols, trow;
  int mx = 0;
  if (fill) SND_CHECK_ARG(*ustride >= 0, "snd_spmm_tile_plan: ustride from the sizing call");
  const int stride = fill ? *ustride : 0;
  long long k_out = 0;
  if (fill) trp[0] = 0;
  for (int t = 0; t < ntiles; ++t) {
    cols.clear();
    trow.clear();
    const int s_lo = t * tile_rows, s_hi = std::min(n_rows, (t + 1) * tile_rows);
    for (int slot = s_lo; slot < s_hi; ++slot) {
      const int r = row_order ? row_order[slot] : slot;
      SND_CHECK_ARG(r >= 0 && r < n_rows, "snd_spmm_tile_plan: row_order entry %d out of range", r);
      trow.push_back(r);
      for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) cols.push_back(colidx[k]);
    }
    std::sort(cols.begin(), cols.end());
    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    const int nu = (int)cols.size();
    SND_CHECK_ARG(nu < 65535, "snd_spmm_tile_plan: tile %d has %d distinct rows (>= 65535)", t, nu);
    mx = std::max(mx, nu);
    if (!fill) continue;
    SND_CHECK_ARG(nu <= stride, "snd_spmm_tile_plan: tile %d set %d > ustride %d", t, nu, stride);
    std::stable_sort(trow.begin(), trow.end(), [&](int x, int y) {
      return rowptr[x + 1] - rowptr[x] > rowptr[y + 1] - rowptr[y];
    });
    int* uc = ucol + (long long)t * stride;
    std::copy(cols.begin(), cols.end(), uc);
    std::fill(uc + nu, uc + stride, -1);
    for (int i = 0; i < (int)trow.size(); ++i) {
      const int r = trow[i];
      rows[s_lo + i] = r;
      for (int k = rowptr[r]; k < rowptr[r + 1]; ++k)
        lcol[k_out++] = (uint16_t)(1 + (std::lower_bound(cols.begin(), cols.end(), colidx[k]) - cols.begin()));
      trp[s_lo + i + 1] = (int)k_out;
    }
  }
  if (!fill) *ustride = mx;
  const long long len = (long long)ntiles * (fill ? stride : mx);
  SND_CHECK_ARG(len < (1ll << 31), "snd_spmm_tile_plan: tile sets beyond 2^31 entries");
  return len;
}
