// The SND-VAE train step as one stream-ordered launch sequence (main.py:315-334).
//
// snd_plan fixes the shapes of one device batch (B graphs x N nodes), the flat
// parameter layout (same order and 64-float alignment as
// snd_vae_amd/params.py::flat_layout) and a workspace map of every
// intermediate.  snd_train_step enqueues forward + hand-derived backward
// (~40 kernels, no allocation, no host sync) so the caller can capture it,
// together with the RCCL gradient all-reduce and snd_adam_tf1, into one HIP
// graph.  Forward/backward equations: SURVEY.md §8 "Composed step";
// oracle/ref_numpy.py restates them in float64.
#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "snd_dec.hpp"
#include "snd_decode.hpp"
#include "snd_elem.hpp"
#include "snd_fast.hpp"
#include "snd_gemm.hpp"
#include "snd_head.hpp"
#include "snd_spmm.hpp"
#include "snd_tref.hpp"
#include "snd_sg.hpp"
#include "snd_zzt.hpp"

namespace snd {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {

struct Block { std::string name; long long off, numel; };
struct Buf { std::string name; long long off, numel; };

// wgrad GEMM split-K geometry
struct Split { int splits, kchunk; };
Split wgrad_split(int M, int N, int R) {
  const int tiles = cdiv(M, 64) * cdiv(N, 64);
  int s = cdiv(512, tiles);
  const int smax = cdiv(R, 256);
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  const int kchunk = (int)round_up(cdiv(R, s), kGemmBK);
  return {cdiv(R, kchunk), kchunk};
}

// padded K of a packed image (16-byte chunk swizzle supports 32 / 64 / 128)
int kp_of(int k) { return k <= 32 ? 32 : (k <= 64 ? 64 : (k <= 128 ? 128 : -1)); }

struct Img { int T, kp, np; long long off; };

}  // namespace
}  // namespace snd

using namespace snd;

struct snd_plan {
  snd_config_t c;
  int B, N, R;
  int W, C1;                   // enc width, fused first decoder conv width
  bool tref = false;           // graph latent (SND_TREF, and SND_SGJOINT's decoder side)
  bool sg = false;             // SND_SGJOINT: spatial-graph encoder over B*S spanning-tree copies
  int S = 1;                   // SND_SGJOINT: copies (spanning trees) per graph
  long long RS = 0;            // SND_SGJOINT: encoder rows B*S*N
  int sgf[2] = {0, 0};         // SND_SGJOINT: each SG layer's input width
  int dj = 0;                  // width of J (decoder / zz^T input)
  int RH = 0;                  // rows of the head tensors h, [mu || s], z: B (tref) or R
  std::vector<Block> blocks;
  long long pcount = 0;
  std::vector<Buf> bufs;
  long long ws = 0;
  // split geometry of the weight-gradient GEMMs
  Split sW0, sW1, sWh, sWms, sK1, sK2s, sK2n, sK3s;
  // ---- bf16 fast decoder (snd_fast.hip)
  bool fast = false;
  bool dec_fused = false;      // fused decoder (snd_dec.hip): 2 launches instead of 7
  int dtiles = 0;
  ColMap m1{}, m2{};
  int ld1 = 0, ld2 = 0, ld3 = 0;
  Img pk1f{}, pk2f{}, pk3f{}, pk3b{}, pk2b{}, pk1b{};
  WgGeom gK1{}, gK2s{}, gK2n{}, gK3s{};
  // ---- bf16 fast encoder (snd_fast_enc.hip + row engine)
  bool fast_enc = false;
  bool head_fused = false;     // fused encoder forward tail (snd_head.hip): 1 launch instead of 4
  bool head_bwd = false;       // fused edge terms + encoder backward head (snd_head.hip): 1 instead of 4
  bool edge_reparam = false;   // without it: per-edge terms + reparam backward in one launch (snd_fast_enc.hip)
  bool front_fused = false;    // gcn0 + H1 W1 + the weight images in one launch (snd_head.hip)
  bool pack_in_gcn0 = false;   // else the weight images inside the gcn0 launch (no pack_kernel)
  bool enc0_gather = false;    // A @ dP1 gathered inside the RC_ENC0 launch (no SpMM launch)
  bool small_head = false;     // graph latent: [mu || s] head + reparameterisation (snd_elem.hip small_head_*)
  int ldh1 = 0, ldg = 0;
  Img pw1f{}, pwhf{}, pwmsf{}, pwmsb{}, pwhb{}, pw1b{};
  Img pidg{};                  // graph latent: identity [W -> W] (dG enters RC_ENC1 directly)
  WgGeom gWms{}, gWh{}, gW1{}, gW0{};
  // wide encoders (d = 128, C5): H1 = [B0 | X] and G are h + f > 128 columns wide -- the
  // images hold the first kw1 / kwh input rows, the f feature rows enter as the row
  // engine's K tail and as separate tail weight gradients; [mu | logstd] (2L = 256) is
  // differentiated in nms-column halves
  int kw1 = 0, kwh = 0, nms = 0;
  WgGeom gW1t{}, gWht{};
  // fused TF1 Adam (snd_plan_fuse_adam): Adam state of the blocks updated inside the step
  float* fuse_m = nullptr; float* fuse_v = nullptr;
  float fuse_lr = 0.f, fuse_b1 = 0.f, fuse_b2 = 0.f, fuse_eps = 0.f;
  // bucketed data parallel (snd_plan_grad_event): events recorded on the step stream
  // right after the kernel that writes a block's gradient complete (graph latent:
  // tref_proj_bwd -> dec.Wp, dec.bp; tref_head_bwd -> enc.Wh)
  hipEvent_t ev_proj = nullptr, ev_head = nullptr;
  int grad_point(const std::string& n) const {   // 1 proj, 2 head, 0 the final reduction
    if (!tref) return 0;
    if (n == "dec.Wp" || n == "dec.bp") return 1;
    if (n == "enc.Wh" && !sg) return 2;
    return 0;
  }
  // Philox row offset of this plan's head rows (snd_plan_set_rng_offset): a data-parallel
  // rank draws the normals a single device would draw for its rows of the global batch
  unsigned long long rng_row0 = 0;
  unsigned long long eps_base() const { return rng_row0 * (unsigned long long)c.latent; }
  // blocks updated inside a weight-gradient stream (graph latent: gradient not written)
  bool stream_fused(const std::string& n) const {
    return fuse_m && tref && (n == "dec.Wp" || n == "dec.bp" || (n == "enc.Wh" && !sg));
  }
  // blocks whose every element the step's final reduction writes exactly once
  // (reduce_adam_cover, at snd_plan_fuse_adam): with fuse_m their Adam update rides in
  // that launch (ReduceAdam), gradient still written
  std::vector<char> radam;
  bool reduce_adam = true;   // plan option "reduce_adam"
  bool reduce_fused(size_t i) const { return fuse_m && reduce_adam && i < radam.size() && radam[i]; }
  // 0 separate Adam, 1 fused into a stream, 2 fused into the final reduction
  int fused_kind(size_t i) const {
    return stream_fused(blocks[i].name) ? 1 : (reduce_fused(i) ? 2 : 0);
  }
  // parameters of the last snd_train_step (snd_plan_launch re-runs kernels on them)
  mutable const float* last_params = nullptr;
  mutable float* last_grads = nullptr;
  mutable std::vector<WgArgs> last_wq;   // the last step's weight-gradient launch (snd_plan_launch)
  // side stream for the independent branches (edge terms, weight gradients); created
  // by the first non-capturing fast-path step, joined back before the reduction
  // concurrent decoder (snd_plan_set_option "conc_decoder"): with B small the zz^T
  // kernel's column splits and the decoder's 32-64 tiles do not both fill the chip, so the
  // fused decoder runs on the side stream beside zz^T, which leaves it dec_tiles CUs
  // (zzt_ts: the column splits every zz^T consumer uses -- launch, split sum, finalize)
  // (default -1 = auto: on for graphs of N >= 2048 with at most 64 128-row tiles, i.e. one
  // or two N = 4096 graphs; C3's one-graph step 0.1704 -> 0.1626 ms,
  // profiles/r04_bench_strong_conc.json.  Small graphs stay serial: launch-bound)
  int conc_dec = -1;
  int zzt_ts = 1;        // zz^T column splits of a serial step
  int zzt_ts_conc = 1;   // ... of a step whose decoder runs beside zz^T (cdec)
  mutable int last_zts = 1;   // the split count the last snd_train_step used (snd_plan_launch)
  bool conc_dec_on() const {
    return (conc_dec > 0 || (conc_dec < 0 && B * ((N + 127) / 128) <= 64 && N >= 2048)) && fast && dec_fused && !tref;
  }
  static constexpr int kEvents = 16;
  mutable hipStream_t side = nullptr;
  mutable hipEvent_t ev[kEvents] = {};
  mutable int conc = 0;   // 0 untried, 1 available, -1 unavailable
  ~snd_plan() {
    if (conc == 1) {
      for (auto& e : ev) if (e) (void)hipEventDestroy(e);
      (void)hipStreamDestroy(side);
    }
  }

  long long blk(const char* n) const {
    for (auto& b : blocks) if (b.name == n) return b.off;
    return -1;
  }
  long long buf(const char* n) const {
    for (auto& b : bufs) if (b.name == n) return b.off;
    return -1;
  }
  long long buf_numel(const char* n) const {
    for (auto& b : bufs) if (b.name == n) return b.numel;
    return 0;
  }
  void add_block(const char* n, long long numel) {
    blocks.push_back({n, pcount, numel});
    pcount += round_up(numel, 64);
  }
  void add_buf(const char* n, long long numel, int esize = 4) {
    bufs.push_back({n, ws, numel});
    ws += round_up(numel * esize, 256);
  }
};

extern "C" const char* snd_last_error(void) { return g_err; }
extern "C" int snd_abi_version(void) { return SND_ABI_VERSION; }

// zz^T column splits with the concurrent decoder on: zz^T keeps the CUs the decoder's
// tiles do not take (one 1024-thread workgroup per CU for either kernel).  A step uses
// this count only when its decoder actually runs on the side stream (cdec); a serial
// step -- a capture before any eager step, or no side stream -- keeps the full count.
#ifndef SND_CONC_TS_EXTRA
#define SND_CONC_TS_EXTRA 0   // A/B builds: zz^T splits beyond the CUs the decoder leaves free
#endif
static void set_zzt_splits(snd_plan& p) {
  p.zzt_ts = zzt_tsplit(p.B, p.N, p.c.dtype);
  p.zzt_ts_conc = p.zzt_ts;
  if (p.conc_dec_on()) {
    const int wgs = p.B * (zzt_npad(p.N) / 128);
    p.zzt_ts_conc = std::max(1, std::min(p.zzt_ts, (device_cu_count() - p.dtiles) / wgs + SND_CONC_TS_EXTRA));
  }
}

extern "C" int snd_plan_create(const snd_config_t* cfg, int n_graphs, snd_plan_t** out) {
  SND_CHECK_ARG(cfg && out && n_graphs > 0, "snd_plan_create: bad args");
  const snd_config_t& c = *cfg;
  SND_CHECK_ARG(c.topology == SND_TSCALE || c.topology == SND_TREF || c.topology == SND_SGJOINT,
                "snd_plan_create: bad topology");
  const bool sg = c.topology == SND_SGJOINT;
  const bool tref = c.topology != SND_TSCALE;
  SND_CHECK_ARG(c.n_nodes > 0 && c.f_in > 0 && (sg || (c.h0 > 0 && c.h1 > 0)) && c.g_hidden > 0,
                "snd_plan_create: non-positive width");
  if (sg) {
    bool ok = c.sampling_num > 0 && c.f_in == c.num_feature;
    for (int i = 0; i < 6; ++i) ok = ok && c.sg_h[i] > 0 && c.sg_h[i] <= 256;
    SND_CHECK_ARG(ok, "snd_plan_create: SND_SGJOINT needs sampling_num > 0, sg_h[6] in (0, 256] and "
                      "f_in == num_feature");
    SND_CHECK_ARG((long long)n_graphs * c.sampling_num <= 4096, "snd_plan_create: B * sampling_num <= 4096");
  }
  const int dj = c.node_h;
  SND_CHECK_ARG(dj == 16 || dj == 32 || dj == 64 || dj == 128,
                "snd_plan_create: node_h %d not in {16,32,64,128}", dj);
  SND_CHECK_ARG(tref || c.latent == dj, "snd_plan_create: node latent needs latent == node_h");
  SND_CHECK_ARG(!tref || (n_graphs <= kTrefMaxB && c.latent <= 128 && c.g_hidden % 4 == 0 &&
                          c.g_hidden <= 128),
                "snd_plan_create: graph latent needs <= %d graphs, latent <= 128, g_hidden %% 4 <= 128",
                kTrefMaxB);
  SND_CHECK_ARG(sg || (c.h0 <= 128 && c.h1 <= 128), "snd_plan_create: g_conv_hidden <= 128");
  SND_CHECK_ARG((sg || c.h1 + c.f_in <= 256) && c.s1 + c.n1 <= 256, "snd_plan_create: width <= 256");
  SND_CHECK_ARG(c.s3 <= 64 && c.n2 <= 64 && c.spatial_dim <= 4 && c.num_feature <= 4,
                "snd_plan_create: head widths");
  SND_CHECK_ARG(c.dtype == SND_F32 || c.dtype == SND_BF16, "snd_plan_create: bad dtype");
  SND_CHECK_ARG((long long)n_graphs * c.n_nodes < (1ll << 30), "snd_plan_create: batch too large");
  snd_plan* p = new (std::nothrow) snd_plan();
  if (!p) { set_error("snd_plan_create: out of memory"); return SND_ERR_ARG; }
  p->c = c;
  p->B = n_graphs; p->N = c.n_nodes; p->R = n_graphs * c.n_nodes;
  p->W = sg ? c.sg_h[5] : c.h1 + c.f_in;
  p->C1 = c.s1 + c.n1;
  p->tref = tref;
  p->sg = sg;
  p->S = sg ? c.sampling_num : 1;
  p->RS = (long long)n_graphs * p->S * c.n_nodes;
  p->dj = dj;
  p->RH = tref ? n_graphs * p->S : p->R;
  const int f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, L = c.latent;
  const int W = p->W, C1 = p->C1;
  const long long R = p->R, RH = p->RH;
  // ---- flat parameter layout (params.py::block_shapes order)
  if (sg) {   // SpatialGraphConvolution layers (snd_sg_param_count layout each)
    p->sgf[0] = f;
    p->sgf[1] = c.sg_h[2];
    p->add_block("enc.sg0", snd_sg_param_count(f, c.sg_h[0], c.sg_h[1], c.sg_h[2]));
    p->add_block("enc.sg1", snd_sg_param_count(c.sg_h[2], c.sg_h[3], c.sg_h[4], c.sg_h[5]));
  } else {
    p->add_block("enc.W0", (long long)f * h0);
    p->add_block("enc.bn0.gamma", h0);
    p->add_block("enc.bn0.beta", h0);
    p->add_block("enc.W1", (long long)(h0 + f) * h1);
    p->add_block("enc.bn1.gamma", h1);
    p->add_block("enc.bn1.beta", h1);
    p->add_block("enc.bne.gamma", W);
    p->add_block("enc.bne.beta", W);
  }
  p->add_block("enc.Wh", (tref ? (long long)p->N * W : W) * gh);
  p->add_block("enc.bh", gh);
  p->add_block("enc.Wms", (long long)gh * 2 * L);
  p->add_block("enc.bms", 2 * L);
  if (tref) {
    p->add_block("dec.Wp", (long long)L * p->N * dj);
    p->add_block("dec.bp", (long long)p->N * dj);
  }
  p->add_block("dec.K1", 5LL * dj * C1);
  p->add_block("dec.b1", C1);
  p->add_block("dec.bn1.gamma", C1);
  p->add_block("dec.bn1.beta", C1);
  p->add_block("dec.K2s", 5LL * c.s1 * c.s2);
  p->add_block("dec.b2s", c.s2);
  p->add_block("dec.bn2s.gamma", c.s2);
  p->add_block("dec.bn2s.beta", c.s2);
  p->add_block("dec.K2n", 5LL * c.n1 * c.n2);
  p->add_block("dec.b2n", c.n2);
  p->add_block("dec.bn2n.gamma", c.n2);
  p->add_block("dec.bn2n.beta", c.n2);
  p->add_block("dec.K3s", 5LL * c.s2 * c.s3);
  p->add_block("dec.b3s", c.s3);
  p->add_block("dec.bn3s.gamma", c.s3);
  p->add_block("dec.bn3s.beta", c.s3);
  p->add_block("dec.Ws", (long long)c.s3 * c.spatial_dim);
  p->add_block("dec.bs", c.spatial_dim);
  p->add_block("dec.Wn", (long long)c.n2 * c.num_feature);
  p->add_block("dec.bn", c.num_feature);

  // ---- workspace
  p->add_buf("XW0", R * h0);  p->add_buf("P0", R * h0);  p->add_buf("H1", R * (h0 + f));
  p->add_buf("XW1", R * h1);  p->add_buf("P1", R * h1);  p->add_buf("H2", R * W);
  p->add_buf("G", R * W);     p->add_buf("Hh", RH * gh); p->add_buf("MS", RH * 2 * L);
  p->add_buf("EPS", RH * L);  p->add_buf("Z", R * dj);
  p->add_buf("ZSTAGE", (long long)zzt_staging_bytes(p->B, p->N, dj, c.dtype), 1);
  p->add_buf("DJD", R * dj);  p->add_buf("EJ", R * dj);
  p->add_buf("DJDX", std::max(1LL, (zzt_tsplit(p->B, p->N, c.dtype) - 1) * R * dj));
  p->add_buf("Y1", R * C1);   p->add_buf("U1", R * C1);
  p->add_buf("Y2S", R * c.s2); p->add_buf("U2S", R * c.s2);
  p->add_buf("Y2N", R * c.n2); p->add_buf("U2N", R * c.n2);
  p->add_buf("Y3S", R * c.s3); p->add_buf("U3S", R * c.s3);
  p->add_buf("SHAT", R * c.spatial_dim); p->add_buf("XHAT", R * c.num_feature);
  p->add_buf("DU3S", R * c.s3); p->add_buf("DY3S", R * c.s3);
  p->add_buf("DU2S", R * c.s2); p->add_buf("DY2S", R * c.s2);
  p->add_buf("DU2N", R * c.n2); p->add_buf("DY2N", R * c.n2);
  p->add_buf("DU1", R * C1);  p->add_buf("DY1", R * C1);  p->add_buf("DZDEC", R * dj);
  p->add_buf("DMS", RH * 2 * L); p->add_buf("DH", RH * gh); p->add_buf("DG", R * W);
  p->add_buf("DP1", R * h1);  p->add_buf("DXW1", R * h1); p->add_buf("DH1", R * h0);
  p->add_buf("DP0", R * h0);  p->add_buf("DXW0", R * h0);
  const int nz = zzt_dense_blocks(p->B, p->N, dj, c.dtype), ne = edge_blocks(p->R, dj);
  const int nk = reparam_blocks(p->RH, L), nh = head_blocks(p->R), nc = col_blocks(p->R);
  p->add_buf("PZZT", 2LL * nz, 8); p->add_buf("PEDGE", 2LL * std::max({ne, edge_bf16_blocks(p->R), head_tiles(p->R)}), 8); p->add_buf("PKL", std::max({nk, reparam_prep_blocks(p->B, zzt_npad(p->N)), small_head_fwd_blocks(c.latent)}), 8);
  p->add_buf("STEPN", 1);   // *step + 1, for the fused-Adam reduction (ReduceAdam)
  p->add_buf("PSSES", nh, 8); p->add_buf("PSSEN", nh, 8);
  p->add_buf("PHS", (long long)nh * (c.s3 * c.spatial_dim + c.spatial_dim));
  p->add_buf("PHN", (long long)nh * (c.n2 * c.num_feature + c.num_feature));
  p->add_buf("PDEC3", (long long)nc * 3 * c.s3); p->add_buf("PDEC2S", (long long)nc * 3 * c.s2);
  p->add_buf("PDEC2N", (long long)nc * 3 * c.n2); p->add_buf("PDEC1", (long long)nc * 3 * C1);
  p->add_buf("PENC1", (long long)nc * (2 * W + 2 * h1)); p->add_buf("PENC0", (long long)nc * 2 * h0);
  p->sW0 = wgrad_split(f, h0, p->R);
  p->sW1 = wgrad_split(h0 + f, h1, p->R);
  p->sWh = sg ? wgrad_split((int)std::min<long long>((long long)p->N * W + 1, 1 << 30), gh, (int)RH)
             : wgrad_split(W + 1, gh, p->R);
  p->sWms = wgrad_split(gh + 1, 2 * L, p->RH);
  // graph latent on <= 16 head rows: the Wms GEMM with the reparameterisation (one launch)
  // and their backward (two launches) instead of five generic launches
  p->small_head = tref && small_head_supported(p->RH, gh, L) && p->sWms.splits == 1;
  p->sK1 = wgrad_split(5 * dj, C1, p->R);
  p->sK2s = wgrad_split(5 * c.s1, c.s2, p->R);
  p->sK2n = wgrad_split(5 * c.n1, c.n2, p->R);
  p->sK3s = wgrad_split(5 * c.s2, c.s3, p->R);
  p->add_buf("SW0", (long long)p->sW0.splits * f * h0);
  p->add_buf("SW1", (long long)p->sW1.splits * (h0 + f) * h1);
  p->add_buf("SWH", (long long)p->sWh.splits * ((sg ? (long long)p->N * W : W) + 1) * gh);
  p->add_buf("SWMS", (long long)p->sWms.splits * (gh + 1) * 2 * L);
  p->add_buf("SK1", (long long)p->sK1.splits * 5 * dj * C1);
  if (sg) {   // spatial-graph encoder over the B*S copies (snd_sg.hip)
    const long long RS = p->RS, nnz = 2LL * (p->N - 1) * n_graphs * p->S;   // spanning forests
    const int* h = c.sg_h;
    p->add_buf("SGLR", std::max(1LL, nnz)); p->add_buf("SGQ", std::max(1LL, nnz));
    p->add_buf("SGREV", std::max(1LL, nnz)); p->add_buf("SGDEG", RS); p->add_buf("SGE", RS);
    p->add_buf("SGBAD", 1);
    p->add_buf("SGY1", RS * h[2]); p->add_buf("SGX1", RS * h[2]); p->add_buf("SGDX1", RS * h[2]);
    p->add_buf("SGY2", RS * W);    p->add_buf("SGG", RS * W);      p->add_buf("SGDG", RS * W);
    p->add_buf("SGWS0", (long long)snd_sg_workspace((int)RS, f, h[0], h[1], h[2]), 1);
    p->add_buf("SGWS1", (long long)snd_sg_workspace((int)RS, h[2], h[3], h[4], h[5]), 1);
    p->add_buf("ZBAR", (long long)n_graphs * L); p->add_buf("DZBAR", (long long)n_graphs * L);
  }
  if (tref) {   // graph-latent heads / projection (snd_tref.hip)
    p->add_buf("ZL", RH * L);   p->add_buf("DZL", RH * L);
    p->add_buf("PHF", (long long)tref_head_fwd_blocks((long long)p->N * W, gh) * RH * gh);
    p->add_buf("PDZ", (long long)tref_proj_bwd_blocks((long long)p->N * dj) * RH * L);
  }
  p->add_buf("SK2S", (long long)p->sK2s.splits * 5 * c.s1 * c.s2);
  p->add_buf("SK2N", (long long)p->sK2n.splits * 5 * c.n1 * c.n2);
  p->add_buf("SK3S", (long long)p->sK3s.splits * 5 * c.s2 * c.s3);

  const int dbg = debug_flags();
  // row chunks per weight gradient: the step launches them all at once (debug bit
  // 4096 or 8192: one launch each with the ~256-workgroup geometry; 16384: 32 chunks).
  // 64 chunks measured best at C2 (32: 35.0 vs 28.8 us; 128: step 0.260 vs 0.252 ms).
  // A one-round geometry (~256 workgroups split over the segments by staged bytes) ran
  // slower, 43 vs 29 us at C2: a workgroup's 128-row units are one DMA round trip each.
  // Under 32768 rows (C5's one N = 16384 graph) 32 chunks: half the slab bytes for the
  // reduction, still >= 384 workgroups (C5 step 0.417 vs 0.403 ms).
#ifndef SND_WGC_SMALL
#define SND_WGC_SMALL 32   // A/B builds: -DSND_WGC_SMALL=16
#endif
  // Per-width counts at C2 (32 or 48 chunks for the k = 1 weights, 96 for the k = 5
  // convolutions) measured slower: wgrad_multi 26.9-30.4 vs 23.7 us
  // (profiles/r06_ab_wgrad_chunks.txt).
  const int wgc = (dbg & (4096 | 8192)) ? 0 : ((dbg & 16384) ? 32 : (R < 32768 ? SND_WGC_SMALL : 64));
  auto wgc_of = [&](int, int, int) { return wgc; };
  // ---- bf16 fast decoder: split [s | n] column layouts, packed weight images
  if (c.dtype == SND_BF16 && !sg && !(debug_flags() & 256)) {
    const ColMap m1 = colmap_split(c.s1, c.n1), m2 = colmap_split(c.s2, c.n2);
    const int w1 = m1.phys(), w2 = m2.phys();
    auto img = [&](int kin, int nout) {
      Img m{5, kp_of(kin), (int)round_up(nout, 16), 0};
      return m;
    };
    Img ims[6] = {img(dj, w1), img(w1, w2), img(c.s2, c.s3), img(c.s3, c.s2), img(w2, w1), img(w1, dj)};
    bool ok = heads_fast_supported(c.s3, c.spatial_dim) && heads_fast_supported(c.n2, c.num_feature) &&
              w1 <= 128;
    for (auto& m : ims)   // images over the LDS budget run in column windows (rc_cols_per_block)
      ok = ok && m.kp > 0 && m.np <= 128 && rc_cols_per_block(m.T, m.kp, m.np) > 0;
    if (ok) {
      p->fast = true;
      p->m1 = m1; p->m2 = m2;
      // row pitch of the decoder activations (A/B build knob SND_LD_ALIGN: elements)
#ifndef SND_LD_ALIGN
#define SND_LD_ALIGN 8
#endif
      p->ld1 = (int)round_up(w1, SND_LD_ALIGN); p->ld2 = (int)round_up(w2, SND_LD_ALIGN);
      p->ld3 = (int)round_up(c.s3, 8);
      const char* nm[6] = {"PK1F", "PK2F", "PK3F", "PK3B", "PK2B", "PK1B"};
      for (int i = 0; i < 6; ++i) {
        p->add_buf(nm[i], (long long)pack_bytes(ims[i].T, ims[i].kp, ims[i].np), 1);
        ims[i].off = p->bufs.back().off;
      }
      p->pk1f = ims[0]; p->pk2f = ims[1]; p->pk3f = ims[2];
      p->pk3b = ims[3]; p->pk2b = ims[4]; p->pk1b = ims[5];
      p->add_buf("ZERO", 64);           // never written: LDS-DMA zero source
      p->add_buf("ZB", R * dj, 2);
      p->add_buf("FY1", R * p->ld1);    p->add_buf("FU1", R * p->ld1, 2);
      p->add_buf("FY2", R * p->ld2);    p->add_buf("FU2", R * p->ld2, 2);
      p->add_buf("FY3", R * p->ld3);    p->add_buf("FU3", R * p->ld3);
      p->add_buf("FDY3", R * p->ld3, 2); p->add_buf("FDY2", R * p->ld2, 2);
      p->add_buf("FDY1", R * p->ld1, 2);
      const int rcb = rc_blocks(p->R), hb = heads_fast_blocks(p->R);
      p->add_buf("PFDEC2S", (long long)rcb * 3 * c.s2);
      p->add_buf("PFDEC1", (long long)rcb * 3 * w1);
      p->add_buf("PFHS", (long long)hb * heads_fast_parts(c.s3, c.spatial_dim));
      p->add_buf("PFHN", (long long)hb * heads_fast_parts(c.n2, c.num_feature));
      p->gK1 = wgrad_geom(p->R, 5, dj, w1, wgc_of(5, dj, w1));
      p->gK2s = wgrad_geom(p->R, 5, c.s1, c.s2, wgc_of(5, c.s1, c.s2));
      p->gK2n = wgrad_geom(p->R, 5, c.n1, c.n2, wgc_of(5, c.n1, c.n2));
      p->gK3s = wgrad_geom(p->R, 5, c.s2, c.s3, wgc_of(5, c.s2, c.s3));
      p->add_buf("FSK1", (long long)p->gK1.gx * 5 * dj * wgrad_n4(w1));
      p->add_buf("FSK2S", (long long)p->gK2s.gx * 5 * c.s1 * wgrad_n4(c.s2));
      p->add_buf("FSK2N", (long long)p->gK2n.gx * 5 * c.n1 * wgrad_n4(c.n2));
      p->add_buf("FSK3S", (long long)p->gK3s.gx * 5 * c.s2 * wgrad_n4(c.s3));
      auto dimg = [&](const Img& im) { return DecImg{nullptr, im.kp, im.np}; };
      if (!(dbg & 32768) &&
          dec_fused_supported(dj, m1, m2, c.s3, c.spatial_dim, c.num_feature, dimg(p->pk1f), dimg(p->pk2f),
                              dimg(p->pk3f), dimg(p->pk3b), dimg(p->pk2b), dimg(p->pk1b))) {
        p->dec_fused = true;
        p->dtiles = dec_tiles(p->B, p->N, dj);
        const long long t = p->dtiles;
        p->add_buf("PDHS", t * dec_head_parts(c.s3, c.spatial_dim));
        p->add_buf("PDHN", t * dec_head_parts(c.n2, c.num_feature));
        p->add_buf("PDSSES", t, 8); p->add_buf("PDSSEN", t, 8);
        p->add_buf("PDC2S", t * 3 * c.s2); p->add_buf("PDC1", t * 3 * w1);
      }
    }
  }
  // ---- bf16 fast encoder, graph latent: GCN layers + BN backward on the fast engine;
  // the heads stream flat(G) in bf16 (snd_tref.hip)
  if (p->fast && tref && !(debug_flags() & 512)) {
    auto img1 = [&](int kin, int nout) { return Img{1, kp_of(kin), (int)round_up(nout, 16), 0}; };
    Img ims[3] = {img1(h0 + f, h1), img1(h1, h0), img1(W, W)};
    bool ok = h0 % 8 == 0 && h1 % 8 == 0 && h1 <= 128 && f <= 4 && W <= 128 && h0 + f <= 128;
    for (auto& m : ims)
      ok = ok && m.kp > 0 && m.np <= 128 && rc_lds_bytes(m.T, m.kp, m.np) <= kRcLdsLimit;
    if (ok) {
      p->fast_enc = true;
      p->kw1 = h0 + f; p->kwh = W; p->nms = 2 * L;
      p->ldh1 = (int)round_up(h0 + f, 8);
      p->ldg = (int)round_up(W, 8);
      const char* nm[3] = {"PW1F", "PW1B", "PIDG"};
      for (int i = 0; i < 3; ++i) {
        p->add_buf(nm[i], (long long)pack_bytes(ims[i].T, ims[i].kp, ims[i].np), 1);
        ims[i].off = p->bufs.back().off;
      }
      p->pw1f = ims[0]; p->pw1b = ims[1]; p->pidg = ims[2];
      p->add_buf("AX", R * 4);            p->add_buf("AXB", R * 8, 2);
      p->add_buf("FH1", R * p->ldh1, 2);  p->add_buf("FXW1", R * h1, 2);
      p->add_buf("FP1", R * h1);          p->add_buf("FG", R * p->ldg, 2);
      p->add_buf("FDG", R * p->ldg, 2);   p->add_buf("FDP1", R * h1, 2);
      p->add_buf("FDXW1", R * h1, 2);     p->add_buf("FDP0", R * h0, 2);
      const int rcb = rc_blocks(p->R);
      p->add_buf("PFENC1", (long long)rcb * 4 * W);
      p->add_buf("PFENC0", (long long)rcb * 2 * h0);
      p->gW1 = wgrad_geom(p->R, 1, h0 + f, h1, wgc_of(1, h0 + f, h1));
      p->gW0 = wgrad_geom(p->R, 1, f, h0, wgc_of(1, f, h0));
      p->add_buf("FSW1", (long long)p->gW1.gx * (h0 + f) * wgrad_n4(h1));
      p->add_buf("FSW0", (long long)p->gW0.gx * f * wgrad_n4(h0));
    }
  }
  // ---- bf16 fast encoder: GraphConvolution 0 as (A X) W0, bf16 operands throughout
  if (p->fast && !tref && !(debug_flags() & 512)) {
    auto img1 = [&](int kin, int nout) { return Img{1, kin <= 128 ? kp_of(kin) : (kin <= 256 ? 256 : -1),
                                                    (int)round_up(nout, 16), 0}; };
    const int kw1 = h0 + f <= 128 ? h0 + f : h0, kwh = W <= 128 ? W : h1;   // the rest: K tails
    Img ims[6] = {img1(kw1, h1), img1(kwh, gh), img1(gh, 2 * L), img1(2 * L, gh), img1(gh, W), img1(h1, h0)};
    bool ok = h0 % 8 == 0 && h1 % 8 == 0 && h1 <= 128 && f <= 4 && W == h1 + f && h0 <= 128 &&
              gh <= 128 && 2 * L <= 256 && (2 * L <= 128 || L % 8 == 0) && ims[0].kp <= 128 && ims[1].kp <= 128;
    for (auto& m : ims)   // images over the LDS budget run in column windows
      ok = ok && m.kp > 0 && m.np <= 256 && rc_cols_per_block(m.T, m.kp, m.np) > 0;
    if (ok) {
      p->kw1 = kw1; p->kwh = kwh; p->nms = 2 * L <= 128 ? 2 * L : L;
      p->fast_enc = true;
      p->ldh1 = (int)round_up(h0 + f, 8);
      p->ldg = (int)round_up(W, 8);
      const char* nm[6] = {"PW1F", "PWHF", "PWMSF", "PWMSB", "PWHB", "PW1B"};
      for (int i = 0; i < 6; ++i) {
        p->add_buf(nm[i], (long long)pack_bytes(ims[i].T, ims[i].kp, ims[i].np), 1);
        ims[i].off = p->bufs.back().off;
      }
      p->pw1f = ims[0]; p->pwhf = ims[1]; p->pwmsf = ims[2];
      p->pwmsb = ims[3]; p->pwhb = ims[4]; p->pw1b = ims[5];
      p->add_buf("AX", R * 4);            p->add_buf("AXB", R * 8, 2);
      p->add_buf("FH1", R * p->ldh1, 2);  p->add_buf("FXW1", R * h1, 2);
      p->add_buf("FP1", R * h1);          p->add_buf("FG", R * p->ldg, 2);
      p->add_buf("FHH", R * gh, 2);       p->add_buf("FDMS", R * 2 * L, 2);
      p->add_buf("FDH", R * gh, 2);       p->add_buf("FDP1", R * h1, 2);
      p->add_buf("FDXW1", R * h1, 2);     p->add_buf("FDP0", R * h0, 2);
      // column partials: the row engine's 128-row blocks, or the backward head's tiles
      const int rcb = std::max(rc_blocks(p->R), head_tiles(p->R));
      p->add_buf("PFBMS", (long long)std::max(reparam_bwd_fast_blocks(p->R, L), edge_reparam_blocks(p->R)) * 2 * L);
      p->add_buf("PFBH", (long long)rcb * gh);
      p->add_buf("PFENC1", (long long)rcb * 4 * W);
      p->add_buf("PFENC0", (long long)rcb * 2 * h0);
      const int nms = p->nms;
      p->gWms = wgrad_geom(p->R, 1, gh, nms, wgc_of(1, gh, nms));
      p->gWh = wgrad_geom(p->R, 1, kwh, gh, wgc_of(1, kwh, gh));
      p->gW1 = wgrad_geom(p->R, 1, kw1, h1, wgc_of(1, kw1, h1));
      p->gW0 = wgrad_geom(p->R, 1, f, h0, wgc_of(1, f, h0));
      p->add_buf("FSWMS", (long long)p->gWms.gx * gh * wgrad_n4(nms) * (2 * L / nms));
      p->add_buf("FSWH", (long long)p->gWh.gx * kwh * wgrad_n4(gh));
      p->add_buf("FSW1", (long long)p->gW1.gx * kw1 * wgrad_n4(h1));
      p->add_buf("FSW0", (long long)p->gW0.gx * f * wgrad_n4(h0));
      if (kwh < W) {
        p->gWht = wgrad_geom(p->R, 1, W - kwh, gh, wgc_of(1, W - kwh, gh));
        p->add_buf("FSWHT", (long long)p->gWht.gx * (W - kwh) * wgrad_n4(gh));
      }
      if (kw1 < h0 + f) {
        p->gW1t = wgrad_geom(p->R, 1, h0 + f - kw1, h1, wgc_of(1, h0 + f - kw1, h1));
        p->add_buf("FSW1T", (long long)p->gW1t.gx * (h0 + f - kw1) * wgrad_n4(h1));
      }
      // GraphConvolution 1 -> heads -> reparameterisation + zz^T staging in one launch
      // (debug bit 65536: the four-launch chain)
      p->head_fused = !(dbg & 65536) && zzt_dp(L) == L &&
                      head_fwd_supported(h1, f, gh, L, p->pwhf.kp, p->pwhf.np, p->pwmsf.kp, p->pwmsf.np);
      // per-edge CE terms -> reparameterisation backward -> dh -> dG -> dP1 in one launch
      // (debug bit 262144: edge_bf16 + reparam_bwd_fast + two row-engine launches)
      p->head_bwd = !(dbg & 262144) &&
                    head_bwd_supported(L, gh, W, h1, p->pwmsb.kp, p->pwmsb.np, p->pwhb.kp, p->pwhb.np);
      if (p->head_bwd) p->add_buf("PHBMS", (long long)head_tiles(p->R) * 2 * L);
      // no fused backward head (L = 128, C5): the per-edge terms ride in the reparameterisation
      // backward's launch (debug bit 1 << 27: edge_bf16 before zz^T + reparam_bwd_fast)
      p->edge_reparam = !p->head_bwd && !tref && !(dbg & (1 << 27));
    }
  }
  // GraphConvolution 0, XW1 and the packed weight images in one launch (debug bit 1048576:
  // pack + gcn0 + a row-engine launch)
  p->front_fused = p->fast_enc && !(dbg & 1048576) && front_supported(c.f_in, c.h0, c.h1, p->pw1f.kp, p->pw1f.np);
  p->pack_in_gcn0 = p->fast && p->fast_enc && !p->front_fused && !p->sg && !(dbg & (1 << 28));
  // the GCN1 backward SpMM A @ dP1 inside the RC_ENC0 launch that consumes it (round 5;
  // debug bit 128: the separate SpMM launch)
  p->enc0_gather = p->fast_enc && !(dbg & 128) && c.h1 == 64 && p->pw1b.kp == 64 && c.f_in <= 4;
  set_zzt_splits(*p);
  *out = p;
  return 0;
}

extern "C" void snd_plan_destroy(snd_plan_t* p) { delete p; }
extern "C" long long snd_plan_param_count(const snd_plan_t* p) { return p ? p->pcount : -1; }
extern "C" int snd_plan_num_blocks(const snd_plan_t* p) { return p ? (int)p->blocks.size() : -1; }
extern "C" int snd_plan_param_block(const snd_plan_t* p, int idx, const char** name,
                                    long long* offset, long long* numel) {
  SND_CHECK_ARG(p && idx >= 0 && idx < (int)p->blocks.size(), "snd_plan_param_block: bad index");
  if (name) *name = p->blocks[idx].name.c_str();
  if (offset) *offset = p->blocks[idx].off;
  if (numel) *numel = p->blocks[idx].numel;
  return 0;
}
extern "C" size_t snd_plan_workspace_bytes(const snd_plan_t* p) { return p ? (size_t)p->ws : 0; }

extern "C" int snd_plan_set_option(snd_plan_t* p, const char* name, int value) {
  SND_CHECK_ARG(p && name, "snd_plan_set_option: bad args");
  if (!strcmp(name, "conc_decoder")) {
    p->conc_dec = value;
    set_zzt_splits(*p);
    return p->conc_dec_on() ? 1 : 0;
  }
  if (!strcmp(name, "reduce_adam")) {
    // the block kinds are fixed while an update is fused: a caller that cached them
    // (OptimizerVAE._adam_ranges) would skip or double a block's update
    SND_CHECK_ARG(!p->fuse_m || (value != 0) == p->reduce_adam,
                  "snd_plan_set_option: reduce_adam cannot change while Adam is fused "
                  "(snd_plan_fuse_adam(plan, NULL, NULL, ...) first)");
    p->reduce_adam = value != 0;
    return p->reduce_adam ? 1 : 0;
  }
  set_error("snd_plan_set_option: unknown option '%s'", name);
  return SND_ERR_ARG;
}

void reduce_adam_cover(snd_plan& p);

extern "C" int snd_plan_fuse_adam(snd_plan_t* p, float* m, float* v, float lr, float beta1,
                                  float beta2, float eps) {
  SND_CHECK_ARG(p && ((m && v) || (!m && !v)), "snd_plan_fuse_adam: bad args");
  p->fuse_m = m; p->fuse_v = v;
  p->fuse_lr = lr; p->fuse_b1 = beta1; p->fuse_b2 = beta2; p->fuse_eps = eps;
  if (m && p->radam.empty()) reduce_adam_cover(*p);
  return 0;
}

extern "C" int snd_plan_set_rng_offset(snd_plan_t* p, long long head_row_offset) {
  SND_CHECK_ARG(p && head_row_offset >= 0, "snd_plan_set_rng_offset: bad args");
  p->rng_row0 = (unsigned long long)head_row_offset;
  return 0;
}

extern "C" int snd_plan_grad_event(snd_plan_t* p, int idx, void* event) {
  SND_CHECK_ARG(p && idx >= 0 && idx < (int)p->blocks.size(), "snd_plan_grad_event: bad index");
  const int pt = p->grad_point(p->blocks[idx].name);
  if (pt == 1) p->ev_proj = (hipEvent_t)event;
  if (pt == 2) p->ev_head = (hipEvent_t)event;
  return pt;
}
extern "C" int snd_plan_grad_event_get(const snd_plan_t* p, int idx, void** event) {
  SND_CHECK_ARG(p && event && idx >= 0 && idx < (int)p->blocks.size(), "snd_plan_grad_event_get: bad args");
  const int pt = p->grad_point(p->blocks[idx].name);
  *event = pt == 1 ? (void*)p->ev_proj : pt == 2 ? (void*)p->ev_head : nullptr;
  return pt;
}
extern "C" int snd_plan_block_fused(const snd_plan_t* p, int idx) {
  SND_CHECK_ARG(p && idx >= 0 && idx < (int)p->blocks.size(), "snd_plan_block_fused: bad index");
  return p->fused_kind((size_t)idx);
}
extern "C" int snd_plan_buffer(const snd_plan_t* p, const char* name, long long* off,
                               long long* numel) {
  SND_CHECK_ARG(p && name, "snd_plan_buffer: bad args");
  for (auto& b : p->bufs)
    if (b.name == name) {
      if (off) *off = b.off;
      if (numel) *numel = b.numel;
      return 0;
    }
  set_error("snd_plan_buffer: no buffer '%s'", name);
  return SND_ERR_ARG;
}

namespace {

struct Ctx {
  const snd_plan* p;
  char* ws;
  const float* P;
  float* Gr;
  hipStream_t s;
  hipStream_t side = nullptr;   // null: single-stream
  int* nev = nullptr;           // next free event of p->ev
  std::vector<WgArgs>* wq = nullptr;   // deferred weight gradients (one launch at the end)
  int zts = 1;                  // zz^T column splits of this step (launch, split sums, finalize)
  float* f(const char* n) const { return (float*)(ws + p->buf(n)); }
  double* d(const char* n) const { return (double*)(ws + p->buf(n)); }
  const float* w(const char* n) const { return P + p->blk(n); }
  float* g(const char* n) const { return Gr + p->blk(n); }
  int* stepn() const { return reinterpret_cast<int*>(ws + p->buf("STEPN")); }
};

// Adam state of a block updated inside the step (snd_plan_fuse_adam); params are
// written in place through the (caller-owned, writable) parameter buffer
AdamFuse fused_adam(const Ctx& x, const char* blk, const int* step) {
  const snd_plan& p = *x.p;
  const long long o = p.blk(blk);
  return AdamFuse{const_cast<float*>(x.P) + o, p.fuse_m + o, p.fuse_v + o,
                  p.fuse_lr, p.fuse_b1, p.fuse_b2, p.fuse_eps, step};
}

// fork: work launched on side() after this point starts after everything so far on main
int fork(const Ctx& x) {
  if (!x.side) return 0;
  SND_CHECK_ARG(*x.nev < snd_plan::kEvents, "train step: out of fork events");
  hipEvent_t e = x.p->ev[(*x.nev)++];
  if (hipEventRecord(e, x.s) != hipSuccess || hipStreamWaitEvent(x.side, e, 0) != hipSuccess) {
    set_error("train step: fork failed");
    return SND_ERR_HIP;
  }
  return 0;
}
// join: main waits for everything launched on side() so far
int join(const Ctx& x) {
  if (!x.side) return 0;
  SND_CHECK_ARG(*x.nev < snd_plan::kEvents, "train step: out of join events");
  hipEvent_t e = x.p->ev[(*x.nev)++];
  if (hipEventRecord(e, x.side) != hipSuccess || hipStreamWaitEvent(x.s, e, 0) != hipSuccess) {
    set_error("train step: join failed");
    return SND_ERR_HIP;
  }
  return 0;
}
hipStream_t side(const Ctx& x) { return x.side ? x.side : x.s; }
// fork_to / join_from: the same on an explicit stream (the concurrent decoder's)
int fork_to(const Ctx& x, hipStream_t o) {
  SND_CHECK_ARG(x.nev && *x.nev < snd_plan::kEvents, "train step: out of fork events");
  hipEvent_t e = x.p->ev[(*x.nev)++];
  if (hipEventRecord(e, x.s) != hipSuccess || hipStreamWaitEvent(o, e, 0) != hipSuccess) {
    set_error("train step: fork failed");
    return SND_ERR_HIP;
  }
  return 0;
}
int join_from(const Ctx& x, hipStream_t o) {
  SND_CHECK_ARG(x.nev && *x.nev < snd_plan::kEvents, "train step: out of join events");
  hipEvent_t e = x.p->ev[(*x.nev)++];
  if (hipEventRecord(e, o) != hipSuccess || hipStreamWaitEvent(x.s, e, 0) != hipSuccess) {
    set_error("train step: join failed");
    return SND_ERR_HIP;
  }
  return 0;
}
// a weight gradient: queued for the step's single multi-segment launch, or launched now
int wgrad(const Ctx& x, const WgArgs& a, hipStream_t s) {
  if (x.wq) { x.wq->push_back(a); return 0; }
  return launch_wgrad(a, s);
}
// mark: an event after the work queued on side() so far; wait_mark: main waits for it
int mark(const Ctx& x) {
  if (!x.side) return -1;
  if (*x.nev >= snd_plan::kEvents) { set_error("train step: out of events"); return -2; }
  const int i = (*x.nev)++;
  if (hipEventRecord(x.p->ev[i], x.side) != hipSuccess) { set_error("train step: mark failed"); return -2; }
  return i;
}
int wait_mark(const Ctx& x, int i) {
  if (i == -1) return 0;
  if (i < 0 || hipStreamWaitEvent(x.s, x.p->ev[i], 0) != hipSuccess) {
    set_error("train step: wait failed");
    return SND_ERR_HIP;
  }
  return 0;
}

// create the side stream once, outside any stream capture
void init_concurrency(const snd_plan& p, hipStream_t main) {
  if (p.conc != 0) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(main, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return;
  p.conc = -1;
  // (a side stream at the device's highest priority made the captured one-graph step
  // 3.5x slower, 0.118 -> 0.42 ms: round 6, profiles/r06_ab_b1_concurrency.txt)
  if (hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking) != hipSuccess) return;
  for (auto& e : p.ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return;
  p.conc = 1;
}

int gemm_fwd(const Ctx& x, int M, int N, int K, const float* A, int lda, const float* B, int ldb,
             int bmode, float* C, int ldc, const float* bias) {
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.bias = bias; g.kchunk = (int)round_up(K, kGemmBK);
  return launch_gemm(g, A_ROW, bmode, E_STORE, x.p->c.dtype, 1, x.s);
}

int gemm_wgrad(const Ctx& x, const float* A, int lda, int Mreal, bool ones, const float* D,
               int ldd, int N, float* slab, const Split& sp, int K = -1) {
  GemmArgs g{};
  g.M = Mreal + (ones ? 1 : 0); g.N = N; g.K = K < 0 ? x.p->R : K;
  g.A = A; g.lda = lda; g.a_ones_m1 = ones ? Mreal + 1 : 0;
  g.B = D; g.ldb = ldd; g.C = slab; g.kchunk = sp.kchunk;
  return launch_gemm(g, A_COL, B_ROW, E_PART, x.p->c.dtype, sp.splits, x.s);
}

int conv_fwd(const Ctx& x, const float* in, int ldi, int cin, const char* K, int cout,
             const char* b, const char* gam, const char* bet, float* ypre, float* out) {
  GemmArgs g{};
  g.M = x.p->R; g.N = cout; g.K = 5 * cin;
  g.A = in; g.lda = ldi; g.a_cin = cin; g.a_npg = x.p->N;
  g.B = x.w(K); g.ldb = cout; g.C = out; g.ldc = cout; g.bias = x.w(b);
  g.gamma = x.w(gam); g.beta = x.w(bet); g.pre = ypre; g.ldp = cout;
  g.kchunk = (int)round_up(g.K, kGemmBK);
  return launch_gemm(g, A_CONV, B_ROW, E_CONV, x.p->c.dtype, 1, x.s);
}

int conv_bwd_data(const Ctx& x, const float* dy, int cout, const char* K, int cin, float* dx,
                  int lddx) {
  GemmArgs g{};
  g.M = x.p->R; g.N = cin; g.K = 5 * cout;
  g.A = dy; g.lda = cout; g.a_cin = cout; g.a_npg = x.p->N;
  g.B = x.w(K); g.b_cout = cout; g.C = dx; g.ldc = lddx;
  g.kchunk = (int)round_up(g.K, kGemmBK);
  return launch_gemm(g, A_CONV, B_FLIP, E_STORE, x.p->c.dtype, 1, x.s);
}

int conv_wgrad(const Ctx& x, const float* in, int ldi, int cin, const float* dy, int cout,
               float* slab, const Split& sp) {
  GemmArgs g{};
  g.M = 5 * cin; g.N = cout; g.K = x.p->R;
  g.A = in; g.lda = ldi; g.a_cin = cin; g.a_npg = x.p->N;
  g.B = dy; g.ldb = cout; g.C = slab; g.kchunk = sp.kchunk;
  return launch_gemm(g, A_CONVT, B_ROW, E_PART, x.p->c.dtype, sp.splits, x.s);
}


// generic-engine encoder forward (model.py:104-115): H_{i+1} = [BN(lrelu(A (H_i W_i))) || X],
// G = BN_enc(H2), heads h and [mu || s] into MS (fp32 buffers, any plan)
int encoder_generic_fwd(const Ctx& x, const snd_batch_t* batch) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, N = p.N, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, L = c.latent;
  const int W = p.W, RH = p.RH;
  const long long KH = (long long)N * W;
  const int* rp = batch->rowptr;
  const int* ci = batch->colidx;
  const float* X = batch->features;
  // encoder, model.py:104-112: H_{i+1} = [BN(lrelu(A (H_i W_i))) || X]
  SND_TRY(gemm_fwd(x, R, h0, f, X, f, x.w("enc.W0"), h0, B_ROW, x.f("XW0"), h0, nullptr));
  {
    SpmmArgs a{rp, ci, R, x.f("XW0"), h0, h0, x.f("H1"), h0 + f, SND_SPMM_GCN,
               x.w("enc.bn0.gamma"), x.w("enc.bn0.beta"), x.f("P0"), h0, X, f, f,
               nullptr, nullptr, nullptr, 0};
    SND_TRY(launch_spmm(a, x.s));
  }
  SND_TRY(gemm_fwd(x, R, h1, h0 + f, x.f("H1"), h0 + f, x.w("enc.W1"), h1, B_ROW, x.f("XW1"), h1,
                   nullptr));
  {
    SpmmArgs a{rp, ci, R, x.f("XW1"), h1, h1, x.f("H2"), W, SND_SPMM_GCN,
               x.w("enc.bn1.gamma"), x.w("enc.bn1.beta"), x.f("P1"), h1, X, f, f,
               x.w("enc.bne.gamma"), x.w("enc.bne.beta"), x.f("G"), W};
    SND_TRY(launch_spmm(a, x.s));
  }
  if (p.tref) {
    // graph heads (model.py:113): h = flat(G) Wh + bh, split-K over the N*W rows of Wh
    TrefHeadFwdArgs a{x.f("G"), KH, p.B, x.w("enc.Wh"), gh, x.w("enc.bh"), x.f("PHF")};
    SND_TRY(launch_tref_head_fwd(a, x.s));
    const ReduceDesc rd{x.f("PHF"), x.f("Hh"), tref_head_fwd_blocks(KH, gh), RH * gh,
                        (long long)RH * gh, 1.f, 0, 0, 0, 0};
    SND_TRY(launch_reduce(&rd, 1, x.s));
  } else {
    // node-wise heads (model.py:113-115): h = G Wh + bh
    SND_TRY(gemm_fwd(x, R, gh, W, x.f("G"), W, x.w("enc.Wh"), gh, B_ROW, x.f("Hh"), gh,
                     x.w("enc.bh")));
  }
  // [mu || s] = h Wms + bms (model.py:114-115; small_head: with the reparameterisation)
  if (!p.small_head)
    SND_TRY(gemm_fwd(x, RH, 2 * L, gh, x.f("Hh"), gh, x.w("enc.Wms"), 2 * L, B_ROW, x.f("MS"), 2 * L,
                     x.w("enc.bms")));
  return 0;
}

// SND_SGJOINT encoder (model_joint.py:72-85 / model.py:134-151): the batch's
// spanning-tree copies through two SpatialGraphConvolution layers (lrelu(BN(.))),
// then per copy h = flat(s_g) Wh + bh and [mu || s] = h Wms + bms (rows RH = B*S).
snd_sg_graph_t sg_graph(const Ctx& x, const snd_batch_t* batch) {
  const snd_plan& p = *x.p;
  return snd_sg_graph_t{batch->tree_rowptr, batch->tree_colidx, (int)p.RS, p.N, x.f("SGLR"), x.f("SGQ"),
                        (int*)x.f("SGREV"), x.f("SGDEG"), x.f("SGE")};
}

int encoder_sg_fwd(const Ctx& x, const snd_batch_t* batch) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int N = p.N, gh = c.g_hidden, L = c.latent, W = p.W, RH = p.RH;
  const int* h = c.sg_h;
  SND_CHECK_ARG(batch->tree_rowptr && batch->tree_colidx && batch->rel,
                "snd_train_step: SND_SGJOINT needs the batch's spanning trees and rel");
  const snd_sg_graph_t g = sg_graph(x, batch);
  SND_TRY(snd_sg_prep(&g, batch->rel, (int*)x.f("SGBAD"), x.s));
  SND_TRY(snd_sg_layer_fwd(&g, batch->features, p.sgf[0], p.sgf[0], h[0], h[1], h[2], x.w("enc.sg0"), 1,
                           x.f("SGY1"), x.f("SGX1"), x.f("SGWS0"), x.s));
  SND_TRY(snd_sg_layer_fwd(&g, x.f("SGX1"), h[2], h[2], h[3], h[4], h[5], x.w("enc.sg1"), 1,
                           x.f("SGY2"), x.f("SGG"), x.f("SGWS1"), x.s));
  const int KH = N * W;   // flat(s_g) per copy: the row-major [N, W] rows of one copy
  SND_TRY(gemm_fwd(x, RH, gh, KH, x.f("SGG"), KH, x.w("enc.Wh"), gh, B_ROW, x.f("Hh"), gh, x.w("enc.bh")));
  if (p.small_head) return 0;   // with the reparameterisation
  return gemm_fwd(x, RH, 2 * L, gh, x.f("Hh"), gh, x.w("enc.Wms"), 2 * L, B_ROW, x.f("MS"), 2 * L,
                  x.w("enc.bms"));
}

// backward from DH (dL/dh per copy): dWh / dbh (split-K slab), dG = DH Wh^T, then
// both SG layers (their gradients written straight into the flat gradient blocks)
int encoder_sg_bwd(const Ctx& x, const snd_batch_t* batch) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int N = p.N, gh = c.g_hidden, W = p.W, RH = p.RH;
  const int* h = c.sg_h;
  const int KH = N * W;
  SND_TRY(gemm_wgrad(x, x.f("SGG"), KH, KH, true, x.f("DH"), gh, gh, x.f("SWH"), p.sWh, RH));
  SND_TRY(gemm_fwd(x, RH, KH, gh, x.f("DH"), gh, x.w("enc.Wh"), gh, B_COL, x.f("SGDG"), KH, nullptr));
  const snd_sg_graph_t g = sg_graph(x, batch);
  SND_TRY(snd_sg_layer_bwd(&g, x.f("SGX1"), h[2], h[2], h[3], h[4], h[5], x.w("enc.sg1"), 1, x.f("SGY2"),
                           x.f("SGDG"), x.f("SGDX1"), h[2], x.g("enc.sg1"), x.f("SGWS1"), x.s));
  return snd_sg_layer_bwd(&g, batch->features, p.sgf[0], p.sgf[0], h[0], h[1], h[2], x.w("enc.sg0"), 1,
                          x.f("SGY1"), x.f("SGDX1"), nullptr, p.sgf[0], x.g("enc.sg0"), x.f("SGWS0"), x.s);
}

// ---- bf16 fast decoder ------------------------------------------------------
RcArgs rc_args(const snd_plan& p, const char* ws, const Img& im, const void* x, int ldx, int K,
               int N, ColMap cols) {
  RcArgs a{};
  a.x = x; a.ldx = ldx; a.K = K; a.x_bf16 = 1;
  a.R = p.R; a.npg = p.N; a.T = im.T;
  a.wpk = reinterpret_cast<const __bf16*>(ws + im.off); a.kp = im.kp; a.np = im.np;
  a.N = N; a.cols = cols;
  a.zero = ws + p.buf("ZERO");
  a.dbg = debug_flags();
  return a;
}

WgArgs wg_args(const snd_plan& p, const char* ws, const WgGeom& g, const void* x, int ldx, int K, const void* dy,
               int lddy, int N, float* slab, int T = 5) {
  WgArgs a{};
  a.x = x; a.ldx = ldx; a.K = K; a.x_bf16 = 1;
  a.dy = dy; a.lddy = lddy; a.N = N; a.dy_bf16 = 1;
  a.R = p.R; a.npg = p.N; a.T = T;
  a.rows_per_wg = g.rows_per_wg; a.pairs_per_wg = g.pairs_per_wg;
  a.slab = slab;
  a.zero = ws + p.buf("ZERO");
  a.dbg = debug_flags();
  return a;
}

// the step's packed bf16 weight images (decoder convs, and the encoder linears on the fast
// encoder); returns the descriptor count
int build_packs(const Ctx& x, PackDesc* e) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int L = c.latent, dj = p.dj, s1 = c.s1, n1 = c.n1, s2 = c.s2, n2 = c.n2, s3 = c.s3;
  const int C1 = p.C1;
  auto dst = [&](const Img& im) { return reinterpret_cast<__bf16*>(x.ws + im.off); };
  auto src = [](const float* w, int A, int B, int a0, int a1, int b0, int b1, int noff, int koff,
                int mode) { return PackSrc{w, A, B, a0, a1, b0, b1, noff, koff, mode}; };
  const float *K1 = x.w("dec.K1"), *K2s = x.w("dec.K2s"), *K2n = x.w("dec.K2n"), *K3s = x.w("dec.K3s");
  const int o1 = p.m1.offb, o2 = p.m2.offb;
  PackDesc d[6]{};
  // conv forward images: n = output channel (split layouts), k = input channel
  d[0] = {dst(p.pk1f), 5, p.pk1f.kp, p.pk1f.np, 2,
          {src(K1, dj, C1, 0, dj, 0, s1, 0, 0, 0), src(K1, dj, C1, 0, dj, s1, C1, o1, 0, 0)}};
  d[1] = {dst(p.pk2f), 5, p.pk2f.kp, p.pk2f.np, 2,
          {src(K2s, s1, s2, 0, s1, 0, s2, 0, 0, 0), src(K2n, n1, n2, 0, n1, 0, n2, o2, o1, 0)}};
  d[2] = {dst(p.pk3f), 5, p.pk3f.kp, p.pk3f.np, 1, {src(K3s, s2, s3, 0, s2, 0, s3, 0, 0, 0), {}}};
  // data-gradient images: n = input channel of the forward conv, k = its output channel
  d[3] = {dst(p.pk3b), 5, p.pk3b.kp, p.pk3b.np, 1, {src(K3s, s2, s3, 0, s2, 0, s3, 0, 0, 1), {}}};
  d[4] = {dst(p.pk2b), 5, p.pk2b.kp, p.pk2b.np, 2,
          {src(K2s, s1, s2, 0, s1, 0, s2, 0, 0, 1), src(K2n, n1, n2, 0, n1, 0, n2, o1, o2, 1)}};
  d[5] = {dst(p.pk1b), 5, p.pk1b.kp, p.pk1b.np, 2,
          {src(K1, dj, C1, 0, dj, 0, s1, 0, 0, 1), src(K1, dj, C1, 0, dj, s1, C1, 0, o1, 1)}};
  for (int i = 0; i < 6; ++i) e[i] = d[i];
  if (!p.fast_enc) return 6;
  const int f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, W = p.W;
  auto one = [&](const Img& im, PackSrc ps) { return PackDesc{dst(im), 1, im.kp, im.np, 1, {ps, {}}}; };
  if (p.tref) {
    const float* W1 = x.w("enc.W1");
    e[6] = one(p.pw1f, src(W1, h0 + f, h1, 0, h0 + f, 0, h1, 0, 0, 0));
    e[7] = one(p.pw1b, src(W1, h0 + f, h1, 0, h0, 0, h1, 0, 0, 1));
    e[8] = one(p.pidg, src(nullptr, W, W, 0, W, 0, W, 0, 0, 2));
    return 9;
  }
  const float *W1 = x.w("enc.W1"), *Wh = x.w("enc.Wh"), *Wms = x.w("enc.Wms");
  e[6] = one(p.pw1f, src(W1, h0 + f, h1, 0, h0 + f, 0, h1, 0, 0, 0));
  e[7] = one(p.pwhf, src(Wh, W, gh, 0, W, 0, gh, 0, 0, 0));
  e[8] = one(p.pwmsf, src(Wms, gh, 2 * L, 0, gh, 0, 2 * L, 0, 0, 0));
  e[9] = one(p.pwmsb, src(Wms, gh, 2 * L, 0, gh, 0, 2 * L, 0, 0, 1));
  e[10] = one(p.pwhb, src(Wh, W, gh, 0, W, 0, gh, 0, 0, 1));
  e[11] = one(p.pw1b, src(W1, h0 + f, h1, 0, h0, 0, h1, 0, 0, 1));
  return 12;
}

int pack_decoder(const Ctx& x) {
  PackDesc e[kMaxPack]{};
  return launch_pack(e, build_packs(x, e), x.s);
}

// The plain bf16 SpMM A @ h (width 64) of the batch: the window kernel when the batch
// carries a window plan that fits the ring, else the row tiles / register gathers.
static int spmm_bf16_plain(const snd_batch_t* batch, int R, int npg, int ngraphs, const __bf16* h,
                           int ldh, int width, __bf16* out, int ldo, hipStream_t s);

// optional row tiles of the batch (snd_row_tiles_t): the SpMM stages neighbour rows in LDS
static void use_tiles(SpmmBfArgs& a, const snd_batch_t* batch, int npg, int ngraphs) {
  a.row_order = batch->row_order;
  if (batch->tiles.tile_rows <= 0) return;
  a.t_rowid = batch->tiles.rows; a.t_trp = batch->tiles.trp; a.t_lcol = batch->tiles.lcol;
  a.t_ucol = batch->tiles.ucol; a.t_rows = batch->tiles.tile_rows; a.t_ustride = batch->tiles.ustride;
  a.npg = npg; a.ngraphs = ngraphs;
}

static int spmm_bf16_plain(const snd_batch_t* batch, int R, int npg, int ngraphs, const __bf16* h,
                           int ldh, int width, __bf16* out, int ldo, hipStream_t s) {
  const snd_window_plan_t& w = batch->window;
  if (w.meta && width == 64 && w.beta >= 0 && ((w.beta + 7) & ~7) <= spmm_win_max_beta() &&
      !(debug_flags() & (1 << 22))) {   // debug bit 1 << 22: the row tiles (A/B)
    SpmmWinArgs a{w.meta, w.slots, w.rows, w.order, w.beta, R, npg, ngraphs, h, ldh, width, out, ldo};
    return launch_spmm_window(a, s);
  }
  SpmmBfArgs a{batch->rowptr, batch->colidx, R, h, ldh, width, SND_SPMM_PLAIN, out, ldo};
  a.xcd_nbg = xcd_nbg(npg, ngraphs);
  use_tiles(a, batch, npg, ngraphs);
  return launch_spmm_bf16(a, s);
}

// encoder forward (model.py:104-115): H1 -> XW1 -> GCN1 -> heads h, [mu | logstd]
int encoder_fast_fwd(const Ctx& x, const snd_batch_t* batch) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, L = c.latent, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, W = p.W;
  auto bf = [&](const char* n) { return reinterpret_cast<__bf16*>(x.f(n)); };
  if (p.front_fused) {   // gcn0 + XW1 + the packed weight images: one launch
    FrontArgs a{};
    a.rowptr = batch->rowptr; a.colidx = batch->colidx; a.R = R;
    a.x = batch->features; a.ldx = f; a.f = f;
    a.w0 = x.w("enc.W0"); a.g0 = x.w("enc.bn0.gamma"); a.b0 = x.w("enc.bn0.beta"); a.h0 = h0;
    a.h1 = bf("FH1"); a.ldh1 = p.ldh1; a.ax = x.f("AX"); a.axb = bf("AXB");
    a.w1 = x.w("enc.W1"); a.n1 = h1; a.kp1 = p.pw1f.kp; a.np1 = p.pw1f.np;
    a.xw1 = bf("FXW1"); a.dbg = debug_flags();
    PackDesc e[kMaxPack]{};
    const int ne = build_packs(x, e);
    SND_TRY(launch_front(a, e, ne, x.s));
  }
  if (!p.front_fused) {
    Gcn0Args a{batch->rowptr, batch->colidx, R, batch->features, f, f, x.w("enc.W0"),
               x.w("enc.bn0.gamma"), x.w("enc.bn0.beta"), h0, bf("FH1"), p.ldh1, x.f("AX"), bf("AXB"),
               xcd_nbg(p.N, p.B)};
    a.row_order = batch->row_order;
    if (p.pack_in_gcn0) a.npack = build_packs(x, a.pack);
    SND_TRY(launch_gcn0(a, x.s));
  }
  if (!p.front_fused) {   // p.kw1 < h0 + f: the X columns as the K tail
    RcArgs a = rc_args(p, x.ws, p.pw1f, bf("FH1"), p.ldh1, p.kw1, h1, colmap_plain(h1));
    a.ktail = h0 + f - p.kw1; a.wtail = x.w("enc.W1") + (long long)p.kw1 * h1; a.ldwt = h1;
    a.out = bf("FXW1"); a.ldo = h1; a.out_bf16 = 1;
    SND_TRY(launch_rowconv(a, RC_LIN, x.s));
  }
  if (p.head_fused) return 0;   // the rest runs in head_fwd_fused (after the eps inputs are known)
  {
    SpmmBfArgs a{batch->rowptr, batch->colidx, R, bf("FXW1"), h1, h1, SND_SPMM_GCN, nullptr, 0,
                 x.f("FP1"), h1, x.w("enc.bn1.gamma"), x.w("enc.bn1.beta"), batch->features, f, f,
                 x.w("enc.bne.gamma"), x.w("enc.bne.beta"), bf("FG"), p.ldg, xcd_nbg(p.N, p.B)};
    use_tiles(a, batch, p.N, p.B);
    SND_TRY(launch_spmm_bf16(a, x.s));
  }
  if (p.tref) return 0;   // graph heads: snd_tref.hip on bf16 flat(G)
  {
    RcArgs a = rc_args(p, x.ws, p.pwhf, bf("FG"), p.ldg, p.kwh, gh, colmap_plain(gh));
    a.ktail = W - p.kwh; a.wtail = x.w("enc.Wh") + (long long)p.kwh * gh; a.ldwt = gh;
    a.bias = x.w("enc.bh"); a.out = bf("FHH"); a.ldo = gh; a.out_bf16 = 1;
    SND_TRY(launch_rowconv(a, RC_LIN, x.s));
  }
  {
    RcArgs a = rc_args(p, x.ws, p.pwmsf, bf("FHH"), gh, gh, 2 * L, colmap_plain(2 * L));
    a.bias = x.w("enc.bms"); a.out = x.f("MS"); a.ldo = 2 * L; a.out_bf16 = 0;
    SND_TRY(launch_rowconv(a, RC_LIN, x.s));
  }
  return 0;
}

// GraphConvolution 1 + heads + reparameterisation + zz^T staging (snd_head.hip)
int head_fwd_fused(const Ctx& x, const snd_batch_t* batch, const float* eps, unsigned long long seed,
                   const int* step_counter, const ZztStage& stg) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  HeadFwdArgs a{};
  a.rowptr = batch->rowptr; a.colidx = batch->colidx;
  a.R = p.R; a.npg = p.N; a.ngraphs = p.B; a.npad = zzt_npad(p.N);
  a.xw1 = reinterpret_cast<const __bf16*>(x.f("FXW1")); a.h1 = c.h1;
  a.g1 = x.w("enc.bn1.gamma"); a.b1 = x.w("enc.bn1.beta");
  a.x = batch->features; a.ldx = c.f_in; a.f = c.f_in;
  a.ge = x.w("enc.bne.gamma"); a.be = x.w("enc.bne.beta");
  a.p1 = x.f("FP1"); a.g = reinterpret_cast<__bf16*>(x.f("FG")); a.ldg = p.ldg;
  a.wh_img = reinterpret_cast<const __bf16*>(x.ws + p.pwhf.off); a.kp1 = p.pwhf.kp; a.np1 = p.pwhf.np;
  a.gh = c.g_hidden; a.bh = x.w("enc.bh"); a.hh = reinterpret_cast<__bf16*>(x.f("FHH"));
  a.wms_img = reinterpret_cast<const __bf16*>(x.ws + p.pwmsf.off); a.kp2 = p.pwmsf.kp; a.np2 = p.pwmsf.np;
  a.bms = x.w("enc.bms"); a.ms = x.f("MS"); a.L = c.latent;
  a.eps_in = eps; a.seed = seed; a.step = step_counter; a.eps_base = p.eps_base();
  a.z = x.f("Z"); a.eps_out = x.f("EPS"); a.zb = reinterpret_cast<__bf16*>(x.f("ZB"));
  a.jrow = reinterpret_cast<__bf16*>(stg.jrow); a.jt = reinterpret_cast<__bf16*>(stg.jt);
  a.colpart = stg.colpart; a.kl_part = x.d("PKL");
  a.stepn = x.stepn();
  a.dbg = debug_flags();
  return launch_head_fwd(a, x.s);
}

int encoder_fast_bwd_tail(const Ctx& x, const snd_batch_t* batch, bool enc1_done = false);

// the fused backward head alone (encoder_fast_bwd; snd_plan_launch "head_bwd")
int head_bwd_fused(const Ctx& x, const snd_batch_t* batch, float adj_scale, float kl_scale) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, L = c.latent, f = c.f_in, h1 = c.h1, gh = c.g_hidden, W = p.W;
  auto bf = [&](const char* n) { return reinterpret_cast<__bf16*>(x.f(n)); };
  {
    HeadBwdArgs a{};
    a.rowptr = batch->rowptr; a.colidx = batch->colidx; a.R = R;
    a.zb = bf("ZB"); a.L = L; a.pos_weight = c.pos_weight; a.edge_part = x.d("PEDGE");
    a.ms = x.f("MS"); a.eps = x.f("EPS"); a.dz_dec = x.f("DZDEC"); a.dJd = x.f("DJD");
    a.dJd_extra = x.f("DJDX"); a.nextra = x.zts - 1;   // deferred split sum
    a.adj_scale = adj_scale; a.kl_scale = kl_scale;
    a.dms = bf("FDMS"); a.bms_part = x.f("PHBMS");
    a.wmsb_img = reinterpret_cast<const __bf16*>(x.ws + p.pwmsb.off); a.kp1 = p.pwmsb.kp; a.np1 = p.pwmsb.np;
    a.gh = gh; a.dh = bf("FDH"); a.bh_part = x.f("PFBH");
    a.whb_img = reinterpret_cast<const __bf16*>(x.ws + p.pwhb.off); a.kp2 = p.pwhb.kp; a.np2 = p.pwhb.np;
    a.W = W; a.h1 = h1;
    a.ge = x.w("enc.bne.gamma"); a.g1 = x.w("enc.bn1.gamma"); a.b1 = x.w("enc.bn1.beta");
    a.p1 = x.f("FP1"); a.x = batch->features; a.ldx = f;
    a.dp1 = bf("FDP1"); a.enc1_part = x.f("PFENC1");
    a.npg = p.N; a.ngraphs = p.B; a.dbg = debug_flags();
    return launch_head_bwd(a, x.s);
  }
}

// encoder backward: reparam -> heads -> GCN1 -> GCN0 (all weight gradients as slabs)
int encoder_fast_bwd(const Ctx& x, const snd_batch_t* batch, float adj_scale, float kl_scale) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, L = c.latent, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, W = p.W;
  auto bf = [&](const char* n) { return reinterpret_cast<__bf16*>(x.f(n)); };
  if (p.head_bwd) {
    SND_TRY(head_bwd_fused(x, batch, adj_scale, kl_scale));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gWms, bf("FHH"), gh, gh, bf("FDMS"), 2 * L, 2 * L, x.f("FSWMS"), 1), x.s));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gWh, bf("FG"), p.ldg, W, bf("FDH"), gh, gh, x.f("FSWH"), 1), x.s));
    return encoder_fast_bwd_tail(x, batch, true);
  }
  {
    ReparamBwdFastArgs a{x.f("MS"), 2 * L, R, L, x.f("EPS"), x.f("DZDEC"), x.f("DJD"), x.f("EJ"),
                         adj_scale, kl_scale, bf("FDMS"), 2 * L, x.f("PFBMS")};
    a.dJd_extra = x.f("DJDX"); a.nextra = x.zts - 1;   // deferred split sum
    if (p.edge_reparam) {   // the per-edge terms here, not before zz^T
      EdgeBfArgs ea{batch->rowptr, batch->colidx, R, reinterpret_cast<const __bf16*>(x.f("ZB")), L, c.pos_weight,
                    nullptr, x.d("PEDGE"), xcd_nbg(p.N, p.B)};
      ea.row_order = batch->row_order;
      SND_TRY(launch_edge_reparam_bwd(ea, a, x.s));
    } else {
      SND_TRY(launch_reparam_bwd_fast(a, x.s));
    }
  }
  SND_TRY(fork(x));
  for (int h = 0; h < 2 * L; h += p.nms)   // [mu | logstd] in nms-column halves
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gWms, bf("FHH"), gh, gh, bf("FDMS") + h, 2 * L, p.nms,
                             x.f("FSWMS") + (long long)(h / p.nms) * p.gWms.gx * gh * wgrad_n4(p.nms), 1),
                  side(x)));
  {
    RcArgs a = rc_args(p, x.ws, p.pwmsb, bf("FDMS"), 2 * L, 2 * L, gh, colmap_plain(gh));
    a.out = bf("FDH"); a.ldo = gh; a.out_bf16 = 1; a.colpart = x.f("PFBH"); a.ncp = 1;
    SND_TRY(launch_rowconv(a, RC_LIN, x.s));
  }
  SND_TRY(fork(x));
  SND_TRY(wgrad(x, wg_args(p, x.ws, p.gWh, bf("FG"), p.ldg, p.kwh, bf("FDH"), gh, gh, x.f("FSWH"), 1), side(x)));
  if (p.kwh < W)
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gWht, bf("FG") + p.kwh, p.ldg, W - p.kwh, bf("FDH"), gh, gh,
                             x.f("FSWHT"), 1), side(x)));
  return encoder_fast_bwd_tail(x, batch);
}

// encoder backward from dG: BN/lrelu backward (RC_ENC1 epilogue) -> GCN1 -> GCN0.
// Node latent: dG = dH Wh^T is the RC_ENC1 GEMM itself; graph latent: dG (bf16,
// from tref_head_bwd) passes through an identity image.
int encoder_fast_bwd_tail(const Ctx& x, const snd_batch_t* batch, bool enc1_done) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, W = p.W;
  auto bf = [&](const char* n) { return reinterpret_cast<__bf16*>(x.f(n)); };
  if (!enc1_done) {
    RcArgs a = p.tref ? rc_args(p, x.ws, p.pidg, bf("FDG"), p.ldg, W, W, colmap_plain(W))
                      : rc_args(p, x.ws, p.pwhb, bf("FDH"), gh, gh, W, colmap_plain(W));
    a.gamma = x.w("enc.bne.gamma"); a.g2 = x.w("enc.bn1.gamma"); a.b2 = x.w("enc.bn1.beta");
    a.p = x.f("FP1"); a.ldp = h1; a.xf = batch->features; a.ldxf = f; a.f = f; a.h = h1;
    a.out = bf("FDP1"); a.ldo = h1; a.out_bf16 = 1; a.colpart = x.f("PFENC1"); a.ncp = 4;
    SND_TRY(launch_rowconv(a, RC_ENC1, x.s));
  }
  auto w1grad = [&]() -> int {
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gW1, bf("FH1"), p.ldh1, p.kw1, bf("FDXW1"), h1, h1, x.f("FSW1"), 1), side(x)));
    if (p.kw1 < h0 + f)
      SND_TRY(wgrad(x, wg_args(p, x.ws, p.gW1t, bf("FH1") + p.kw1, p.ldh1, h0 + f - p.kw1, bf("FDXW1"), h1, h1,
                               x.f("FSW1T"), 1), side(x)));
    return 0;
  };
  if (!p.enc0_gather) {
    SND_TRY(spmm_bf16_plain(batch, R, p.N, p.B, bf("FDP1"), h1, h1, bf("FDXW1"), h1, x.s));
    SND_TRY(fork(x));
    SND_TRY(w1grad());
  }
  {
    RcArgs a = rc_args(p, x.ws, p.pw1b, p.enc0_gather ? (const void*)bf("FDP1") : (const void*)bf("FDXW1"), h1, h1,
                       h0, colmap_plain(h0));
    a.gamma = x.w("enc.bn0.gamma"); a.p = x.f("AX"); a.ldp = 4; a.w0 = x.w("enc.W0"); a.f = f;
    a.out = bf("FDP0"); a.ldo = h0; a.out_bf16 = 1; a.colpart = x.f("PFENC0"); a.ncp = 2;
    if (p.enc0_gather) {   // dXW1 = A @ dP1 gathered by the launch (and stored for dW1)
      a.g_rowptr = batch->rowptr; a.g_colidx = batch->colidx; a.gout = bf("FDXW1"); a.ldgo = h1;
    }
    SND_TRY(launch_rowconv(a, RC_ENC0, x.s));
  }
  if (p.enc0_gather) {
    SND_TRY(fork(x));
    SND_TRY(w1grad());
  }
  SND_TRY(fork(x));
  return wgrad(x, wg_args(p, x.ws, p.gW0, bf("AXB"), 8, f, bf("FDP0"), h0, h0, x.f("FSW0"), 1), side(x));
}

void encoder_fast_reduce(const Ctx& x, std::vector<ReduceDesc>& rd) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int L = c.latent, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, W = p.W;
  const int rcb = rc_blocks(p.R);
  // PFBH / PFENC1 come from the fused backward head (its tiles) or the row engine (rcb)
  const int hcb = p.head_bwd ? head_tiles(p.R) : rcb;
  auto flat = [&](const char* buf, int parts, long long len, long long stride, const char* dst, float sc) {
    rd.push_back({x.f(buf), x.g(dst), parts, (int)len, stride, sc, 0, 0, 0, 0});
  };
  auto slab2d = [&](const char* buf, int parts, int rows, int N, const char* dst) {
    const int n4 = wgrad_n4(N);
    rd.push_back({x.f(buf), x.g(dst), parts, N, (long long)rows * n4, 1.f, 0, rows, n4, N});
  };
  // slab [parts][rows][n4] -> rows [rows][N] of a weight with row stride dst_rs, at dst
  auto slab_at = [&](const float* src, int parts, int rows, int N, float* dst, long long dst_rs) {
    const int n4 = wgrad_n4(N);
    rd.push_back({src, dst, parts, N, (long long)rows * n4, 1.f, 0, rows, n4, dst_rs});
  };
  if (!p.tref) {   // graph-latent heads are reduced by the generic path / written directly
    for (int h = 0; h < 2 * L; h += p.nms)
      slab_at(x.f("FSWMS") + (long long)(h / p.nms) * p.gWms.gx * gh * wgrad_n4(p.nms), p.gWms.gx, gh, p.nms,
              x.g("enc.Wms") + h, 2 * L);
    if (p.head_bwd) flat("PHBMS", head_tiles(p.R), 2 * L, 2 * L, "enc.bms", 1.f);
    else flat("PFBMS", p.edge_reparam ? edge_reparam_blocks(p.R) : reparam_bwd_fast_blocks(p.R, L), 2 * L, 2 * L,
              "enc.bms", 1.f);
    slab2d("FSWH", p.gWh.gx, p.kwh, gh, "enc.Wh");
    if (p.kwh < W) slab_at(x.f("FSWHT"), p.gWht.gx, W - p.kwh, gh, x.g("enc.Wh") + (long long)p.kwh * gh, gh);
    flat("PFBH", hcb, gh, gh, "enc.bh", 1.f);
  }
  slab2d("FSW1", p.gW1.gx, p.kw1, h1, "enc.W1");
  if (p.kw1 < h0 + f) slab_at(x.f("FSW1T"), p.gW1t.gx, h0 + f - p.kw1, h1, x.g("enc.W1") + (long long)p.kw1 * h1, h1);
  slab2d("FSW0", p.gW0.gx, f, h0, "enc.W0");
  const float* e1 = x.f("PFENC1");
  rd.push_back({e1, x.g("enc.bne.gamma"), hcb, W, 4LL * W, kBnC, 0, 0, 0, 0});
  rd.push_back({e1 + W, x.g("enc.bne.beta"), hcb, W, 4LL * W, 1.f, 0, 0, 0, 0});
  rd.push_back({e1 + 2 * W, x.g("enc.bn1.gamma"), hcb, h1, 4LL * W, kBnC, 0, 0, 0, 0});
  rd.push_back({e1 + 3 * W, x.g("enc.bn1.beta"), hcb, h1, 4LL * W, 1.f, 0, 0, 0, 0});
  const float* e0 = x.f("PFENC0");
  rd.push_back({e0, x.g("enc.bn0.gamma"), rcb, h0, 2LL * h0, kBnC, 0, 0, 0, 0});
  rd.push_back({e0 + h0, x.g("enc.bn0.beta"), rcb, h0, 2LL * h0, 1.f, 0, 0, 0, 0});
}

// decoder forward + heads + backward (model_joint.py:112-145, optimizer.py:149,153)
int decoder_fast(const Ctx& x, const snd_batch_t* batch, int only = -1) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, L = p.dj, s2 = c.s2, s3 = c.s3, n2 = c.n2;   // L: width of J here
  const int sd = c.spatial_dim, nf = c.num_feature;
  const int w1 = p.m1.phys(), w2 = p.m2.phys(), o1 = p.m1.offb, o2 = p.m2.offb;
  auto bf = [&](const char* n) { return reinterpret_cast<__bf16*>(x.f(n)); };
  if (p.dec_fused && (only < 0 || only >= 100)) {   // 100: forward kernel only, 101: backward only
    auto img = [&](const Img& im) {
      return DecImg{reinterpret_cast<const __bf16*>(x.ws + im.off), im.kp, im.np};
    };
    DecChainFwdArgs f{};
    f.zb = bf("ZB"); f.ldz = L; f.dj = L;
    f.R = R; f.npg = p.N; f.ngraphs = p.B;
    f.k1 = img(p.pk1f); f.k2 = img(p.pk2f); f.k3 = img(p.pk3f);
    f.m1 = p.m1; f.m2 = p.m2; f.s3 = s3;
    f.b1 = x.w("dec.b1"); f.g1 = x.w("dec.bn1.gamma"); f.be1 = x.w("dec.bn1.beta");
    f.b2s = x.w("dec.b2s"); f.g2s = x.w("dec.bn2s.gamma"); f.be2s = x.w("dec.bn2s.beta");
    f.b2n = x.w("dec.b2n"); f.g2n = x.w("dec.bn2n.gamma"); f.be2n = x.w("dec.bn2n.beta");
    f.b3 = x.w("dec.b3s"); f.g3 = x.w("dec.bn3s.gamma"); f.be3 = x.w("dec.bn3s.beta");
    f.y1 = x.f("FY1"); f.ldy1 = p.ld1; f.u1 = bf("FU1");
    f.y2 = x.f("FY2"); f.ldy2 = p.ld2; f.u2 = bf("FU2");
    f.ws = x.w("dec.Ws"); f.bs = x.w("dec.bs"); f.sd = sd; f.s_truth = batch->spatial_truth;
    f.cnt_s = (float)R * sd; f.shat = x.f("SHAT");
    f.wn = x.w("dec.Wn"); f.bn = x.w("dec.bn"); f.nf = nf; f.x_truth = batch->feature_truth;
    f.cnt_n = (float)R * nf; f.xhat = x.f("XHAT");
    f.dy3 = bf("FDY3"); f.lddy3 = p.ld3; f.dy2 = bf("FDY2"); f.lddy2 = p.ld2;
    f.phs = x.f("PDHS"); f.phn = x.f("PDHN"); f.sse_s = x.d("PDSSES"); f.sse_n = x.d("PDSSEN");
    f.zero = x.ws + p.buf("ZERO");
    f.dbg = debug_flags();
    if (only != 101) SND_TRY(launch_dec_chain_fwd(f, x.s));
    if (only == 100) return 0;
    DecChainBwdArgs b{};
    b.R = R; b.npg = p.N; b.ngraphs = p.B; b.dj = L;
    b.k3t = img(p.pk3b); b.k2t = img(p.pk2b); b.k1t = img(p.pk1b);
    b.m1 = p.m1; b.m2 = p.m2; b.s3 = s3;
    b.g1 = x.w("dec.bn1.gamma"); b.be1 = x.w("dec.bn1.beta");
    b.g2s = x.w("dec.bn2s.gamma"); b.be2s = x.w("dec.bn2s.beta");
    b.y1 = x.f("FY1"); b.ldy1 = p.ld1; b.y2 = x.f("FY2"); b.ldy2 = p.ld2;
    b.dy3 = bf("FDY3"); b.lddy3 = p.ld3; b.dy2 = bf("FDY2"); b.lddy2 = p.ld2;
    b.dy1 = bf("FDY1"); b.lddy1 = p.ld1; b.dz = x.f("DZDEC"); b.lddz = L;
    b.pc2s = x.f("PDC2S"); b.pc1 = x.f("PDC1");
    b.zero = x.ws + p.buf("ZERO");
    b.dbg = debug_flags();
    SND_TRY(launch_dec_chain_bwd(b, x.s));
    if (only == 101) return 0;
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK3s, bf("FU2"), p.ld2, s2, bf("FDY3"), p.ld3, s3, x.f("FSK3S")), x.s));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK2s, bf("FU1"), p.ld1, c.s1, bf("FDY2"), p.ld2, s2, x.f("FSK2S")), x.s));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK2n, bf("FU1") + o1, p.ld1, c.n1, bf("FDY2") + o2, p.ld2, n2,
                             x.f("FSK2N")), x.s));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK1, bf("ZB"), L, L, bf("FDY1"), p.ld1, w1, x.f("FSK1")), x.s));
    return 0;
  }
  // conv1 (fused [s1 | n0] branches): z -> Y1, U1
  {
    RcArgs a = rc_args(p, x.ws, p.pk1f, bf("ZB"), L, L, w1, p.m1);
    a.bias = x.w("dec.b1"); a.gamma = x.w("dec.bn1.gamma"); a.beta = x.w("dec.bn1.beta");
    a.y = x.f("FY1"); a.ldy = p.ld1; a.out = bf("FU1"); a.ldo = p.ld1; a.out_bf16 = 1;
    if (only < 0 || only == 0) SND_TRY(launch_rowconv(a, RC_FWD, x.s));
  }
  // conv2 (block-diagonal s2 | n1): U1 -> Y2, U2
  {
    RcArgs a = rc_args(p, x.ws, p.pk2f, bf("FU1"), p.ld1, w1, w2, p.m2);
    a.bias = x.w("dec.b2s"); a.gamma = x.w("dec.bn2s.gamma"); a.beta = x.w("dec.bn2s.beta");
    a.bias_b = x.w("dec.b2n"); a.gamma_b = x.w("dec.bn2n.gamma"); a.beta_b = x.w("dec.bn2n.beta");
    a.y = x.f("FY2"); a.ldy = p.ld2; a.out = bf("FU2"); a.ldo = p.ld2; a.out_bf16 = 1;
    if (only < 0 || only == 1) SND_TRY(launch_rowconv(a, RC_FWD, x.s));
  }
  // conv3 (s3): U2s -> Y3, U3 (fp32: head input)
  {
    RcArgs a = rc_args(p, x.ws, p.pk3f, bf("FU2"), p.ld2, s2, s3, colmap_plain(s3));
    a.bias = x.w("dec.b3s"); a.gamma = x.w("dec.bn3s.gamma"); a.beta = x.w("dec.bn3s.beta");
    a.y = x.f("FY3"); a.ldy = p.ld3; a.out = x.f("FU3"); a.ldo = p.ld3; a.out_bf16 = 0;
    if (only < 0 || only == 2) SND_TRY(launch_rowconv(a, RC_FWD, x.s));
  }
  // heads + MSE + backward, fused with the BN/lrelu backward of conv3 / conv2n
  {
    HeadFastArgs h[2]{};
    h[0] = {x.f("FU3"), p.ld3, 0, x.f("FY3"), p.ld3, x.w("dec.bn3s.gamma"), x.w("dec.bn3s.beta"), s3,
            x.w("dec.Ws"), x.w("dec.bs"), sd, batch->spatial_truth, sd, (float)R * sd, x.f("SHAT"),
            bf("FDY3"), p.ld3, x.f("PFHS"), x.d("PSSES")};
    h[1] = {bf("FU2") + o2, p.ld2, 1, x.f("FY2") + o2, p.ld2, x.w("dec.bn2n.gamma"),
            x.w("dec.bn2n.beta"), n2, x.w("dec.Wn"), x.w("dec.bn"), nf, batch->feature_truth, nf,
            (float)R * nf, x.f("XHAT"), bf("FDY2") + o2, p.ld2, x.f("PFHN"), x.d("PSSEN")};
    if (only < 0 || only == 3) SND_TRY(launch_heads_fast(h, 2, R, x.s));
  }
  // conv3 data gradient -> dU2s, fused BN/lrelu backward of conv2s -> dY2[:, :s2]
  {
    RcArgs a = rc_args(p, x.ws, p.pk3b, bf("FDY3"), p.ld3, s3, s2, colmap_plain(s2));
    a.gamma = x.w("dec.bn2s.gamma"); a.beta = x.w("dec.bn2s.beta");
    a.y = x.f("FY2"); a.ldy = p.ld2; a.out = bf("FDY2"); a.ldo = p.ld2; a.out_bf16 = 1;
    a.colpart = x.f("PFDEC2S"); a.ncp = 3;
    if (only < 0 || only == 4) SND_TRY(launch_rowconv(a, RC_DECBWD, x.s));
  }
  if (only < 0 || only == 5) {
    SND_TRY(fork(x));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK3s, bf("FU2"), p.ld2, s2, bf("FDY3"), p.ld3, s3, x.f("FSK3S")), side(x)));
  }
  // conv2 data gradient -> dU1, fused BN/lrelu backward of conv1 -> dY1
  {
    RcArgs a = rc_args(p, x.ws, p.pk2b, bf("FDY2"), p.ld2, w2, w1, p.m1);
    a.gamma = x.w("dec.bn1.gamma"); a.beta = x.w("dec.bn1.beta");
    a.y = x.f("FY1"); a.ldy = p.ld1; a.out = bf("FDY1"); a.ldo = p.ld1; a.out_bf16 = 1;
    a.colpart = x.f("PFDEC1"); a.ncp = 3;
    if (only < 0 || only == 6) SND_TRY(launch_rowconv(a, RC_DECBWD, x.s));
  }
  if (only < 0 || only == 7) {
    SND_TRY(fork(x));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK2s, bf("FU1"), p.ld1, c.s1, bf("FDY2"), p.ld2, s2, x.f("FSK2S")), side(x)));
  }
  if (only < 0 || only == 8) {
    SND_TRY(fork(x));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK2n, bf("FU1") + o1, p.ld1, c.n1, bf("FDY2") + o2, p.ld2, n2,
                               x.f("FSK2N")), side(x)));
  }
  // conv1 data gradient -> dz (decoder part)
  {
    RcArgs a = rc_args(p, x.ws, p.pk1b, bf("FDY1"), p.ld1, w1, L, colmap_plain(L));
    a.out = x.f("DZDEC"); a.ldo = L; a.out_bf16 = 0;
    if (only < 0 || only == 9) SND_TRY(launch_rowconv(a, RC_LIN, x.s));
  }
  if (only < 0 || only == 10) {
    SND_TRY(fork(x));
    SND_TRY(wgrad(x, wg_args(p, x.ws, p.gK1, bf("ZB"), L, L, bf("FDY1"), p.ld1, w1, x.f("FSK1")), side(x)));
  }
  return 0;
}

// reduce descriptors of the fast decoder's partials
void decoder_fast_reduce(const Ctx& x, std::vector<ReduceDesc>& rd) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int L = p.dj, s1 = c.s1, n1 = c.n1, s2 = c.s2, n2 = c.n2, s3 = c.s3, C1 = p.C1;
  const int sd = c.spatial_dim, nf = c.num_feature;
  const int w1 = p.m1.phys(), o1 = p.m1.offb;
  const int rcb = p.dec_fused ? p.dtiles : rc_blocks(p.R);
  const int hb = p.dec_fused ? p.dtiles : heads_fast_blocks(p.R);
  // slab [parts][rows][n4] -> weight [rows][N]
  auto slab2d = [&](const char* buf, int parts, int rows, int N, const char* dst) {
    const int n4 = wgrad_n4(N);
    rd.push_back({x.f(buf), x.g(dst), parts, N, (long long)rows * n4, 1.f, 0, rows, n4, N});
  };
  slab2d("FSK3S", p.gK3s.gx, 5 * s2, s3, "dec.K3s");
  slab2d("FSK2S", p.gK2s.gx, 5 * s1, s2, "dec.K2s");
  slab2d("FSK2N", p.gK2n.gx, 5 * n1, n2, "dec.K2n");
  {  // [5][L][w1] split columns -> dec.K1 [5][L][C1]
    const int n4 = wgrad_n4(w1);
    const long long st = 5LL * L * n4;
    rd.push_back({x.f("FSK1"), x.g("dec.K1"), p.gK1.gx, s1, st, 1.f, 0, 5 * L, n4, C1});
    rd.push_back({x.f("FSK1") + o1, x.g("dec.K1") + s1, p.gK1.gx, n1, st, 1.f, 0, 5 * L, n4, C1});
  }
  // per-column partials {sum dt*y (x c), sum dt, sum dy} -> gamma, beta, bias
  auto cols3 = [&](const char* buf, int parts, int width, int src0, int len, const char* g,
                   const char* b, const char* bias, int dst0) {
    const long long st = 3LL * width;
    const float* s0 = x.f(buf) + src0;
    rd.push_back({s0, x.g(g) + dst0, parts, len, st, kBnC, 0, 0, 0, 0});
    rd.push_back({s0 + width, x.g(b) + dst0, parts, len, st, 1.f, 0, 0, 0, 0});
    rd.push_back({s0 + 2 * width, x.g(bias) + dst0, parts, len, st, 1.f, 0, 0, 0, 0});
  };
  const char* pc2 = p.dec_fused ? "PDC2S" : "PFDEC2S";
  const char* pc1 = p.dec_fused ? "PDC1" : "PFDEC1";
  cols3(pc2, rcb, s2, 0, s2, "dec.bn2s.gamma", "dec.bn2s.beta", "dec.b2s", 0);
  cols3(pc1, rcb, w1, 0, s1, "dec.bn1.gamma", "dec.bn1.beta", "dec.b1", 0);
  cols3(pc1, rcb, w1, o1, n1, "dec.bn1.gamma", "dec.bn1.beta", "dec.b1", s1);
  // heads: {dW, db, sum dt*y, sum dt, sum dy}
  auto head = [&](const char* buf, int cin, int cout, const char* W, const char* bb, const char* g,
                  const char* be, const char* bias) {
    const long long st = heads_fast_parts(cin, cout);
    const float* s0 = x.f(buf);
    rd.push_back({s0, x.g(W), hb, cin * cout, st, 1.f, 0, 0, 0, 0});
    rd.push_back({s0 + cin * cout, x.g(bb), hb, cout, st, 1.f, 0, 0, 0, 0});
    const int q = cin * cout + cout;
    rd.push_back({s0 + q, x.g(g), hb, cin, st, kBnC, 0, 0, 0, 0});
    rd.push_back({s0 + q + cin, x.g(be), hb, cin, st, 1.f, 0, 0, 0, 0});
    rd.push_back({s0 + q + 2 * cin, x.g(bias), hb, cin, st, 1.f, 0, 0, 0, 0});
  };
  head(p.dec_fused ? "PDHS" : "PFHS", s3, sd, "dec.Ws", "dec.bs", "dec.bn3s.gamma", "dec.bn3s.beta", "dec.b3s");
  head(p.dec_fused ? "PDHN" : "PFHN", n2, nf, "dec.Wn", "dec.bn", "dec.bn2n.gamma", "dec.bn2n.beta", "dec.b2n");
}

}  // namespace

// Forward-only pass for evaluation and sampling (main.py:358-469 generate_new*,
// model.py:163-169 get_random_z) on the generic kernels of the plan's dtype:
// encoder (modes SAMPLE / MEAN) -> z -> [d_sg_lin1] -> J -> conv decoders + sigmoid
// heads (SHAT, XHAT) -> optional predicted adjacency (model.py:205-208).
extern "C" int snd_generate(const snd_plan_t* plan, const snd_batch_t* batch, const float* params,
                            void* workspace, int mode, const float* eps_or_z,
                            unsigned long long seed, const int* step_counter,
                            unsigned char* gen_adj, snd_stream_t stream) {
  SND_CHECK_ARG(plan && params && workspace, "snd_generate: null argument");
  SND_CHECK_ARG(mode >= SND_GEN_SAMPLE && mode <= SND_GEN_GIVEN, "snd_generate: bad mode %d", mode);
  const bool enc = mode == SND_GEN_SAMPLE || mode == SND_GEN_MEAN;
  SND_CHECK_ARG(!enc || (batch && batch->rowptr && batch->colidx && batch->features),
                "snd_generate: modes SAMPLE/MEAN encode a batch (rowptr, colidx, features)");
  SND_CHECK_ARG(mode != SND_GEN_GIVEN || eps_or_z, "snd_generate: mode GIVEN needs z");
  const snd_plan& p = *plan;
  const snd_config_t& c = p.c;
  Ctx x{&p, (char*)workspace, params, nullptr, (hipStream_t)stream};
  const int R = p.R, N = p.N, L = c.latent, RH = p.RH, dj = p.dj, C1 = p.C1;
  const int sd = c.spatial_dim, nf = c.num_feature;
  const long long CP = (long long)N * dj;
  float* zl = p.tref ? x.f("ZL") : x.f("Z");
  if (enc) SND_TRY(p.sg ? encoder_sg_fwd(x, batch) : encoder_generic_fwd(x, batch));
  if (enc && p.small_head)   // the step folds [mu || s] into small_head_fwd; here it is read directly
    SND_TRY(gemm_fwd(x, RH, 2 * L, c.g_hidden, x.f("Hh"), c.g_hidden, x.w("enc.Wms"), 2 * L, B_ROW, x.f("MS"),
                     2 * L, x.w("enc.bms")));
  if (mode == SND_GEN_MEAN) {             // z = mu
    if (hipMemcpy2DAsync(zl, (size_t)L * 4, x.f("MS"), (size_t)2 * L * 4, (size_t)L * 4, RH,
                         hipMemcpyDeviceToDevice, x.s) != hipSuccess) {
      set_error("snd_generate: copy of mu failed");
      return SND_ERR_HIP;
    }
  } else if (mode == SND_GEN_GIVEN) {
    if (hipMemcpyAsync(zl, eps_or_z, (size_t)RH * L * 4, hipMemcpyDeviceToDevice, x.s) !=
        hipSuccess) {
      set_error("snd_generate: copy of z failed");
      return SND_ERR_HIP;
    }
  } else {                                // z = mu + eps exp(s); PRIOR: mu = s = 0
    if (mode == SND_GEN_PRIOR &&
        hipMemsetAsync(x.f("MS"), 0, (size_t)RH * 2 * L * 4, x.s) != hipSuccess) {
      set_error("snd_generate: memset failed");
      return SND_ERR_HIP;
    }
    ReparamFwdArgs a{x.f("MS"), 2 * L, RH, L, eps_or_z, seed, step_counter, x.f("EPS"), zl,
                     x.d("PKL"), nullptr, L};
    a.eps_base = p.eps_base();
    SND_TRY(launch_reparam_fwd(a, x.s));
  }
  if (p.sg) SND_TRY(launch_sg_mean(x.f("ZL"), x.f("ZBAR"), p.B, p.S, L, x.s));   // model.py:177,180
  if (p.tref) {   // J = reshape(z Wp + bp, [B, N, node_h]) (model_joint.py:97)
    TrefProjFwdArgs a{x.f(p.sg ? "ZBAR" : "ZL"), p.B, L, x.w("dec.Wp"), x.w("dec.bp"), CP, x.f("Z")};
    SND_TRY(launch_tref_proj_fwd(a, x.s));
  }
  // decoders (model_joint.py:112-145): conv1d k5 SAME -> BN -> lrelu, sigmoid heads
  SND_TRY(conv_fwd(x, x.f("Z"), dj, dj, "dec.K1", C1, "dec.b1", "dec.bn1.gamma", "dec.bn1.beta",
                   x.f("Y1"), x.f("U1")));
  SND_TRY(conv_fwd(x, x.f("U1"), C1, c.s1, "dec.K2s", c.s2, "dec.b2s", "dec.bn2s.gamma",
                   "dec.bn2s.beta", x.f("Y2S"), x.f("U2S")));
  SND_TRY(conv_fwd(x, x.f("U1") + c.s1, C1, c.n1, "dec.K2n", c.n2, "dec.b2n", "dec.bn2n.gamma",
                   "dec.bn2n.beta", x.f("Y2N"), x.f("U2N")));
  SND_TRY(conv_fwd(x, x.f("U2S"), c.s2, c.s2, "dec.K3s", c.s3, "dec.b3s", "dec.bn3s.gamma",
                   "dec.bn3s.beta", x.f("Y3S"), x.f("U3S")));
  {
    HeadArgs h[2] = {
        {x.f("U3S"), c.s3, c.s3, x.w("dec.Ws"), x.w("dec.bs"), sd, nullptr, sd, (float)R * sd,
         x.f("SHAT"), x.f("DU3S"), c.s3, x.f("PHS"), x.d("PSSES")},
        {x.f("U2N"), c.n2, c.n2, x.w("dec.Wn"), x.w("dec.bn"), nf, nullptr, nf, (float)R * nf,
         x.f("XHAT"), x.f("DU2N"), c.n2, x.f("PHN"), x.d("PSSEN")}};
    SND_TRY(launch_heads(h, 2, R, x.s));
  }
  if (gen_adj) {
    GenAdjArgs a{x.f("Z"), dj, dj, N, p.B, gen_adj};
    SND_TRY(launch_gen_adj(a, x.s));
  }
  return 0;
}

extern "C" int snd_plan_launch(const snd_plan_t* plan, const snd_batch_t* batch,
                               void* workspace, const char* kernel, snd_stream_t stream) {
  SND_CHECK_ARG(plan && batch && workspace && kernel, "snd_plan_launch: null argument");
  SND_TRY(zzt_init_attributes());
  const snd_plan& p = *plan;
  char* ws = (char*)workspace;
  hipStream_t s = (hipStream_t)stream;
  const int L = p.dj;
  if (!strncmp(kernel, "zzt_dense", 9)) {   // zzt_dense | zzt_dense_v<variant> (ZztArgs.variant)
    const ZztStage stg = zzt_stage(ws + p.buf("ZSTAGE"), p.B, p.N, L, p.c.dtype);
    const int variant = kernel[9] == '_' ? atoi(kernel + 11) : 0;   // zzt_dense_v<N>
    ZztArgs za{stg.jrow, stg.jt, p.N, zzt_npad(p.N), p.B, L, (float*)(ws + p.buf("DJD")),
               (double*)(ws + p.buf("PZZT")), stg.colpart, variant, (float*)(ws + p.buf("DJDX"))};
    return launch_zzt_dense(za, p.c.dtype, s);
  }
  if (!strcmp(kernel, "spmm_dxw1")) {   // A @ dP1 (plain SpMM, width h1)
    SpmmArgs a{batch->rowptr, batch->colidx, p.R, (const float*)(ws + p.buf("DP1")), p.c.h1,
               p.c.h1, (float*)(ws + p.buf("DXW1")), p.c.h1, SND_SPMM_PLAIN};
    return launch_spmm(a, s);
  }
  if (!strcmp(kernel, "edge_bf16")) {   // per-edge CE terms of the fast path (A = 1 pairs)
    SND_CHECK_ARG(p.fast, "snd_plan_launch: edge_bf16 needs the bf16 fast path");
    EdgeBfArgs ea{batch->rowptr, batch->colidx, p.R, (const __bf16*)(ws + p.buf("ZB")), p.dj, p.c.pos_weight,
                  (float*)(ws + p.buf("EJ")), (double*)(ws + p.buf("PEDGE")), xcd_nbg(p.N, p.B)};
    ea.row_order = batch->row_order;
    return launch_edge_bf16(ea, s);
  }
  if (!strcmp(kernel, "spmm_bf16")) {   // backward GCN1 SpMM of the fast path: A @ dP1 (bf16)
    SND_CHECK_ARG(p.fast_enc, "snd_plan_launch: spmm_bf16 needs the bf16 fast encoder");
    return spmm_bf16_plain(batch, p.R, p.N, p.B, (const __bf16*)(ws + p.buf("FDP1")), p.c.h1, p.c.h1,
                           (__bf16*)(ws + p.buf("FDXW1")), p.c.h1, s);
  }
  if (!strcmp(kernel, "spmm_bf16_tiled")) {   // the same SpMM on the row tiles (A/B)
    SND_CHECK_ARG(p.fast_enc, "snd_plan_launch: spmm_bf16_tiled needs the bf16 fast encoder");
    SpmmBfArgs a{batch->rowptr, batch->colidx, p.R, (const __bf16*)(ws + p.buf("FDP1")), p.c.h1,
                 p.c.h1, SND_SPMM_PLAIN, (__bf16*)(ws + p.buf("FDXW1")), p.c.h1};
    a.xcd_nbg = xcd_nbg(p.N, p.B);
    use_tiles(a, batch, p.N, p.B);
    return launch_spmm_bf16(a, s);
  }
  if (!strncmp(kernel, "tref_", 5)) {   // graph-latent weight-streaming kernels
    SND_CHECK_ARG(p.tref && !p.sg && p.last_params, "snd_plan_launch: no graph-latent step has run");
    Ctx x{&p, ws, p.last_params, p.last_grads, s};
    const snd_config_t& c = p.c;
    const long long KH = (long long)p.N * p.W, CP = (long long)p.N * p.dj;
    const float adj_scale = (float)(2.0 * (double)c.norm / ((double)p.B * p.N * (double)p.N));
    const __bf16* gb = p.fast_enc ? reinterpret_cast<const __bf16*>(x.f("FG")) : nullptr;
    if (!strcmp(kernel, "tref_head_fwd")) {
      TrefHeadFwdArgs a{gb ? nullptr : x.f("G"), KH, p.B, x.w("enc.Wh"), c.g_hidden, x.w("enc.bh"),
                        x.f("PHF"), gb, p.ldg, p.W, p.N};
      return launch_tref_head_fwd(a, s);
    }
    if (!strcmp(kernel, "tref_head_bwd")) {
      TrefHeadBwdArgs a{gb ? nullptr : x.f("G"), KH, p.B, x.w("enc.Wh"), c.g_hidden, x.f("DH"),
                        x.g("enc.Wh"), gb ? nullptr : x.f("DG"), gb, p.ldg, p.W, p.N,
                        gb ? reinterpret_cast<__bf16*>(x.f("FDG")) : nullptr};
      return launch_tref_head_bwd(a, s);
    }
    if (!strcmp(kernel, "tref_proj_fwd")) {
      TrefProjFwdArgs a{x.f("ZL"), p.B, c.latent, x.w("dec.Wp"), x.w("dec.bp"), CP, x.f("Z")};
      return launch_tref_proj_fwd(a, s);
    }
    if (!strcmp(kernel, "tref_proj_bwd")) {
      TrefProjBwdArgs a{x.f("ZL"), p.B, c.latent, x.w("dec.Wp"), CP, x.f("DZDEC"), x.f("DJD"), x.f("EJ"),
                        adj_scale, x.g("dec.Wp"), x.g("dec.bp"), x.f("PDZ")};
      return launch_tref_proj_bwd(a, s);
    }
  }
  if (!strcmp(kernel, "wgrad_multi")) {   // the last step's weight gradients (current debug bits)
    SND_CHECK_ARG(!p.last_wq.empty(), "snd_plan_launch: no multi-segment weight-gradient launch yet");
    std::vector<WgArgs> q = p.last_wq;
    for (auto& w : q) {
      w.dbg = debug_flags();
      // measurement only: per-workgroup stamps into the fused decoder's head partials
      // (unused by this launch; launch_wgrad_multi checks that 12 words x the workgroups
      // of all its launches fit the buffer)
      const bool st = (w.dbg & (1 << 21)) && p.dec_fused;
      w.stamps = st ? reinterpret_cast<unsigned*>(ws + p.buf("PDHS")) : nullptr;
      w.stamp_words = st ? p.buf_numel("PDHS") : 0;
    }
    return launch_wgrad_multi(q.data(), (int)q.size(), s);
  }
  if (!strcmp(kernel, "head_bwd")) {   // fused backward head (the step's scales)
    SND_CHECK_ARG(p.head_bwd && p.last_params, "snd_plan_launch: head_bwd needs a fused-head step first");
    Ctx x{&p, ws, p.last_params, p.last_grads, s};
    x.zts = p.last_zts;
    const double pairs = (double)p.B * p.N * (double)p.N;
    return head_bwd_fused(x, batch, (float)(2.0 * (double)p.c.norm / pairs),
                          (float)((double)p.c.beta / ((double)p.RH * p.c.latent)));
  }
  if (!strcmp(kernel, "head_fwd")) {   // fused encoder forward tail (device eps, seed 0)
    SND_CHECK_ARG(p.head_fused && p.last_params, "snd_plan_launch: head_fwd needs a fused-head step first");
    Ctx x{&p, ws, p.last_params, p.last_grads, s};
    const ZztStage stg = zzt_stage(ws + p.buf("ZSTAGE"), p.B, p.N, p.dj, p.c.dtype);
    return head_fwd_fused(x, batch, nullptr, 0ull, nullptr, stg);
  }
  if (!strncmp(kernel, "dec:", 4) || !strcmp(kernel, "pack")) {   // fast decoder kernel k
    SND_CHECK_ARG(p.fast && p.last_params, "snd_plan_launch: no fast-path step has run");
    SND_TRY(fast_init_attributes());
    Ctx x{&p, ws, p.last_params, p.last_grads, s};
    if (kernel[0] == 'p') return pack_decoder(x);
    if (!strcmp(kernel, "dec:fwd") || !strcmp(kernel, "dec:bwd")) {
      SND_CHECK_ARG(p.dec_fused, "snd_plan_launch: %s needs the fused decoder", kernel);
      return decoder_fast(x, batch, kernel[4] == 'f' ? 100 : 101);
    }
    return decoder_fast(x, batch, atoi(kernel + 4));
  }
  set_error("snd_plan_launch: unknown kernel '%s'", kernel);
  return SND_ERR_ARG;
}

// the step's final reduction: every slab / column partial -> its gradient block, in one
// launch with the loss terms (snd_train_step); also walked, on placeholder bases, by
// reduce_adam_cover to find the blocks the reduction writes complete
void final_reduce_descs(const Ctx& x, std::vector<ReduceDesc>& rd) {
  const snd_plan& p = *x.p;
  const snd_config_t& c = p.c;
  const int R = p.R, N = p.N, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, L = c.latent;
  const int W = p.W, C1 = p.C1, s1 = c.s1, s2 = c.s2, s3 = c.s3, n1 = c.n1, n2 = c.n2;
  const int sd = c.spatial_dim, nf = c.num_feature;
  const int dj = p.dj, RH = p.RH;
  const long long KH = (long long)N * W;
  const int nc = col_blocks(R), nh = head_blocks(R);
  auto slab = [&](const char* buf, const Split& sp, int Mtot, int N_, const char* wname,
                  int wlen, const char* bname) {
    const float* s0 = x.f(buf);
    rd.push_back({s0, x.g(wname), sp.splits, wlen, (long long)Mtot * N_, 1.f, 0});
    if (bname) rd.push_back({s0 + wlen, x.g(bname), sp.splits, N_, (long long)Mtot * N_, 1.f, 0});
  };
  if (p.sg) {
    slab("SWH", p.sWh, (int)KH + 1, gh, "enc.Wh", (int)KH * gh, "enc.bh");
  } else if (p.fast_enc) {
    encoder_fast_reduce(x, rd);
  } else {
    slab("SW0", p.sW0, f, h0, "enc.W0", f * h0, nullptr);
    slab("SW1", p.sW1, h0 + f, h1, "enc.W1", (h0 + f) * h1, nullptr);
    if (!p.tref) slab("SWH", p.sWh, W + 1, gh, "enc.Wh", W * gh, "enc.bh");
  }
  if (p.tref && !p.sg)   // dbh = sum over graphs of dh
    rd.push_back({x.f("DH"), x.g("enc.bh"), RH, gh, (long long)gh, 1.f, 0});
  if (!p.fast_enc || p.tref) slab("SWMS", p.sWms, gh + 1, 2 * L, "enc.Wms", gh * 2 * L, "enc.bms");
  if (!p.fast) {
    slab("SK1", p.sK1, 5 * dj, C1, "dec.K1", 5 * dj * C1, nullptr);
    slab("SK2S", p.sK2s, 5 * s1, s2, "dec.K2s", 5 * s1 * s2, nullptr);
    slab("SK2N", p.sK2n, 5 * n1, n2, "dec.K2n", 5 * n1 * n2, nullptr);
    slab("SK3S", p.sK3s, 5 * s2, s3, "dec.K3s", 5 * s2 * s3, nullptr);
  }
  auto cols = [&](const char* buf, int stride, int off, int len, const char* dst) {
    rd.push_back({x.f(buf) + off, x.g(dst), nc, len, (long long)stride, 1.f, 0});
  };
  if (!p.fast_enc && !p.sg) {
    cols("PENC1", 2 * W + 2 * h1, 0, W, "enc.bne.gamma");
    cols("PENC1", 2 * W + 2 * h1, W, W, "enc.bne.beta");
    cols("PENC1", 2 * W + 2 * h1, 2 * W, h1, "enc.bn1.gamma");
    cols("PENC1", 2 * W + 2 * h1, 2 * W + h1, h1, "enc.bn1.beta");
    cols("PENC0", 2 * h0, 0, h0, "enc.bn0.gamma");
    cols("PENC0", 2 * h0, h0, h0, "enc.bn0.beta");
  }
  auto dec = [&](const char* buf, int w, const char* g, const char* b, const char* bias) {
    cols(buf, 3 * w, 0, w, g);
    cols(buf, 3 * w, w, w, b);
    cols(buf, 3 * w, 2 * w, w, bias);
  };
  if (p.fast) {
    decoder_fast_reduce(x, rd);
  } else {
    dec("PDEC3", s3, "dec.bn3s.gamma", "dec.bn3s.beta", "dec.b3s");
    dec("PDEC2S", s2, "dec.bn2s.gamma", "dec.bn2s.beta", "dec.b2s");
    dec("PDEC2N", n2, "dec.bn2n.gamma", "dec.bn2n.beta", "dec.b2n");
    dec("PDEC1", C1, "dec.bn1.gamma", "dec.bn1.beta", "dec.b1");
    const int hs = s3 * sd + sd, hn = n2 * nf + nf;
    rd.push_back({x.f("PHS"), x.g("dec.Ws"), nh, s3 * sd, (long long)hs, 1.f, 0});
    rd.push_back({x.f("PHS") + s3 * sd, x.g("dec.bs"), nh, sd, (long long)hs, 1.f, 0});
    rd.push_back({x.f("PHN"), x.g("dec.Wn"), nh, n2 * nf, (long long)hn, 1.f, 0});
    rd.push_back({x.f("PHN") + n2 * nf, x.g("dec.bn"), nh, nf, (long long)hn, 1.f, 0});
  }
}

// Which blocks the final reduction writes complete: its descriptors built on placeholder
// bases (offsets, not addresses), every element of a block written exactly once, by a
// descriptor that stores (no accumulate).  Structural, so computed once per plan.
void reduce_adam_cover(snd_plan& p) {
  const uintptr_t wsb = (uintptr_t)1 << 44, gb = (uintptr_t)1 << 45;
  Ctx x{&p, (char*)wsb, (const float*)((uintptr_t)1 << 46), (float*)gb, nullptr};
  std::vector<ReduceDesc> rd;
  final_reduce_descs(x, rd);
  std::vector<unsigned char> hits((size_t)p.pcount, 0);
  std::vector<char> bad(p.blocks.size(), 0);
  for (const ReduceDesc& d : rd) {
    const long long o = d.dst - (float*)gb;
    const int rows = d.rows > 0 ? d.rows : 1;
    for (int r = 0; r < rows; ++r)
      for (int i = 0; i < d.len; ++i) {
        const long long k = o + (long long)r * d.dst_rs + i;
        if (k < 0 || k >= p.pcount) continue;
        if (hits[(size_t)k] < 2) ++hits[(size_t)k];
        if (d.accumulate) hits[(size_t)k] = 2;
      }
  }
  p.radam.assign(p.blocks.size(), 0);
  for (size_t b = 0; b < p.blocks.size(); ++b) {
    const Block& bl = p.blocks[b];
    if (p.stream_fused(bl.name) || bl.numel == 0) continue;
    bool ok = true;
    for (long long k = bl.off; k < bl.off + bl.numel && ok; ++k) ok = hits[(size_t)k] == 1;
    p.radam[b] = ok;
  }
}

// the final reduction's fused-Adam descriptors: those whose destination lies in a
// reduce-fused block (a descriptor never straddles blocks)
unsigned long long reduce_adam_mask(const snd_plan& p, const std::vector<ReduceDesc>& rd, const float* G) {
  unsigned long long mask = 0;
  for (size_t i = 0; i < rd.size() && i < 64; ++i) {
    const long long o = rd[i].dst - G;
    for (size_t b = 0; b < p.blocks.size(); ++b)
      if (o >= p.blocks[b].off && o < p.blocks[b].off + p.blocks[b].numel && p.reduce_fused(b))
        mask |= 1ull << i;
  }
  return mask;
}

extern "C" int snd_train_step(const snd_plan_t* plan, const snd_batch_t* batch,
                              const float* params, float* grads, void* workspace,
                              const float* eps, unsigned long long seed, int* step_counter,
                              double* losses, snd_stream_t stream) {
  SND_CHECK_ARG(plan && batch && params && grads && workspace && losses,
                "snd_train_step: null argument");
  SND_CHECK_ARG(batch->rowptr && batch->colidx && batch->features && batch->feature_truth &&
                    batch->spatial_truth, "snd_train_step: incomplete batch");
  SND_TRY(zzt_init_attributes());
  const snd_plan& p = *plan;
  const snd_config_t& c = p.c;
  Ctx x{&p, (char*)workspace, params, grads, (hipStream_t)stream};
  p.last_params = params;
  p.last_grads = grads;
  int nev = 0;
  // Side-stream branches are opt-in (debug bit 1024): on ROCm 7.2 a captured
  // graph spreads them over several hardware queues, and the cross-queue
  // dependencies cost more (5-12 us each, measured) than the overlap saves.
  if (p.fast && (debug_flags() & 1024)) {
    init_concurrency(p, x.s);
    if (p.conc == 1) { x.side = p.side; x.nev = &nev; }
  }
  // the concurrent decoder needs the side stream, created by a non-capturing step
  bool cdec = false;
  if (p.conc_dec_on() && !x.side) {
    init_concurrency(p, x.s);
    cdec = p.conc == 1;
    if (cdec) x.nev = &nev;
  }
  x.zts = cdec ? p.zzt_ts_conc : p.zzt_ts;
  p.last_zts = x.zts;
  // single stream: every fast-path weight gradient waits for one launch before the
  // reduction (debug bit 4096: one launch per weight, as before)
  std::vector<WgArgs> wq;
  if (p.fast && !x.side && !(debug_flags() & (4096 | 8192))) {
    wq.reserve(kMaxWgMulti);
    x.wq = &wq;
  }
  const int R = p.R, N = p.N, f = c.f_in, h0 = c.h0, h1 = c.h1, gh = c.g_hidden, L = c.latent;
  const int W = p.W, C1 = p.C1, s1 = c.s1, s2 = c.s2, s3 = c.s3, n1 = c.n1, n2 = c.n2;
  const int sd = c.spatial_dim, nf = c.num_feature;
  const int dj = p.dj, RH = p.RH;
  const long long KH = (long long)N * W, CP = (long long)N * dj;   // tref: flat(G) / flat(J) widths
  const int* rp = batch->rowptr;
  const int* ci = batch->colidx;
  const float* X = batch->features;
  if (p.fast) {
    SND_TRY(fast_init_attributes());
    // bf16 weight images of this step's parameters (inside the encoder front when fused)
    // (or inside the gcn0 launch: C5 step 0.3726-0.3730 -> 0.3658-0.3683 ms, debug bit 1 << 28 restores pack_kernel)
    if (!p.front_fused && !p.pack_in_gcn0) SND_TRY(pack_decoder(x));
  }

  // =============================== forward ===============================
  if (p.sg) {
    SND_TRY(encoder_sg_fwd(x, batch));
  } else if (p.fast_enc) {
    SND_TRY(encoder_fast_fwd(x, batch));
  } else {
    SND_TRY(encoder_generic_fwd(x, batch));
  }
  if (p.fast_enc && p.tref) {   // graph heads on the fast encoder's bf16 G
    TrefHeadFwdArgs a{nullptr, KH, p.B, x.w("enc.Wh"), gh, x.w("enc.bh"), x.f("PHF"),
                      reinterpret_cast<const __bf16*>(x.f("FG")), p.ldg, W, N};
    SND_TRY(launch_tref_head_fwd(a, x.s));
    const ReduceDesc rd{x.f("PHF"), x.f("Hh"), tref_head_fwd_blocks(KH, gh), RH * gh,
                        (long long)RH * gh, 1.f, 0, 0, 0, 0};
    SND_TRY(launch_reduce(&rd, 1, x.s));
    if (!p.small_head)
      SND_TRY(gemm_fwd(x, RH, 2 * L, gh, x.f("Hh"), gh, x.w("enc.Wms"), 2 * L, B_ROW, x.f("MS"), 2 * L,
                       x.w("enc.bms")));
  }
  // z = mu + eps exp(s) (model.py:159); KL partials (optimizer.py:193)
  const ZztStage stg = zzt_stage(x.ws + p.buf("ZSTAGE"), p.B, N, dj, c.dtype);
  if (p.tref) {
    if (p.small_head) {   // [mu || s] = h Wms + bms, z and the KL terms in one launch
      SmallHeadFwdArgs a{x.f("Hh"), RH, gh, x.w("enc.Wms"), x.w("enc.bms"), L, x.f("MS"), eps, seed,
                         step_counter, p.eps_base(), x.f("EPS"), x.f("ZL"), x.d("PKL")};
      a.stepn = x.stepn();
      SND_TRY(launch_small_head_fwd(a, x.s));
    } else {   // z [B, L] (model_joint.py:89); SND_SGJOINT: [B*S, L] (model.py:157)
      ReparamFwdArgs a{x.f("MS"), 2 * L, RH, L, eps, seed, step_counter, x.f("EPS"), x.f("ZL"),
                       x.d("PKL"), nullptr, L};
      a.eps_base = p.eps_base();
      a.stepn = x.stepn();
      SND_TRY(launch_reparam_fwd(a, x.s));
    }
    // SND_SGJOINT: mean over the copies before the (affine) projection (model.py:177,180)
    if (p.sg) SND_TRY(launch_sg_mean(x.f("ZL"), x.f("ZBAR"), p.B, p.S, L, x.s));
    {   // J = reshape(z Wp + bp, [B, N, node_h]) (model_joint.py:97)
      TrefProjFwdArgs a{x.f(p.sg ? "ZBAR" : "ZL"), p.B, L, x.w("dec.Wp"), x.w("dec.bp"), CP, x.f("Z")};
      SND_TRY(launch_tref_proj_fwd(a, x.s));
    }
    if (p.fast) {   // bf16 J for the decoder + zz^T staging images
      ReparamPrepArgs a{x.f("Z"), dj, N, zzt_npad(N), p.B, dj, nullptr, 0, nullptr, nullptr,
                        nullptr, (__bf16*)x.f("ZB"), (__bf16*)stg.jrow, (__bf16*)stg.jt, stg.colpart,
                        nullptr, 1};
      SND_TRY(launch_reparam_prep(a, zzt_dp(dj), x.s));
    }
  } else if (p.head_fused) {
    SND_TRY(head_fwd_fused(x, batch, eps, seed, step_counter, stg));
  } else if (p.fast) {   // fused with the zz^T staging images
    ReparamPrepArgs a{x.f("MS"), 2 * L, N, zzt_npad(N), p.B, L, eps, seed, step_counter, x.f("Z"),
                      x.f("EPS"), (__bf16*)x.f("ZB"), (__bf16*)stg.jrow, (__bf16*)stg.jt, stg.colpart,
                      x.d("PKL")};
    a.eps_base = p.eps_base();
    a.stepn = x.stepn();
    SND_TRY(launch_reparam_prep(a, zzt_dp(L), x.s));
  } else {
    ReparamFwdArgs a{x.f("MS"), 2 * L, R, L, eps, seed, step_counter, x.f("EPS"), x.f("Z"),
                     x.d("PKL"), nullptr, L};
    a.eps_base = p.eps_base();
    a.stepn = x.stepn();
    SND_TRY(launch_reparam_fwd(a, x.s));
  }
  // inner-product decoder + CE (fused) and per-edge terms
  int edge_mark = -1;
  {
    // per-edge terms on the side stream, overlapping the dense kernel / decoder
    SND_TRY(fork(x));
    if (p.head_bwd || p.edge_reparam) {
      // per-edge terms run inside head_bwd_kernel (the backward head) / edge_reparam_bwd_kernel
    } else if (p.fast) {
      EdgeBfArgs ea{rp, ci, R, (const __bf16*)x.f("ZB"), dj, c.pos_weight, x.f("EJ"), x.d("PEDGE"),
                    xcd_nbg(N, p.B)};
      ea.row_order = batch->row_order;
      SND_TRY(launch_edge_bf16(ea, side(x)));
    } else {
      EdgeArgs ea{rp, ci, R, x.f("Z"), dj, c.pos_weight, x.f("EJ"), x.d("PEDGE")};
      SND_TRY(launch_edge(ea, side(x)));
    }
    edge_mark = mark(x);
    if (edge_mark < -1) return SND_ERR_HIP;
    if (!p.fast) SND_TRY(launch_zzt_prep(x.f("Z"), p.B, N, dj, c.dtype, stg, x.s));
    ZztArgs za{stg.jrow, stg.jt, N, zzt_npad(N), p.B, dj, x.f("DJD"), x.d("PZZT"), stg.colpart, 0,
               x.f("DJDX")};
    za.tsplit = x.zts;
    // concurrent decoder: the fused decoder on the side stream beside zz^T (forked after
    // the staging that both read, joined before the backward head that reads both)
    // (the roles swapped -- zz^T on the side stream, the decoder chain on main, so that the
    // main stream has no cross-queue wait before the decoder -- measured 0.1163-0.1183 ->
    // 0.1353-0.1356 ms: zz^T, dispatched first, takes the CUs the decoder needs; round 6)
    if (cdec) {
      SND_TRY(fork_to(x, p.side));
      Ctx xd = x;
      xd.s = p.side;
      xd.side = nullptr;
      SND_TRY(decoder_fast(xd, batch));
    }
    // the column-split sum is folded into head_bwd / reparam_bwd_fast (node latent, fast encoder)
    SND_TRY(launch_zzt_dense(za, c.dtype, x.s, p.fast_enc && !p.tref));
    // measurement only (debug bit 1 << 17): the same zz^T launch again (it recomputes the
    // same partials), so a kernel trace shows a warm in-step launch beside the first one
    if (debug_flags() & (1 << 17)) SND_TRY(launch_zzt_dense(za, c.dtype, x.s, p.fast_enc && !p.tref));
    if (cdec) SND_TRY(join_from(x, p.side));
  }
  if (p.fast) {
    if (!cdec) SND_TRY(decoder_fast(x, batch));
  } else {
    // decoders (model_joint.py:112-145): conv1d k5 SAME -> BN -> lrelu
    SND_TRY(conv_fwd(x, x.f("Z"), dj, dj, "dec.K1", C1, "dec.b1", "dec.bn1.gamma", "dec.bn1.beta",
                     x.f("Y1"), x.f("U1")));
    SND_TRY(conv_fwd(x, x.f("U1"), C1, s1, "dec.K2s", s2, "dec.b2s", "dec.bn2s.gamma",
                     "dec.bn2s.beta", x.f("Y2S"), x.f("U2S")));
    SND_TRY(conv_fwd(x, x.f("U1") + s1, C1, n1, "dec.K2n", n2, "dec.b2n", "dec.bn2n.gamma",
                     "dec.bn2n.beta", x.f("Y2N"), x.f("U2N")));
    SND_TRY(conv_fwd(x, x.f("U2S"), s2, s2, "dec.K3s", s3, "dec.b3s", "dec.bn3s.gamma",
                     "dec.bn3s.beta", x.f("Y3S"), x.f("U3S")));
    // sigmoid heads + MSE + their backward (optimizer.py:149,153)
    {
      HeadArgs h[2] = {
          {x.f("U3S"), s3, s3, x.w("dec.Ws"), x.w("dec.bs"), sd, batch->spatial_truth, sd,
           (float)R * sd, x.f("SHAT"), x.f("DU3S"), s3, x.f("PHS"), x.d("PSSES")},
          {x.f("U2N"), n2, n2, x.w("dec.Wn"), x.w("dec.bn"), nf, batch->feature_truth, nf,
           (float)R * nf, x.f("XHAT"), x.f("DU2N"), n2, x.f("PHN"), x.d("PSSEN")}};
      SND_TRY(launch_heads(h, 2, R, x.s));
    }
    // =============================== backward ==============================
    {
      DecBwdArgs d{x.f("DU3S"), s3, x.f("Y3S"), s3, x.w("dec.bn3s.gamma"), x.w("dec.bn3s.beta"), s3,
                   x.f("DY3S"), s3, x.f("PDEC3")};
      SND_TRY(launch_dec_bwd(&d, 1, R, x.s));
    }
    SND_TRY(conv_bwd_data(x, x.f("DY3S"), s3, "dec.K3s", s2, x.f("DU2S"), s2));
    SND_TRY(conv_wgrad(x, x.f("U2S"), s2, s2, x.f("DY3S"), s3, x.f("SK3S"), p.sK3s));
    {
      DecBwdArgs d[2] = {
          {x.f("DU2S"), s2, x.f("Y2S"), s2, x.w("dec.bn2s.gamma"), x.w("dec.bn2s.beta"), s2,
           x.f("DY2S"), s2, x.f("PDEC2S")},
          {x.f("DU2N"), n2, x.f("Y2N"), n2, x.w("dec.bn2n.gamma"), x.w("dec.bn2n.beta"), n2,
           x.f("DY2N"), n2, x.f("PDEC2N")}};
      SND_TRY(launch_dec_bwd(d, 2, R, x.s));
    }
    SND_TRY(conv_bwd_data(x, x.f("DY2S"), s2, "dec.K2s", s1, x.f("DU1"), C1));
    SND_TRY(conv_bwd_data(x, x.f("DY2N"), n2, "dec.K2n", n1, x.f("DU1") + s1, C1));
    SND_TRY(conv_wgrad(x, x.f("U1"), C1, s1, x.f("DY2S"), s2, x.f("SK2S"), p.sK2s));
    SND_TRY(conv_wgrad(x, x.f("U1") + s1, C1, n1, x.f("DY2N"), n2, x.f("SK2N"), p.sK2n));
    {
      DecBwdArgs d{x.f("DU1"), C1, x.f("Y1"), C1, x.w("dec.bn1.gamma"), x.w("dec.bn1.beta"), C1,
                   x.f("DY1"), C1, x.f("PDEC1")};
      SND_TRY(launch_dec_bwd(&d, 1, R, x.s));
    }
    SND_TRY(conv_bwd_data(x, x.f("DY1"), C1, "dec.K1", dj, x.f("DZDEC"), dj));
    SND_TRY(conv_wgrad(x, x.f("Z"), dj, dj, x.f("DY1"), C1, x.f("SK1"), p.sK1));
  }
  // reparameterisation + KL backward; dJ = conv-decoder grad + zz^T CE grad
  const double pairs = (double)p.B * N * (double)N;
  // dL/dJ_i = sum_j (G_ij + G_ji) J_j = 2 sum_j G_ij J_j (G symmetric)
  const float adj_scale = (float)(2.0 * (double)c.norm / pairs);
  const float kl_scale = (float)((double)c.beta / ((double)RH * L));
  SND_TRY(wait_mark(x, edge_mark));   // EJ
  if (p.fast_enc && !p.tref) {
    SND_TRY(encoder_fast_bwd(x, batch, adj_scale, kl_scale));
  } else {
    if (p.tref) {
      {   // d_sg_lin1 backward: dWp, dbp written; dz partials per block
        TrefProjBwdArgs a{x.f(p.sg ? "ZBAR" : "ZL"), p.B, L, x.w("dec.Wp"), CP, x.f("DZDEC"), x.f("DJD"),
                          x.f("EJ"), adj_scale, x.g("dec.Wp"), x.g("dec.bp"), x.f("PDZ")};
        if (p.stream_fused("dec.Wp")) a.adam = fused_adam(x, "dec.Wp", step_counter);
        if (p.stream_fused("dec.bp")) a.adam_b = fused_adam(x, "dec.bp", step_counter);
        SND_TRY(launch_tref_proj_bwd(a, x.s));
        if (p.ev_proj && hipEventRecord(p.ev_proj, x.s) != hipSuccess) {
          set_error("train step: grad event (dec.Wp) record failed");
          return SND_ERR_HIP;
        }
        const int rz = p.B;   // rows of the projection's input: B graphs
        const ReduceDesc rd{x.f("PDZ"), x.f(p.sg ? "DZBAR" : "DZL"), tref_proj_bwd_blocks(CP), rz * L,
                            (long long)rz * L, 1.f, 0, 0, 0, 0};
        SND_TRY(launch_reduce(&rd, 1, x.s));
        if (p.sg) SND_TRY(launch_sg_spread(x.f("DZBAR"), x.f("DZL"), p.B, p.S, L, x.s));
      }
      if (p.small_head) {   // reparam/KL backward + the Wms slab, then dh
        SmallHeadBwdArgs a{x.f("Hh"), RH, gh, x.w("enc.Wms"), L, x.f("MS"), x.f("EPS"), x.f("DZL"), kl_scale,
                           x.f("DMS"), x.f("SWMS"), x.f("DH")};
        SND_TRY(launch_small_head_bwd(a, x.s));
      } else {
        ReparamBwdArgs a{x.f("MS"), 2 * L, RH, L, x.f("EPS"), x.f("DZL"), nullptr, nullptr, 0.f,
                         kl_scale, x.f("DMS"), 2 * L};
        SND_TRY(launch_reparam_bwd(a, x.s));
      }
    } else {
      ReparamBwdArgs a{x.f("MS"), 2 * L, R, L, x.f("EPS"), x.f("DZDEC"), x.f("DJD"), x.f("EJ"),
                       adj_scale, kl_scale, x.f("DMS"), 2 * L};
      SND_TRY(launch_reparam_bwd(a, x.s));
    }
    if (!p.small_head) {
      SND_TRY(gemm_wgrad(x, x.f("Hh"), gh, gh, true, x.f("DMS"), 2 * L, 2 * L, x.f("SWMS"), p.sWms, RH));
      SND_TRY(gemm_fwd(x, RH, gh, 2 * L, x.f("DMS"), 2 * L, x.w("enc.Wms"), 2 * L, B_COL, x.f("DH"), gh,
                       nullptr));
    }
    if (p.sg) {
      SND_TRY(encoder_sg_bwd(x, batch));
    } else if (p.tref) {   // dWh written complete; dG = dh Wh^T per graph
      TrefHeadBwdArgs a{x.f("G"), KH, p.B, x.w("enc.Wh"), gh, x.f("DH"), x.g("enc.Wh"), x.f("DG")};
      if (p.fast_enc) {   // bf16 G in, bf16 dG rows out (the fast encoder's operands)
        a.g = nullptr; a.dg = nullptr;
        a.gb = reinterpret_cast<const __bf16*>(x.f("FG")); a.ldg = p.ldg; a.W = W; a.npg = N;
        a.dgb = reinterpret_cast<__bf16*>(x.f("FDG"));
      }
      if (p.stream_fused("enc.Wh")) a.adam = fused_adam(x, "enc.Wh", step_counter);
      SND_TRY(launch_tref_head_bwd(a, x.s));
      if (p.ev_head && hipEventRecord(p.ev_head, x.s) != hipSuccess) {
        set_error("train step: grad event (enc.Wh) record failed");
        return SND_ERR_HIP;
      }
    } else {
      SND_TRY(gemm_wgrad(x, x.f("G"), W, W, true, x.f("DH"), gh, gh, x.f("SWH"), p.sWh));
      SND_TRY(gemm_fwd(x, R, W, gh, x.f("DH"), gh, x.w("enc.Wh"), gh, B_COL, x.f("DG"), W, nullptr));
    }
  }
  if (p.fast_enc && p.tref) {
    SND_TRY(encoder_fast_bwd_tail(x, batch));
  } else if (!p.fast_enc && !p.sg) {
    {
      EncBwdArgs a{x.f("DG"), W, x.f("H2"), W, x.w("enc.bne.gamma"), W, x.f("P1"), h1,
                   x.w("enc.bn1.gamma"), h1, x.f("DP1"), h1, x.f("PENC1"), 1};
      SND_TRY(launch_enc_bwd(a, R, x.s));
    }
    {
      SpmmArgs a{rp, ci, R, x.f("DP1"), h1, h1, x.f("DXW1"), h1, SND_SPMM_PLAIN};
      SND_TRY(launch_spmm(a, x.s));
    }
    SND_TRY(gemm_wgrad(x, x.f("H1"), h0 + f, h0 + f, false, x.f("DXW1"), h1, h1, x.f("SW1"), p.sW1));
    SND_TRY(gemm_fwd(x, R, h0, h1, x.f("DXW1"), h1, x.w("enc.W1"), h1, B_COL, x.f("DH1"), h0,
                     nullptr));
    {
      EncBwdArgs a{x.f("DH1"), h0, nullptr, 0, nullptr, 0, x.f("P0"), h0, x.w("enc.bn0.gamma"), h0,
                   x.f("DP0"), h0, x.f("PENC0"), 0};
      SND_TRY(launch_enc_bwd(a, R, x.s));
    }
    {
      SpmmArgs a{rp, ci, R, x.f("DP0"), h0, h0, x.f("DXW0"), h0, SND_SPMM_PLAIN};
      SND_TRY(launch_spmm(a, x.s));
    }
    SND_TRY(gemm_wgrad(x, X, f, f, false, x.f("DXW0"), h0, h0, x.f("SW0"), p.sW0));
  }

  SND_TRY(join(x));   // weight-gradient slabs from the side stream
  if (x.wq && !x.wq->empty()) {
    // largest weight first: its workgroups start in the first wave of the launch
    // except the k = 5 weights with narrow outputs (the decoder's conv2): the round-5 stamps
    // (tools/wg_stamps.py) measured their workgroups longest, 20 us against 10-15, so they
    // start first (C2 step 0.2178 -> 0.2168 ms; host debug bit 1 << 25: the plain order)
    const bool k5n = !(debug_flags() & (1 << 25));
    auto key = [k5n](const WgArgs& u) {
      const long long c = (long long)u.T * u.K * u.N;
      return k5n && u.T == 5 && u.N <= 32 && u.K >= 32 ? 8 * c : c;
    };
    std::stable_sort(x.wq->begin(), x.wq->end(), [&](const WgArgs& u, const WgArgs& v) { return key(u) > key(v); });
    SND_TRY(launch_wgrad_multi(x.wq->data(), (int)x.wq->size(), x.s));
    p.last_wq = *x.wq;
  }

  // ======================= deterministic gradient reduction =================
  std::vector<ReduceDesc> rd;
  final_reduce_descs(x, rd);
  const int nh = head_blocks(R);
  const int n_kl = (p.fast && !p.tref) ? reparam_prep_blocks(p.B, zzt_npad(N))
                   : (p.small_head ? small_head_fwd_blocks(L) : reparam_blocks(RH, L));
  FinalizeArgs fa{x.d("PZZT"), p.B * (zzt_npad(N) / 128) * (c.dtype == SND_BF16 ? x.zts : 1) * zzt_wpb(dj, c.dtype), x.d("PEDGE"),
                  p.head_bwd ? head_tiles(R) : (p.fast ? edge_bf16_blocks(R) : edge_blocks(R, dj)),
                  x.d("PKL"), n_kl, x.d(p.dec_fused ? "PDSSES" : "PSSES"),
                  x.d(p.dec_fused ? "PDSSEN" : "PSSEN"), p.dec_fused ? p.dtiles : nh,
                  rp, p.B, N, L, sd, nf, c.beta, c.norm, losses, grads + p.pcount, step_counter,
                  (double)RH * L};
  const unsigned long long amask = p.fuse_m ? reduce_adam_mask(p, rd, grads) : 0ull;
  if (amask) {   // + TF1 Adam of the blocks it completes (snd_plan_fuse_adam)
    SND_CHECK_ARG(step_counter && rd.size() <= 64, "train step: fused Adam needs the step counter");
    const ReduceAdam ra{grads, const_cast<float*>(params), p.fuse_m, p.fuse_v, p.fuse_lr, p.fuse_b1,
                        p.fuse_b2, p.fuse_eps, reinterpret_cast<const int*>(x.f("STEPN")), amask};
    return launch_reduce(rd.data(), (int)rd.size(), x.s, &fa, &ra);
  }
  return launch_reduce(rd.data(), (int)rd.size(), x.s, &fa);   // + loss terms in one launch
}
