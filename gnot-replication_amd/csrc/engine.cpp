// GNOT engine: the native host runtime behind the C ABI (include/gnot_hip.h).
//
// It owns no device memory.  From the constructor arguments (reference model.py:143) it derives the
// canonical Linear list (state_dict order), from the batch offsets (the packed replacement for
// utils.py:3-4 / main.py:60-89 padding) it carves one caller-provided workspace into named
// activation buffers, builds every small device table once (weight-pack jobs, chain layer tables,
// weight-gradient job lists, point-segment lists) and then runs the whole forward
// (model.py:154-173) and backward as a fixed sequence of kernel launches on the caller's stream —
// no allocation, no host sync, capturable into a hipGraph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/gnot_hip.h"
#include "gnot_kernels.h"

namespace gnot {

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define GNOT_CK(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail(GNOT_E_HIP, std::string(#expr) + " -> " + hipGetErrorString(e_));             \
  } while (0)

static inline long r4(long x) { return (x + 3) & ~3L; }
static inline int tiles16(int x) { return (x + 15) / 16; }

constexpr int kSeg = 256;            // points per attention segment (state slab / apply block)
constexpr int kWgradChunk = 1024;    // points per split of the weight-gradient GEMM
constexpr int kWgradMaxSplits = 64;

struct Img {                 // one packed MFMA A-operand image in the packed arena
  size_t off4 = 0;           // offset in float4 units
  int OT = 0, KT = 0;
  const float4* p = nullptr;
};

struct Buf {
  size_t off = 0;            // bytes
  long ld = 0;
  float* p = nullptr;
};

struct WgradGroup {
  std::vector<WgradJob> jobs;
  int total_waves = 0, total_red = 0;
  size_t slab_floats = 0;
  // device copies
  WgradJob* d_jobs = nullptr;
  int* d_wave_prefix = nullptr;
  int* d_red_prefix = nullptr;
  std::vector<int> wave_prefix, red_prefix;
};

struct ChainTable {
  std::vector<ChainLayer> host;
  ChainLayer* dev = nullptr;
  int KT0 = 1, OTL = 1, nchains = 1, in_dim = 0, out_dim = 0;
};

}  // namespace gnot

using namespace gnot;

struct gnot_plan {
  gnot_config c{};
  int D = 0, H = 0, dh = 0, E = 0, NL = 0, L = 0, I = 0, KI = 0, DT = 0;
  int in = 0, th = 0, F = 0, out = 0;
  std::vector<int> lin_o, lin_i;   // out / in features per canonical Linear
  std::vector<const float*> W, b;
  bool params_bound = false;

  // batch
  int B = 0;
  long P = 0;
  std::vector<long> xoff;
  std::vector<std::vector<long>> fnoff;
  std::vector<long> Q;
  bool training = true;
  bool batch_set = false;

  // workspace layout
  size_t ws_need = 0;
  char* ws = nullptr;
  std::map<std::string, Buf> bufs;
  std::vector<std::string> buf_order;

  // packed weights
  size_t packed4 = 0, pbias = 0;
  std::vector<PackJob> pack_jobs;       // dst/bias_dst hold OFFSETS until bind
  std::vector<size_t> pack_dst_off4, pack_bias_off;
  std::vector<int> pack_prefix;
  int pack_tiles = 0;
  // images
  std::vector<Img> fwd_img, T_img;      // per canonical linear (fwd_img unused for attention q/k/v)
  std::vector<size_t> fwd_bias;         // per canonical linear: offset of padded bias (floats) in pbias
  struct AttnImgs { Img qkv, q, o; std::vector<Img> kv; size_t bqkv = 0, bq = 0, bo = 0; std::vector<size_t> bkv; };
  std::vector<AttnImgs> cross_img, self_img;

  // grads
  std::vector<long> grad_off;           // 2 per linear
  long grad_floats = 0;

  // device tables
  ChainTable ch_gate, ch_x, ch_out;
  std::vector<ChainTable> ch_fn, ch_m1, ch_m2;
  std::vector<int4> qchunks;
  std::vector<int> qchunk_off;
  std::vector<std::vector<int4>> fchunks;
  std::vector<std::vector<int>> fchunk_off;
  WgradGroup wg_out, wg_x, wg_gate;
  std::vector<WgradGroup> wg_fn;
  std::vector<WgradGroup> wg_m1, wg_m2, wg_self, wg_cross;
  size_t table_bytes = 0;
  size_t slab_state_floats = 0, slab_wgrad_floats = 0;
  int4* d_qchunks = nullptr;
  int* d_qchunk_off = nullptr;
  std::vector<int4*> d_fchunks;
  std::vector<int*> d_fchunk_off;
  long* d_xoff = nullptr;
  std::vector<long*> d_fnoff;
  PackJob* d_pack_jobs = nullptr;
  int* d_pack_prefix = nullptr;
  bool ws_bound = false;
  bool packed = false;
  bool fwd_done = false;

  // ------------------------------------------------------------------ canonical indices
  int lin_x(int j) const { return j; }
  int lin_g(int j) const { return NL + j; }
  int lin_fn(int i, int j) const { return 2 * NL + i * NL + j; }
  int blk0() const { return 2 * NL + I * NL; }
  int per_block() const { return 6 + 2 * KI + 2 * E * NL; }
  int lin_cq(int l) const { return blk0() + l * per_block(); }
  int lin_co(int l) const { return lin_cq(l) + 1; }
  int lin_ck(int l, int i) const { return lin_cq(l) + 2 + i; }
  int lin_cv(int l, int i) const { return lin_cq(l) + 2 + KI + i; }
  int lin_sq(int l) const { return lin_cq(l) + 2 + 2 * KI; }
  int lin_so(int l) const { return lin_sq(l) + 1; }
  int lin_sk(int l) const { return lin_sq(l) + 2; }
  int lin_sv(int l) const { return lin_sq(l) + 3; }
  int lin_f1(int l, int e, int j) const { return lin_sq(l) + 4 + e * NL + j; }
  int lin_f2(int l, int e, int j) const { return lin_sq(l) + 4 + E * NL + e * NL + j; }
  int lin_out(int j) const { return blk0() + L * per_block() + j; }
  int n_lin() const { return lin_out(NL - 1) + 1; }

  std::string final_query() const {
    return L > 0 ? "b" + std::to_string(L - 1) + ".query2" : std::string("query0");
  }
  std::string block_query(int l) const {   // query entering block l
    return l == 0 ? std::string("query0") : "b" + std::to_string(l - 1) + ".query2";
  }
  float* P_(const char* name) const { return bufs.at(name).p; }
  float* P_(const std::string& name) const { return bufs.at(name).p; }
};

// ====================================================================== construction
static void add_linear(gnot_plan* p, int out, int in) {
  p->lin_o.push_back(out);
  p->lin_i.push_back(in);
}

extern "C" int gnot_plan_create(const gnot_config* cfg, gnot_plan** out) {
  if (!cfg || !out) return fail(GNOT_E_INVALID, "null argument");
  const gnot_config& c = *cfg;
  if (c.n_attn_hidden_dim != c.n_mlp_hidden_dim || c.n_attn_hidden_dim != c.n_input_hidden_dim)
    return fail(GNOT_E_INVALID,
                "n_attn_hidden_dim, n_mlp_hidden_dim and n_input_hidden_dim must be equal (the residual "
                "adds of model.py:131/137 need it)");
  const int D = c.n_attn_hidden_dim;
  if (c.n_head <= 0 || D % c.n_head != 0)
    return fail(GNOT_E_INVALID, "n_embed should be divisible by head");   // model.py:41
  const int dh = D / c.n_head;
  if (!(D == 32 || D == 48 || D == 64 || D == 128 || D == 256))
    return fail(GNOT_E_INVALID, "hidden width must be one of 32, 48, 64, 128, 256 on the MI355X kernels");
  if (!(dh == 4 || dh == 8 || dh == 16 || dh == 32 || dh == 48 || dh == 64))
    return fail(GNOT_E_INVALID, "head width d/n_head must be one of 4, 8, 16, 32, 48, 64");
  if (c.n_expert < 1 || c.n_attn_layers < 0 || c.n_input_functions < 0 || c.n_input_functions > 8)
    return fail(GNOT_E_INVALID, "bad n_expert / n_attn_layers / n_input_functions");
  if (c.input_dim + c.theta_dim > D || c.input_dim > D || c.input_func_dim > D || c.out_dim > D ||
      c.n_expert > D || c.input_dim < 1 || c.out_dim < 1)
    return fail(GNOT_E_INVALID, "input/output widths must be in [1, hidden width]");
  gnot_plan* p = new gnot_plan();
  p->c = c;
  p->D = D; p->H = c.n_head; p->dh = dh; p->E = c.n_expert; p->L = c.n_attn_layers;
  p->I = c.n_input_functions; p->KI = std::max(p->I, 1); p->DT = D / 16;
  p->NL = std::max(c.n_mlp_num_layers, 1) + 1;   // MLP(nl) has max(nl,1)+1 Linears (model.py:9-14)
  p->in = c.input_dim; p->th = c.theta_dim; p->F = c.input_func_dim; p->out = c.out_dim;
  const int NL = p->NL;
  auto mlp = [&](int in, int outd) {
    for (int j = 0; j < NL; ++j) add_linear(p, j == NL - 1 ? outd : D, j == 0 ? in : D);
  };
  mlp(p->in + p->th, D);                                   // x
  mlp(p->in, p->E);                                        // gating
  for (int i = 0; i < p->I; ++i) mlp(p->F, D);             // input_func_mlps
  for (int l = 0; l < p->L; ++l) {
    for (int k = 0; k < 2 + 2 * p->KI; ++k) add_linear(p, D, D);   // cross q, fc_out, keys, values
    for (int k = 0; k < 4; ++k) add_linear(p, D, D);               // self q, fc_out, key, value
    for (int e = 0; e < 2 * p->E; ++e) mlp(D, D);                  // ffn1, ffn2 experts
  }
  mlp(D, p->out);                                          // out
  if ((int)p->lin_o.size() != p->n_lin()) {
    delete p;
    return fail(GNOT_E_INVALID, "internal: linear count mismatch");
  }
  p->W.assign(p->n_lin(), nullptr);
  p->b.assign(p->n_lin(), nullptr);
  *out = p;
  return GNOT_OK;
}

extern "C" void gnot_plan_destroy(gnot_plan* plan) { delete plan; }

extern "C" int gnot_plan_num_linears(const gnot_plan* p) { return p ? p->n_lin() : 0; }

extern "C" int gnot_plan_linear_dims(const gnot_plan* p, int32_t* dims) {
  if (!p || !dims) return fail(GNOT_E_INVALID, "null argument");
  for (int i = 0; i < p->n_lin(); ++i) {
    dims[2 * i] = p->lin_o[i];
    dims[2 * i + 1] = p->lin_i[i];
  }
  return GNOT_OK;
}

extern "C" int gnot_plan_bind_params(gnot_plan* p, const float* const* weights, const float* const* biases) {
  if (!p || !weights || !biases) return fail(GNOT_E_INVALID, "null argument");
  for (int i = 0; i < p->n_lin(); ++i) {
    if (!weights[i] || !biases[i]) return fail(GNOT_E_INVALID, "null parameter pointer");
    p->W[i] = weights[i];
    p->b[i] = biases[i];
  }
  p->params_bound = true;
  p->packed = false;
  return GNOT_OK;
}

// ====================================================================== layout
namespace {

struct Carver {
  size_t top = 0;
  gnot_plan* p;
  void add(const std::string& name, size_t nfloats, long ld) {
    Buf b;
    b.off = top;
    b.ld = ld;
    top += ((nfloats * sizeof(float) + 255) / 256) * 256;
    p->bufs[name] = b;
    p->buf_order.push_back(name);
  }
  size_t raw(size_t bytes) {
    const size_t o = top;
    top += ((bytes + 255) / 256) * 256;
    return o;
  }
};

void make_chunks(const std::vector<long>& off, std::vector<int4>& ch, std::vector<int>& choff) {
  ch.clear();
  choff.assign(1, 0);
  const int B = (int)off.size() - 1;
  for (int b = 0; b < B; ++b) {
    for (long s = off[b]; s < off[b + 1]; s += kSeg) {
      const int len = (int)std::min<long>(kSeg, off[b + 1] - s);
      ch.push_back(make_int4(b, (int)s, len, 0));
    }
    choff.push_back((int)ch.size());
  }
}

}  // namespace

// build the packed-weight images and pack jobs (offsets relative to the packed arena)
static void plan_images(gnot_plan* p) {
  const int DT = p->DT, NL = p->NL;
  p->pack_jobs.clear();
  p->pack_dst_off4.clear();
  p->pack_bias_off.clear();
  p->fwd_img.assign(p->n_lin(), Img());
  p->T_img.assign(p->n_lin(), Img());
  p->fwd_bias.assign(p->n_lin(), 0);
  p->packed4 = 0;
  p->pbias = 0;
  auto new_img = [&](int OT, int KT) {
    Img im;
    im.off4 = p->packed4;
    im.OT = OT;
    im.KT = KT;
    p->packed4 += (size_t)OT * KT * 64;
    return im;
  };
  auto new_bias = [&](int n) {
    const size_t o = p->pbias;
    p->pbias += (size_t)((n + 63) / 64) * 64;
    return o;
  };
  // job: linear li into image im at tile offsets (o0, t0); transposed flag; bias destination
  auto job = [&](int li, const Img& im, int o0, int t0, int OTp, int KTp, int tr, long bias_off) {
    PackJob J{};
    J.out = p->lin_o[li];
    J.in = p->lin_i[li];
    J.transposed = tr;
    J.o0 = o0; J.t0 = t0; J.ktot = im.KT;
    J.OTp = OTp; J.KTp = KTp;
    p->pack_jobs.push_back(J);
    p->pack_dst_off4.push_back(im.off4);
    p->pack_bias_off.push_back(bias_off < 0 ? (size_t)-1 : (size_t)bias_off);
    // remember which linear: encode in W/b later
    p->pack_jobs.back().W = reinterpret_cast<const float*>((intptr_t)li);
  };
  auto chain_imgs = [&](int first, int KT0, int OTL) {
    for (int j = 0; j < NL; ++j) {
      const int li = first + j;
      const int KTp = (j == 0) ? KT0 : DT;
      const int OTp = (j == NL - 1) ? OTL : DT;
      Img f = new_img(OTp, KTp);
      const size_t bo = new_bias(16 * OTp);
      job(li, f, 0, 0, OTp, KTp, 0, (long)bo);
      Img t = new_img(KTp, OTp);
      job(li, t, 0, 0, KTp, OTp, 1, -1);
      p->fwd_img[li] = f;
      p->T_img[li] = t;
      p->fwd_bias[li] = bo;
    }
  };
  auto kt_of = [&](int w) { return w <= 16 ? 1 : DT; };
  chain_imgs(p->lin_x(0), kt_of(p->in + p->th), DT);
  chain_imgs(p->lin_g(0), kt_of(p->in), kt_of(p->E));
  for (int i = 0; i < p->I; ++i) chain_imgs(p->lin_fn(i, 0), kt_of(p->F), DT);
  p->cross_img.assign(p->L, gnot_plan::AttnImgs());
  p->self_img.assign(p->L, gnot_plan::AttnImgs());
  auto attn_imgs = [&](gnot_plan::AttnImgs& A, int iq, int io, const std::vector<int>& ik,
                       const std::vector<int>& iv, bool selftype) {
    const int D = p->D;
    if (selftype) {
      A.qkv = new_img(3 * DT, DT);
      A.bqkv = new_bias(3 * D);
      job(iq, A.qkv, 0, 0, DT, DT, 0, (long)A.bqkv);
      job(ik[0], A.qkv, DT, 0, DT, DT, 0, (long)(A.bqkv + D));
      job(iv[0], A.qkv, 2 * DT, 0, DT, DT, 0, (long)(A.bqkv + 2 * D));
    } else {
      A.q = new_img(DT, DT);
      A.bq = new_bias(D);
      job(iq, A.q, 0, 0, DT, DT, 0, (long)A.bq);
      for (size_t i = 0; i < ik.size(); ++i) {
        Img kv = new_img(2 * DT, DT);
        const size_t bkv = new_bias(2 * D);
        job(ik[i], kv, 0, 0, DT, DT, 0, (long)bkv);
        job(iv[i], kv, DT, 0, DT, DT, 0, (long)(bkv + D));
        A.kv.push_back(kv);
        A.bkv.push_back(bkv);
      }
    }
    A.o = new_img(DT, DT);
    A.bo = new_bias(D);
    job(io, A.o, 0, 0, DT, DT, 0, (long)A.bo);
    std::vector<int> all = {iq, io};
    all.insert(all.end(), ik.begin(), ik.end());
    all.insert(all.end(), iv.begin(), iv.end());
    for (int li : all) {
      Img t = new_img(DT, DT);
      job(li, t, 0, 0, DT, DT, 1, -1);
      p->T_img[li] = t;
    }
  };
  for (int l = 0; l < p->L; ++l) {
    std::vector<int> ck, cv;
    for (int i = 0; i < p->KI; ++i) { ck.push_back(p->lin_ck(l, i)); cv.push_back(p->lin_cv(l, i)); }
    attn_imgs(p->cross_img[l], p->lin_cq(l), p->lin_co(l), ck, cv, p->I == 0);
    attn_imgs(p->self_img[l], p->lin_sq(l), p->lin_so(l), {p->lin_sk(l)}, {p->lin_sv(l)}, true);
    for (int e = 0; e < p->E; ++e) {
      chain_imgs(p->lin_f1(l, e, 0), DT, DT);
      chain_imgs(p->lin_f2(l, e, 0), DT, DT);
    }
  }
  chain_imgs(p->lin_out(0), DT, kt_of(p->out));
  p->pack_prefix.clear();
  int acc = 0;
  for (auto& J : p->pack_jobs) {
    p->pack_prefix.push_back(acc);
    acc += J.OTp * J.KTp;
  }
  p->pack_tiles = acc;
}

extern "C" int gnot_plan_set_batch(gnot_plan* p, int B, const int64_t* x_off, const int64_t* fn_off,
                                   int training) {
  if (!p || B <= 0 || !x_off) return fail(GNOT_E_INVALID, "bad batch arguments");
  if (p->I > 0 && !fn_off) return fail(GNOT_E_INVALID, "fn_off required when n_input_functions > 0");
  p->B = B;
  p->xoff.assign(x_off, x_off + B + 1);
  if (p->xoff[0] != 0) return fail(GNOT_E_INVALID, "x_off[0] must be 0");
  for (int b = 0; b < B; ++b)
    if (p->xoff[b + 1] < p->xoff[b]) return fail(GNOT_E_INVALID, "x_off must be non-decreasing");
  p->P = p->xoff[B];
  p->fnoff.assign(p->I, {});
  p->Q.assign(p->I, 0);
  for (int i = 0; i < p->I; ++i) {
    p->fnoff[i].assign(fn_off + i * (B + 1), fn_off + (i + 1) * (B + 1));
    if (p->fnoff[i][0] != 0) return fail(GNOT_E_INVALID, "fn_off[i][0] must be 0");
    for (int b = 0; b < B; ++b)
      if (p->fnoff[i][b + 1] < p->fnoff[i][b]) return fail(GNOT_E_INVALID, "fn_off must be non-decreasing");
    p->Q[i] = p->fnoff[i][B];
  }
  if (p->P <= 0) return fail(GNOT_E_INVALID, "empty batch (no query points)");
  if (p->P >= (1L << 31) / 4) return fail(GNOT_E_INVALID, "batch too large for 32-bit segment indices");
  p->training = training != 0;

  // ---------------- workspace carve
  plan_images(p);
  p->bufs.clear();
  p->buf_order.clear();
  Carver C{0, p};
  const long P = p->P, D = p->D, E = p->E, NL = p->NL, H = p->H;
  const long per_state = (long)p->H * (p->dh * p->dh + p->dh);
  const int I = p->I, KI = p->KI;
  long Qmax = 0;
  for (long q : p->Q) Qmax = std::max(Qmax, q);
  C.add("packed", p->packed4 * 4, 0);
  C.add("pbias", p->pbias, 0);
  // gradient arena
  p->grad_off.clear();
  long g = 0;
  for (int li = 0; li < p->n_lin(); ++li) {
    p->grad_off.push_back(g);
    g += (long)p->lin_o[li] * p->lin_i[li];
    p->grad_off.push_back(g);
    g += p->lin_o[li];
  }
  p->grad_floats = g;
  C.add("grads", g, 0);
  const bool tr = p->training;
  C.add("x", P * r4(p->in), r4(p->in));
  C.add("theta", (long)p->B * p->th, p->th);
  C.add("xin", P * r4(p->in + p->th), r4(p->in + p->th));
  for (int i = 0; i < I; ++i) C.add("fn" + std::to_string(i), p->Q[i] * r4(p->F), r4(p->F));
  const long ldsc = r4(E);
  C.add("scores", P * ldsc, ldsc);
  if (tr) {
    C.add("dscore", P * ldsc, ldsc);
    C.add("gate_save", NL * P * D, D);
    C.add("x_save", NL * P * D, D);
    C.add("out_save", NL * P * D, D);
  }
  C.add("query0", P * D, D);
  for (int i = 0; i < I; ++i) {
    if (tr) C.add("fn_save" + std::to_string(i), NL * p->Q[i] * D, D);
    C.add("fnenc" + std::to_string(i), p->Q[i] * D, D);
  }
  for (int l = 0; l < p->L; ++l) {
    const std::string s = "b" + std::to_string(l) + ".";
    if (I > 0) {
      C.add(s + "cq", P * D, D);
      for (int i = 0; i < I; ++i) C.add(s + "ckv" + std::to_string(i), p->Q[i] * 2 * D, 2 * D);
    } else {
      C.add(s + "cq", P * 3 * D, 3 * D);     // q | k | v of the cross module in self mode
    }
    for (int i = 0; i < KI; ++i) C.add(s + "cstate" + std::to_string(i), p->B * per_state, per_state);
    C.add(s + "cres", P * D, D);
    C.add(s + "a", P * D, D);
    if (tr) C.add(s + "m1save", E * NL * P * D, D);
    C.add(s + "query1", P * D, D);
    C.add(s + "sq", P * 3 * D, 3 * D);
    C.add(s + "sstate", p->B * per_state, per_state);
    C.add(s + "sres", P * D, D);
    C.add(s + "bb", P * D, D);
    if (tr) C.add(s + "m2save", E * NL * P * D, D);
    C.add(s + "query2", P * D, D);
  }
  C.add("stage", E * P * D, D);
  // attention segments
  make_chunks(p->xoff, p->qchunks, p->qchunk_off);
  p->fchunks.assign(I, {});
  p->fchunk_off.assign(I, {});
  size_t maxchunks = p->qchunks.size();
  for (int i = 0; i < I; ++i) {
    make_chunks(p->fnoff[i], p->fchunks[i], p->fchunk_off[i]);
    maxchunks = std::max(maxchunks, p->fchunks[i].size());
  }
  p->slab_state_floats = maxchunks * per_state;
  C.add("slab_state", p->slab_state_floats, 0);
  if (tr) {
    C.add("dout", P * r4(p->out), r4(p->out));
    C.add("dquery", P * D, D);
    C.add("dsum", P * D, D);
    C.add("dres", P * D, D);
    C.add("dqkv", P * 3 * D, 3 * D);
    for (int i = 0; i < KI; ++i) {
      C.add("du" + std::to_string(i), P * D, D);
      C.add("dden" + std::to_string(i), P * H, H);
      C.add("dstate" + std::to_string(i), p->B * per_state, per_state);
    }
    for (int i = 0; i < I; ++i) {
      C.add("dkv" + std::to_string(i), p->Q[i] * 2 * D, 2 * D);
      C.add("dfn" + std::to_string(i), p->Q[i] * D, D);
    }
    C.add("dz", E * NL * std::max(P, Qmax) * D, D);
  }

  // ---------------- device tables (host images; uploaded at bind)
  p->table_bytes = 0;
  p->ch_gate = {}; p->ch_x = {}; p->ch_out = {};
  p->ch_fn.assign(I, {});
  p->ch_m1.assign(p->L, {});
  p->ch_m2.assign(p->L, {});
  const int DT = p->DT;
  auto kt_of = [&](int w) { return w <= 16 ? 1 : DT; };
  auto chain = [&](ChainTable& T, std::vector<int> firsts, int in_dim, int out_dim) {
    T.nchains = (int)firsts.size();
    T.in_dim = in_dim;
    T.out_dim = out_dim;
    T.KT0 = kt_of(in_dim);
    T.OTL = kt_of(out_dim);
    T.host.clear();
    for (int f : firsts)
      for (int j = 0; j < NL; ++j) T.host.push_back(ChainLayer{nullptr, nullptr, nullptr});  // filled at bind
  };
  chain(p->ch_gate, {p->lin_g(0)}, p->in, E);
  chain(p->ch_x, {p->lin_x(0)}, p->in + p->th, (int)D);
  chain(p->ch_out, {p->lin_out(0)}, (int)D, p->out);
  for (int i = 0; i < I; ++i) chain(p->ch_fn[i], {p->lin_fn(i, 0)}, p->F, (int)D);
  for (int l = 0; l < p->L; ++l) {
    std::vector<int> f1, f2;
    for (int e = 0; e < E; ++e) { f1.push_back(p->lin_f1(l, e, 0)); f2.push_back(p->lin_f2(l, e, 0)); }
    chain(p->ch_m1[l], f1, (int)D, (int)D);
    chain(p->ch_m2[l], f2, (int)D, (int)D);
  }
  auto tbl = [&](size_t bytes) { p->table_bytes += ((bytes + 255) / 256) * 256; };
  tbl(p->pack_jobs.size() * sizeof(PackJob));
  tbl(p->pack_prefix.size() * sizeof(int));
  auto tbl_chain = [&](const ChainTable& T) { tbl(T.host.size() * sizeof(ChainLayer)); };
  tbl_chain(p->ch_gate); tbl_chain(p->ch_x); tbl_chain(p->ch_out);
  for (auto& T : p->ch_fn) tbl_chain(T);
  for (auto& T : p->ch_m1) tbl_chain(T);
  for (auto& T : p->ch_m2) tbl_chain(T);
  tbl(p->qchunks.size() * sizeof(int4));
  tbl(p->qchunk_off.size() * sizeof(int));
  for (int i = 0; i < I; ++i) { tbl(p->fchunks[i].size() * sizeof(int4)); tbl(p->fchunk_off[i].size() * sizeof(int)); }
  tbl((p->B + 1) * sizeof(long) * (1 + I));

  // wgrad groups (pointers resolved at bind; sizes known now)
  auto splits_of = [&](long rows) {
    return (int)std::max<long>(1, std::min<long>(kWgradMaxSplits, (rows + kWgradChunk - 1) / kWgradChunk));
  };
  auto wjob = [&](WgradGroup& G, int li, long rows) {
    WgradJob J{};
    J.out = p->lin_o[li];
    J.in = p->lin_i[li];
    J.P = (int)rows;
    J.tiles_o = (J.out + 31) / 32;
    J.tiles_i = (J.in + 31) / 32;
    J.splits = splits_of(rows);
    J.slab_off = (long)G.slab_floats;
    J.accumulate = 0;
    // stash the linear index in dW until bind
    J.dW = reinterpret_cast<float*>((intptr_t)li);
    G.slab_floats += (size_t)J.splits * (J.tiles_o * 32) * (J.tiles_i * 32 + 1);
    G.jobs.push_back(J);
  };
  auto finish_group = [&](WgradGroup& G) {
    G.wave_prefix.clear();
    G.red_prefix.clear();
    int w = 0, r = 0;
    for (auto& J : G.jobs) {
      G.wave_prefix.push_back(w);
      w += J.tiles_o * J.tiles_i * J.splits;
      G.red_prefix.push_back(r);
      r += (J.tiles_o * 32) * (J.tiles_i * 32 + 1);
    }
    G.total_waves = w;
    G.total_red = r;
    p->slab_wgrad_floats = std::max(p->slab_wgrad_floats, G.slab_floats);
    tbl(G.jobs.size() * sizeof(WgradJob));
    tbl(G.jobs.size() * sizeof(int) * 2);
  };
  p->slab_wgrad_floats = 0;
  if (tr) {
    p->wg_out = {}; p->wg_x = {}; p->wg_gate = {};
    for (int j = 0; j < NL; ++j) wjob(p->wg_out, p->lin_out(j), P);
    finish_group(p->wg_out);
    for (int j = 0; j < NL; ++j) wjob(p->wg_x, p->lin_x(j), P);
    finish_group(p->wg_x);
    for (int j = 0; j < NL; ++j) wjob(p->wg_gate, p->lin_g(j), P);
    finish_group(p->wg_gate);
    p->wg_fn.assign(I, {});
    for (int i = 0; i < I; ++i) {
      for (int j = 0; j < NL; ++j) wjob(p->wg_fn[i], p->lin_fn(i, j), p->Q[i]);
      finish_group(p->wg_fn[i]);
    }
    p->wg_m1.assign(p->L, {}); p->wg_m2.assign(p->L, {});
    p->wg_self.assign(p->L, {}); p->wg_cross.assign(p->L, {});
    for (int l = 0; l < p->L; ++l) {
      for (int e = 0; e < E; ++e)
        for (int j = 0; j < NL; ++j) {
          wjob(p->wg_m1[l], p->lin_f1(l, e, j), P);
          wjob(p->wg_m2[l], p->lin_f2(l, e, j), P);
        }
      finish_group(p->wg_m1[l]);
      finish_group(p->wg_m2[l]);
      for (int li : {p->lin_so(l), p->lin_sq(l), p->lin_sk(l), p->lin_sv(l)}) wjob(p->wg_self[l], li, P);
      finish_group(p->wg_self[l]);
      wjob(p->wg_cross[l], p->lin_co(l), P);
      wjob(p->wg_cross[l], p->lin_cq(l), P);
      for (int i = 0; i < KI; ++i) {
        const long rows = I > 0 ? p->Q[i] : P;
        wjob(p->wg_cross[l], p->lin_ck(l, i), rows);
        wjob(p->wg_cross[l], p->lin_cv(l, i), rows);
      }
      finish_group(p->wg_cross[l]);
    }
    C.add("slab_wgrad", p->slab_wgrad_floats, 0);
  }
  const size_t table_off = C.raw(p->table_bytes);
  p->bufs["__tables"] = Buf{table_off, 0, nullptr};
  p->ws_need = C.top;
  p->batch_set = true;
  p->ws_bound = false;
  p->packed = false;
  p->fwd_done = false;
  return GNOT_OK;
}

extern "C" size_t gnot_plan_workspace_bytes(const gnot_plan* p) { return (p && p->batch_set) ? p->ws_need : 0; }

extern "C" int gnot_plan_grad_offsets(const gnot_plan* p, int64_t* grad_off) {
  if (!p || !grad_off || !p->batch_set) return fail(GNOT_E_STATE, "set_batch first");
  for (size_t i = 0; i < p->grad_off.size(); ++i) grad_off[i] = p->grad_off[i];
  return GNOT_OK;
}

// ====================================================================== bind
extern "C" int gnot_plan_bind_workspace(gnot_plan* p, void* workspace, size_t bytes) {
  if (!p || !p->batch_set) return fail(GNOT_E_STATE, "set_batch first");
  if (!p->params_bound) return fail(GNOT_E_STATE, "bind_params first");
  if (!workspace || bytes < p->ws_need) return fail(GNOT_E_WORKSPACE, "workspace missing or too small");
  if (reinterpret_cast<uintptr_t>(workspace) & 255) return fail(GNOT_E_WORKSPACE, "workspace must be 256-byte aligned");
  p->ws = static_cast<char*>(workspace);
  for (auto& kv : p->bufs) kv.second.p = reinterpret_cast<float*>(p->ws + kv.second.off);
  const int D = p->D, NL = p->NL;

  // ---- tables in the workspace tail
  char* tp = p->ws + p->bufs["__tables"].off;
  std::vector<char> host(p->table_bytes, 0);
  size_t cur = 0;
  auto put = [&](const void* src, size_t bytes) -> void* {
    void* dev = tp + cur;
    if (bytes) std::memcpy(host.data() + cur, src, bytes);
    cur += ((bytes + 255) / 256) * 256;
    return dev;
  };
  // pack jobs with real pointers
  float4* packed = reinterpret_cast<float4*>(p->P_("packed"));
  float* pbias = p->P_("pbias");
  std::vector<PackJob> jobs = p->pack_jobs;
  for (size_t k = 0; k < jobs.size(); ++k) {
    const int li = (int)reinterpret_cast<intptr_t>(jobs[k].W);
    jobs[k].W = p->W[li];
    jobs[k].b = p->b[li];
    jobs[k].dst = packed + p->pack_dst_off4[k];
    jobs[k].bias_dst = (p->pack_bias_off[k] == (size_t)-1) ? nullptr : pbias + p->pack_bias_off[k];
  }
  p->d_pack_jobs = static_cast<PackJob*>(put(jobs.data(), jobs.size() * sizeof(PackJob)));
  p->d_pack_prefix = static_cast<int*>(put(p->pack_prefix.data(), p->pack_prefix.size() * sizeof(int)));
  // resolve images
  auto rimg = [&](Img& im) { im.p = packed + im.off4; };
  for (auto& im : p->fwd_img) rimg(im);
  for (auto& im : p->T_img) rimg(im);
  for (auto* v : {&p->cross_img, &p->self_img})
    for (auto& A : *v) {
      rimg(A.qkv); rimg(A.q); rimg(A.o);
      for (auto& k : A.kv) rimg(k);
    }
  // chain tables
  auto fill_chain = [&](ChainTable& T, const std::vector<int>& firsts) {
    T.host.clear();
    for (int f : firsts)
      for (int j = 0; j < NL; ++j) {
        const int li = f + j;
        T.host.push_back(ChainLayer{p->fwd_img[li].p, p->T_img[li].p, pbias + p->fwd_bias[li]});
      }
    T.dev = static_cast<ChainLayer*>(put(T.host.data(), T.host.size() * sizeof(ChainLayer)));
  };
  fill_chain(p->ch_gate, {p->lin_g(0)});
  fill_chain(p->ch_x, {p->lin_x(0)});
  fill_chain(p->ch_out, {p->lin_out(0)});
  for (int i = 0; i < p->I; ++i) fill_chain(p->ch_fn[i], {p->lin_fn(i, 0)});
  for (int l = 0; l < p->L; ++l) {
    std::vector<int> f1, f2;
    for (int e = 0; e < p->E; ++e) { f1.push_back(p->lin_f1(l, e, 0)); f2.push_back(p->lin_f2(l, e, 0)); }
    fill_chain(p->ch_m1[l], f1);
    fill_chain(p->ch_m2[l], f2);
  }
  p->d_qchunks = static_cast<int4*>(put(p->qchunks.data(), p->qchunks.size() * sizeof(int4)));
  p->d_qchunk_off = static_cast<int*>(put(p->qchunk_off.data(), p->qchunk_off.size() * sizeof(int)));
  p->d_fchunks.assign(p->I, nullptr);
  p->d_fchunk_off.assign(p->I, nullptr);
  for (int i = 0; i < p->I; ++i) {
    p->d_fchunks[i] = static_cast<int4*>(put(p->fchunks[i].data(), p->fchunks[i].size() * sizeof(int4)));
    p->d_fchunk_off[i] = static_cast<int*>(put(p->fchunk_off[i].data(), p->fchunk_off[i].size() * sizeof(int)));
  }
  {
    std::vector<long> offs(p->xoff);
    for (int i = 0; i < p->I; ++i) offs.insert(offs.end(), p->fnoff[i].begin(), p->fnoff[i].end());
    long* d = static_cast<long*>(put(offs.data(), offs.size() * sizeof(long)));
    p->d_xoff = d;
    p->d_fnoff.assign(p->I, nullptr);
    for (int i = 0; i < p->I; ++i) p->d_fnoff[i] = d + (p->B + 1) * (i + 1);
  }
  // wgrad groups
  if (p->training) {
    float* grads = p->P_("grads");
    auto fill_group = [&](WgradGroup& G) {
      std::vector<WgradJob> J = G.jobs;
      for (auto& j : J) {
        const int li = (int)reinterpret_cast<intptr_t>(j.dW);
        j.dW = grads + p->grad_off[2 * li];
        j.db = grads + p->grad_off[2 * li + 1];
      }
      G.jobs = J;   // dz/x pointers are set below per group
    };
    // dz / x sources
    auto set_chain_src = [&](WgradGroup& G, int chain_idx, int j, const float* dz, long lddz,
                             const float* x, long ldx, int gelu_x) {
      WgradJob& w = G.jobs[chain_idx * NL + j];
      w.dz = dz; w.lddz = lddz; w.x = x; w.ldx = ldx; w.x_gelu = gelu_x;
    };
    const long P = p->P;
    float* dz = p->P_("dz");
    auto chain_group = [&](WgradGroup& G, int nchains, long rows, const float* x0, long ldx0,
                           const float* save) {
      fill_group(G);
      for (int e = 0; e < nchains; ++e)
        for (int j = 0; j < NL; ++j) {
          const float* dzp = dz + ((long)e * NL + j) * rows * D;
          if (j == 0) set_chain_src(G, e, j, dzp, D, x0, ldx0, 0);
          else set_chain_src(G, e, j, dzp, D, save + ((long)e * NL + (j - 1)) * rows * D, D, 1);
        }
    };
    chain_group(p->wg_out, 1, P, p->P_(p->final_query()), D, p->P_("out_save"));
    chain_group(p->wg_x, 1, P, p->P_("xin"), p->bufs["xin"].ld, p->P_("x_save"));
    chain_group(p->wg_gate, 1, P, p->P_("x"), p->bufs["x"].ld, p->P_("gate_save"));
    for (int i = 0; i < p->I; ++i) {
      const std::string s = std::to_string(i);
      chain_group(p->wg_fn[i], 1, p->Q[i], p->P_("fn" + s), p->bufs["fn" + s].ld, p->P_("fn_save" + s));
    }
    for (int l = 0; l < p->L; ++l) {
      const std::string s = "b" + std::to_string(l) + ".";
      chain_group(p->wg_m1[l], p->E, P, p->P_(s + "a"), D, p->P_(s + "m1save"));
      chain_group(p->wg_m2[l], p->E, P, p->P_(s + "bb"), D, p->P_(s + "m2save"));
      // self attention: Wo, Wq, Wk, Wv
      fill_group(p->wg_self[l]);
      {
        auto& J = p->wg_self[l].jobs;
        float* dqkv = p->P_("dqkv");
        J[0].dz = p->P_("dsum"); J[0].lddz = D; J[0].x = p->P_(s + "sres"); J[0].ldx = D;
        for (int k = 0; k < 3; ++k) {
          J[1 + k].dz = dqkv + k * D; J[1 + k].lddz = 3 * D;
          J[1 + k].x = p->P_(s + "query1"); J[1 + k].ldx = D;
        }
      }
      fill_group(p->wg_cross[l]);
      {
        auto& J = p->wg_cross[l].jobs;
        const float* qin = p->P_(p->block_query(l));
        J[0].dz = p->P_("dsum"); J[0].lddz = D; J[0].x = p->P_(s + "cres"); J[0].ldx = D;
        if (p->I > 0) {
          J[1].dz = p->P_("dqkv"); J[1].lddz = D; J[1].x = qin; J[1].ldx = D;   // dQ in dqkv[:, :D], ld D
          for (int i = 0; i < p->I; ++i) {
            const std::string si = std::to_string(i);
            float* dkv = p->P_("dkv" + si);
            J[2 + 2 * i].dz = dkv; J[2 + 2 * i].lddz = 2 * D;
            J[2 + 2 * i].x = p->P_("fnenc" + si); J[2 + 2 * i].ldx = D;
            J[3 + 2 * i].dz = dkv + D; J[3 + 2 * i].lddz = 2 * D;
            J[3 + 2 * i].x = p->P_("fnenc" + si); J[3 + 2 * i].ldx = D;
          }
        } else {
          float* dqkv = p->P_("dqkv");
          J[1].dz = dqkv; J[1].lddz = 3 * D; J[1].x = qin; J[1].ldx = D;
          J[2].dz = dqkv + D; J[2].lddz = 3 * D; J[2].x = qin; J[2].ldx = D;
          J[3].dz = dqkv + 2 * D; J[3].lddz = 3 * D; J[3].x = qin; J[3].ldx = D;
        }
      }
    }
    auto upload_group = [&](WgradGroup& G) {
      G.d_jobs = static_cast<WgradJob*>(put(G.jobs.data(), G.jobs.size() * sizeof(WgradJob)));
      std::vector<int> pre(G.wave_prefix);
      pre.insert(pre.end(), G.red_prefix.begin(), G.red_prefix.end());
      int* d = static_cast<int*>(put(pre.data(), pre.size() * sizeof(int)));
      G.d_wave_prefix = d;
      G.d_red_prefix = d + G.jobs.size();
    };
    upload_group(p->wg_out); upload_group(p->wg_x); upload_group(p->wg_gate);
    for (auto& G : p->wg_fn) upload_group(G);
    for (int l = 0; l < p->L; ++l) {
      upload_group(p->wg_m1[l]); upload_group(p->wg_m2[l]);
      upload_group(p->wg_self[l]); upload_group(p->wg_cross[l]);
    }
  }
  if (cur > p->table_bytes) return fail(GNOT_E_INVALID, "internal: table overflow");
  GNOT_CK(hipMemcpy(tp, host.data(), cur, hipMemcpyHostToDevice));
  p->ws_bound = true;
  p->packed = false;
  p->fwd_done = false;
  return GNOT_OK;
}

extern "C" int gnot_pack_weights(gnot_plan* p, void* stream) {
  if (!p || !p->ws_bound) return fail(GNOT_E_STATE, "bind_workspace first");
  GNOT_CK(launch_pack(p->d_pack_jobs, p->d_pack_prefix, (int)p->pack_jobs.size(), p->pack_tiles,
                      static_cast<hipStream_t>(stream)));
  p->packed = true;
  return GNOT_OK;
}

// ====================================================================== forward / backward
namespace {

struct Ctx {
  gnot_plan* p;
  hipStream_t s;
};

int run_linear(Ctx& c, const float* X, long ldx, int K, const Img& A, const float* bias, float* Y, long ldy,
               int NO, long P, int epi, int nsoft) {
  LinearArgs a{};
  a.X = X; a.ldx = ldx; a.nsum = 1; a.sum_stride = 0; a.K = K;
  a.Wp = A.p; a.bias = bias; a.Y = Y; a.ldy = ldy; a.NO = NO; a.P = (int)P;
  a.epi = epi; a.nsoft = nsoft; a.dh = c.p->dh;
  GNOT_CK(launch_linear(a, c.p->D, c.s));
  return GNOT_OK;
}

ChainArgs chain_args(gnot_plan* p, const ChainTable& T, long P) {
  ChainArgs a{};
  a.D = p->D; a.KT0 = T.KT0; a.OTL = T.OTL; a.nlin = p->NL;
  a.in_dim = T.in_dim; a.out_dim = T.out_dim; a.P = (int)P; a.nchains = T.nchains; a.layers = T.dev;
  return a;
}

int run_state(Ctx& c, const float* A, long lda, const float* Bv, long ldb, const float* w, long ldw,
              const int4* chunks, int nchunks, const int* choff, float* state) {
  gnot_plan* p = c.p;
  AttnStateArgs a{};
  a.A = A; a.lda = lda; a.Bv = Bv; a.ldb = ldb; a.w = w; a.ldw = ldw;
  a.H = p->H; a.dh = p->dh; a.chunks = chunks; a.nchunks = nchunks;
  a.slab = p->P_("slab_state"); a.sample_chunk_off = choff; a.B = p->B; a.state = state;
  GNOT_CK(launch_attn_state(a, c.s));
  return GNOT_OK;
}

int run_wgrad(Ctx& c, const WgradGroup& G) {
  if (G.jobs.empty()) return GNOT_OK;
  GNOT_CK(launch_wgrad(G.d_jobs, G.d_wave_prefix, (int)G.jobs.size(), G.total_waves, G.d_red_prefix,
                       G.total_red, c.p->P_("slab_wgrad"), c.s));
  return GNOT_OK;
}

#define GNOT_RUN(expr)              \
  do {                              \
    const int rc_ = (expr);         \
    if (rc_ != GNOT_OK) return rc_; \
  } while (0)

// one LinearAttention call (model.py:53-107). q_in: the query rows [P, D].
int attn_forward(Ctx& c, int l, bool cross, const float* q_in, float* res_out, float* out) {
  gnot_plan* p = c.p;
  const long P = p->P;
  const int D = p->D;
  const std::string s = "b" + std::to_string(l) + ".";
  const gnot_plan::AttnImgs& A = cross ? p->cross_img[l] : p->self_img[l];
  float* pbias = p->P_("pbias");
  const int nq = (int)p->qchunks.size();
  if (cross && p->I > 0) {
    float* q = p->P_(s + "cq");
    GNOT_RUN(run_linear(c, q_in, D, D, A.q, pbias + A.bq, q, D, D, P, EPI_STORE, D));
    AttnApplyArgs ap{};
    for (int i = 0; i < p->I; ++i) {
      const std::string si = std::to_string(i);
      float* kv = p->P_(s + "ckv" + si);
      GNOT_RUN(run_linear(c, p->P_("fnenc" + si), D, D, A.kv[i], pbias + A.bkv[i], kv, 2 * D, 2 * D, p->Q[i],
                          EPI_STORE, D));
      float* st = p->P_(s + "cstate" + si);
      GNOT_RUN(run_state(c, kv, 2 * D, kv + D, 2 * D, nullptr, 0, p->d_fchunks[i], (int)p->fchunks[i].size(),
                         p->d_fchunk_off[i], st));
      ap.state[i] = st;
    }
    ap.q = q; ap.ldq = D; ap.nsrc = p->I; ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff;
    ap.H = p->H; ap.dh = p->dh; ap.res = res_out;
    GNOT_CK(launch_attn_apply_fwd(ap, c.s));
  } else {
    float* qkv = p->P_(cross ? s + "cq" : s + "sq");
    GNOT_RUN(run_linear(c, q_in, D, D, A.qkv, pbias + A.bqkv, qkv, 3 * D, 3 * D, P, EPI_STORE, 2 * D));
    float* st = p->P_(cross ? s + "cstate0" : s + "sstate");
    GNOT_RUN(run_state(c, qkv + D, 3 * D, qkv + 2 * D, 3 * D, nullptr, 0, p->d_qchunks, nq, p->d_qchunk_off, st));
    AttnApplyArgs ap{};
    ap.q = qkv; ap.ldq = 3 * D; ap.nsrc = 1; ap.state[0] = st; ap.chunks = p->d_qchunks; ap.nchunks = nq;
    ap.off = p->d_xoff; ap.H = p->H; ap.dh = p->dh; ap.res = res_out;
    GNOT_CK(launch_attn_apply_fwd(ap, c.s));
  }
  GNOT_RUN(run_linear(c, res_out, D, D, A.o, pbias + A.bo, out, D, D, P, EPI_STORE, 0));
  return GNOT_OK;
}

// backward of one LinearAttention call. dout: grad of its output [P, D] (materialised in "dsum").
// Accumulates d(q_in) into dquery.
int attn_backward(Ctx& c, int l, bool cross, const float* q_in) {
  gnot_plan* p = c.p;
  const long P = p->P;
  const int D = p->D;
  const std::string s = "b" + std::to_string(l) + ".";
  const int lo = cross ? p->lin_co(l) : p->lin_so(l);
  const int lq = cross ? p->lin_cq(l) : p->lin_sq(l);
  float* dsum = p->P_("dsum");
  float* dres = p->P_("dres");
  float* dquery = p->P_("dquery");
  float* dqkv = p->P_("dqkv");
  const int nq = (int)p->qchunks.size();
  // fc_out backward-data: dres = dout W_o
  GNOT_RUN(run_linear(c, dsum, D, D, p->T_img[lo], nullptr, dres, D, D, P, EPI_STORE, 0));
  if (cross && p->I > 0) {
    const float* q = p->P_(s + "cq");
    AttnApplyArgs ap{};
    ap.q = q; ap.ldq = D; ap.nsrc = p->I; ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff;
    ap.H = p->H; ap.dh = p->dh; ap.dres = dres; ap.dq_pre = dqkv; ap.lddq = D; ap.lddu = D;
    for (int i = 0; i < p->I; ++i) {
      const std::string si = std::to_string(i);
      ap.state[i] = p->P_(s + "cstate" + si);
      ap.du[i] = p->P_("du" + si);
      ap.dden[i] = p->P_("dden" + si);
    }
    GNOT_CK(launch_attn_apply_bwd(ap, c.s));
    for (int i = 0; i < p->I; ++i) {
      const std::string si = std::to_string(i);
      float* dst = p->P_("dstate" + si);
      GNOT_RUN(run_state(c, q, D, p->P_("du" + si), D, p->P_("dden" + si), p->H, p->d_qchunks, nq,
                         p->d_qchunk_off, dst));
      const float* kv = p->P_(s + "ckv" + si);
      float* dkv = p->P_("dkv" + si);
      AttnKVBwdArgs kb{};
      kb.k = kv; kb.v = kv + D; kb.ldkv = 2 * D; kb.dstate = dst; kb.chunks = p->d_fchunks[i];
      kb.nchunks = (int)p->fchunks[i].size(); kb.H = p->H; kb.dh = p->dh; kb.dk = dkv; kb.dv = dkv + D;
      kb.lddkv = 2 * D;
      GNOT_CK(launch_attn_kv_bwd(kb, c.s));
      float* dfn = p->P_("dfn" + si);
      GNOT_RUN(run_linear(c, dkv, 2 * D, D, p->T_img[p->lin_ck(l, i)], nullptr, dfn, D, D, p->Q[i], EPI_ACCUM, 0));
      GNOT_RUN(run_linear(c, dkv + D, 2 * D, D, p->T_img[p->lin_cv(l, i)], nullptr, dfn, D, D, p->Q[i], EPI_ACCUM, 0));
    }
    GNOT_RUN(run_linear(c, dqkv, D, D, p->T_img[lq], nullptr, dquery, D, D, P, EPI_ACCUM, 0));
  } else {
    const float* qkv = p->P_(cross ? s + "cq" : s + "sq");
    const int lk = cross ? p->lin_ck(l, 0) : p->lin_sk(l);
    const int lv = cross ? p->lin_cv(l, 0) : p->lin_sv(l);
    AttnApplyArgs ap{};
    ap.q = qkv; ap.ldq = 3 * D; ap.nsrc = 1; ap.state[0] = p->P_(cross ? s + "cstate0" : s + "sstate");
    ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff; ap.H = p->H; ap.dh = p->dh;
    ap.dres = dres; ap.dq_pre = dqkv; ap.lddq = 3 * D; ap.du[0] = p->P_("du0"); ap.lddu = D;
    ap.dden[0] = p->P_("dden0");
    GNOT_CK(launch_attn_apply_bwd(ap, c.s));
    float* dst = p->P_("dstate0");
    GNOT_RUN(run_state(c, qkv, 3 * D, p->P_("du0"), D, p->P_("dden0"), p->H, p->d_qchunks, nq,
                       p->d_qchunk_off, dst));
    AttnKVBwdArgs kb{};
    kb.k = qkv + D; kb.v = qkv + 2 * D; kb.ldkv = 3 * D; kb.dstate = dst; kb.chunks = p->d_qchunks;
    kb.nchunks = nq; kb.H = p->H; kb.dh = p->dh; kb.dk = dqkv + D; kb.dv = dqkv + 2 * D; kb.lddkv = 3 * D;
    GNOT_CK(launch_attn_kv_bwd(kb, c.s));
    GNOT_RUN(run_linear(c, dqkv, 3 * D, D, p->T_img[lq], nullptr, dquery, D, D, P, EPI_ACCUM, 0));
    GNOT_RUN(run_linear(c, dqkv + D, 3 * D, D, p->T_img[lk], nullptr, dquery, D, D, P, EPI_ACCUM, 0));
    GNOT_RUN(run_linear(c, dqkv + 2 * D, 3 * D, D, p->T_img[lv], nullptr, dquery, D, D, P, EPI_ACCUM, 0));
  }
  (void)q_in;
  return GNOT_OK;
}

}  // namespace

extern "C" int gnot_forward(gnot_plan* p, const float* x, const float* theta, const float* const* fns,
                            float* out, void* stream) {
  if (!p || !p->ws_bound) return fail(GNOT_E_STATE, "bind_workspace first");
  if (!p->packed) return fail(GNOT_E_STATE, "gnot_pack_weights must run before gnot_forward");
  if (!x || !theta || !out || (p->I > 0 && !fns)) return fail(GNOT_E_INVALID, "null input");
  Ctx c{p, static_cast<hipStream_t>(stream)};
  const long P = p->P;
  const int D = p->D, E = p->E, NL = p->NL;
  const bool tr = p->training;
  // inputs into the workspace (row pitch rounded to 16 B)
  GNOT_CK(hipMemcpy2DAsync(p->P_("x"), p->bufs["x"].ld * 4, x, p->in * 4, p->in * 4, P, hipMemcpyDeviceToDevice, c.s));
  GNOT_CK(hipMemcpyAsync(p->P_("theta"), theta, (size_t)p->B * p->th * 4, hipMemcpyDeviceToDevice, c.s));
  for (int i = 0; i < p->I; ++i) {
    const std::string n = "fn" + std::to_string(i);
    if (p->Q[i] > 0)
      GNOT_CK(hipMemcpy2DAsync(p->P_(n), p->bufs[n].ld * 4, fns[i], p->F * 4, p->F * 4, p->Q[i],
                               hipMemcpyDeviceToDevice, c.s));
  }
  GNOT_CK(launch_concat_theta(p->P_("x"), p->bufs["x"].ld, p->in, p->P_("theta"), p->th, p->d_xoff, p->B,
                              p->P_("xin"), p->bufs["xin"].ld, (int)P, c.s));
  // gating (model.py:155-156)
  {
    ChainArgs a = chain_args(p, p->ch_gate, P);
    a.X = p->P_("x"); a.ldx = p->bufs["x"].ld;
    a.Y = p->P_("scores"); a.ldy = p->bufs["scores"].ld; a.mode = CH_SOFTMAX;
    if (tr) { a.save = p->P_("gate_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(a, c.s));
  }
  // query encoder (model.py:158-161)
  {
    ChainArgs a = chain_args(p, p->ch_x, P);
    a.X = p->P_("xin"); a.ldx = p->bufs["xin"].ld;
    a.Y = p->P_("query0"); a.ldy = D; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("x_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(a, c.s));
  }
  // input-function encoders (model.py:164-166)
  for (int i = 0; i < p->I; ++i) {
    const std::string si = std::to_string(i);
    ChainArgs a = chain_args(p, p->ch_fn[i], p->Q[i]);
    a.X = p->P_("fn" + si); a.ldx = p->bufs["fn" + si].ld;
    a.Y = p->P_("fnenc" + si); a.ldy = D; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("fn_save" + si); a.save_layer_stride = p->Q[i] * D; a.save_chain_stride = NL * p->Q[i] * D; }
    GNOT_CK(launch_chain_fwd(a, c.s));
  }
  // blocks (model.py:126-139)
  for (int l = 0; l < p->L; ++l) {
    const std::string s = "b" + std::to_string(l) + ".";
    const float* qin = p->P_(p->block_query(l));
    GNOT_RUN(attn_forward(c, l, true, qin, p->P_(s + "cres"), p->P_(s + "a")));
    {
      ChainArgs a = chain_args(p, p->ch_m1[l], P);
      a.X = p->P_(s + "a"); a.ldx = D; a.Y = p->P_("stage"); a.ldy = D; a.y_chain_stride = P * D;
      a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.mode = CH_MOE;
      if (tr) { a.save = p->P_(s + "m1save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
      GNOT_CK(launch_chain_fwd(a, c.s));
      GNOT_CK(launch_moe_combine(qin, p->P_("stage"), P * D, E, p->P_(s + "query1"), P * D, c.s));
    }
    GNOT_RUN(attn_forward(c, l, false, p->P_(s + "query1"), p->P_(s + "sres"), p->P_(s + "bb")));
    {
      ChainArgs a = chain_args(p, p->ch_m2[l], P);
      a.X = p->P_(s + "bb"); a.ldx = D; a.Y = p->P_("stage"); a.ldy = D; a.y_chain_stride = P * D;
      a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.mode = CH_MOE;
      if (tr) { a.save = p->P_(s + "m2save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
      GNOT_CK(launch_chain_fwd(a, c.s));
      GNOT_CK(launch_moe_combine(p->P_(s + "query1"), p->P_("stage"), P * D, E, p->P_(s + "query2"), P * D, c.s));
    }
  }
  // decoder (model.py:171)
  {
    ChainArgs a = chain_args(p, p->ch_out, P);
    a.X = p->P_(p->final_query()); a.ldx = D; a.Y = out; a.ldy = p->out; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("out_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(a, c.s));
  }
  p->fwd_done = true;
  return GNOT_OK;
}

extern "C" int gnot_backward(gnot_plan* p, const float* dout, void* stream) {
  if (!p || !p->ws_bound || !p->fwd_done) return fail(GNOT_E_STATE, "gnot_forward must run before gnot_backward");
  if (!p->training) return fail(GNOT_E_STATE, "plan was set up with training = 0");
  if (!dout) return fail(GNOT_E_INVALID, "null dout");
  Ctx c{p, static_cast<hipStream_t>(stream)};
  const long P = p->P;
  const int D = p->D, E = p->E, NL = p->NL;
  float* dz = p->P_("dz");
  float* dquery = p->P_("dquery");
  float* stage = p->P_("stage");
  GNOT_CK(hipMemcpy2DAsync(p->P_("dout"), p->bufs["dout"].ld * 4, dout, p->out * 4, p->out * 4, P,
                           hipMemcpyDeviceToDevice, c.s));
  GNOT_CK(hipMemsetAsync(p->P_("dscore"), 0, P * p->bufs["dscore"].ld * 4, c.s));
  for (int i = 0; i < p->I; ++i)
    GNOT_CK(hipMemsetAsync(p->P_("dfn" + std::to_string(i)), 0, p->Q[i] * D * 4, c.s));
  // decoder
  {
    ChainArgs a = chain_args(p, p->ch_out, P);
    a.dY = p->P_("dout"); a.lddy = p->bufs["dout"].ld; a.mode = CH_STORE;
    a.save = p->P_("out_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
    a.dX = dquery; a.lddx = D; a.dx_chain_stride = 0;
    GNOT_CK(launch_chain_bwd(a, c.s));
    GNOT_RUN(run_wgrad(c, p->wg_out));
  }
  for (int l = p->L - 1; l >= 0; --l) {
    const std::string s = "b" + std::to_string(l) + ".";
    // ffn2 experts: query2 = query1 + sum_e s_e ffn2_e(bb)
    {
      ChainArgs a = chain_args(p, p->ch_m2[l], P);
      a.dY = dquery; a.lddy = D; a.mode = CH_MOE;
      a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.dscore = p->P_("dscore");
      a.save = p->P_(s + "m2save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
      a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
      a.dX = stage; a.lddx = D; a.dx_chain_stride = P * D;
      GNOT_CK(launch_chain_bwd(a, c.s));
      GNOT_RUN(run_wgrad(c, p->wg_m2[l]));
      GNOT_CK(launch_moe_combine(nullptr, stage, P * D, E, p->P_("dsum"), P * D, c.s));
    }
    GNOT_RUN(attn_backward(c, l, false, p->P_(s + "query1")));
    GNOT_RUN(run_wgrad(c, p->wg_self[l]));
    // ffn1 experts: query1 = query0 + sum_e s_e ffn1_e(a)
    {
      ChainArgs a = chain_args(p, p->ch_m1[l], P);
      a.dY = dquery; a.lddy = D; a.mode = CH_MOE;
      a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.dscore = p->P_("dscore");
      a.save = p->P_(s + "m1save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
      a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
      a.dX = stage; a.lddx = D; a.dx_chain_stride = P * D;
      GNOT_CK(launch_chain_bwd(a, c.s));
      GNOT_RUN(run_wgrad(c, p->wg_m1[l]));
      GNOT_CK(launch_moe_combine(nullptr, stage, P * D, E, p->P_("dsum"), P * D, c.s));
    }
    GNOT_RUN(attn_backward(c, l, true, p->P_(p->block_query(l))));
    GNOT_RUN(run_wgrad(c, p->wg_cross[l]));
  }
  // input-function encoders (their inputs need no gradient)
  for (int i = 0; i < p->I; ++i) {
    const std::string si = std::to_string(i);
    ChainArgs a = chain_args(p, p->ch_fn[i], p->Q[i]);
    a.dY = p->P_("dfn" + si); a.lddy = D; a.mode = CH_STORE;
    a.save = p->P_("fn_save" + si); a.save_layer_stride = p->Q[i] * D; a.save_chain_stride = NL * p->Q[i] * D;
    a.dz = dz; a.dz_layer_stride = p->Q[i] * D; a.dz_chain_stride = NL * p->Q[i] * D;
    GNOT_CK(launch_chain_bwd(a, c.s));
    GNOT_RUN(run_wgrad(c, p->wg_fn[i]));
  }
  // query encoder
  {
    ChainArgs a = chain_args(p, p->ch_x, P);
    a.dY = dquery; a.lddy = D; a.mode = CH_STORE;
    a.save = p->P_("x_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
    GNOT_CK(launch_chain_bwd(a, c.s));
    GNOT_RUN(run_wgrad(c, p->wg_x));
  }
  // gating: d scores accumulated over every MoE above -> softmax backward -> chain
  {
    ChainArgs a = chain_args(p, p->ch_gate, P);
    a.mode = CH_SOFTMAX; a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld;
    a.dscore = p->P_("dscore");
    a.save = p->P_("gate_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
    GNOT_CK(launch_chain_bwd(a, c.s));
    GNOT_RUN(run_wgrad(c, p->wg_gate));
  }
  (void)E;
  return GNOT_OK;
}

extern "C" int gnot_debug_buffer(const gnot_plan* p, const char* name, float** ptr, int64_t* ld) {
  if (!p || !name || !ptr || !p->ws_bound) return fail(GNOT_E_STATE, "bind_workspace first");
  auto it = p->bufs.find(name);
  if (it == p->bufs.end()) return fail(GNOT_E_INVALID, std::string("unknown buffer ") + name);
  *ptr = it->second.p;
  if (ld) *ld = it->second.ld;
  return GNOT_OK;
}

extern "C" const char* gnot_last_error(void) { return g_err.c_str(); }
extern "C" const char* gnot_version(void) { return "gnot-mi355x 0.1 (gfx950, fp32 MFMA)"; }
