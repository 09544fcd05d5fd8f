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
#include <cstdlib>
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

constexpr int kSeg = 64;             // points per attention segment (one wave of the apply kernels)
constexpr int kPTile = 128;          // output tile edge of the point-reduction GEMM (wgrad.hip)
constexpr int kTargetWGs = 512;      // aim for ~2 workgroups per CU per point-reduction launch
constexpr int kMinSplitPoints = 128; // never split below this many points

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
  std::vector<int> wg_prefix, red_prefix;
  int total_wgs = 0, total_red = 0;
  size_t slab_floats = 0;
  bool x6 = false;                   // plain weight-gradient jobs: the bf16x6 MFMA kernel
  bool wide = false;                 // ... on the 256 x 256-tile kernel (d = 256: one workgroup per job split)
  int tw = 256;                      // wide geometry's output edge: 256, or 128 (d <= 128, jobs within 128 x 128)
  bool b16 = false;                  // bf16-storage jobs (bf16 mode soft-MoE): pgemm_b16_kernel, wide geometry
  std::vector<int> lins;             // weight-gradient groups: the canonical Linears whose (dW, db) they write
  int state_pts = 0, state_nw = 0;
  bool state_mfma = false;   // state groups: points per workgroup, per-point weights (0 or H)
  // balanced wide groups: per-workgroup point ranges {job, slot, begin, end} (launch_wgrad segs) and the
  // first range of every workgroup (+ the end)
  std::vector<int4> segs;
  std::vector<int> seg_start;
  WgradJob* d_jobs = nullptr;        // device copies (workspace tables)
  int* d_wg_prefix = nullptr;
  int* d_red_prefix = nullptr;
  int4* d_segs = nullptr;
  int* d_seg_start = nullptr;
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
  // Dr: the model's hidden width (n_embed); D: the width the kernels run, Dr rounded up to whole
  // 16-wide tiles when Dr is not one the kernels take (gnot_plan_create).  Every activation row keeps D
  // columns whose pad columns Dr .. D-1 stay exact zeros (zero weight rows / columns and biases in the
  // packed images, pad columns of the feature softmax zeroed); parameters and gradients have Dr.
  int Dr = 0;
  bool padded() const { return Dr != D; }
  // padded heads (a head width Dr / H that is not a multiple of 4, d <= 192): the attention runs heads of
  // dh = the next multiple of 4 (q / k / v projections place head h's rows at h * dh, the feature softmax
  // masks the pad features, pack.hip PackJob::hr / hp), while the scramble rows (model.py:81-83) keep the
  // real head width dhr = Dr / H.  dhr == dh otherwise
  int dhr = 0;
  bool head_padded() const { return dhr != dh; }
  int hd() const { return H * dh; }                 // attention feature columns (<= D)
  // the projections' feature-softmax pad columns: features past the H heads of dh are written as 0
  int attn_dreal() const { return hd() < D ? hd() : 0; }
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
  // attention states as point-reduction GEMM jobs (one job per sample)
  std::vector<std::vector<WgradGroup>> st_c, dst_c;   // [l][source i]
  // cross attention with input functions: the input-function side of EVERY block is batched
  WgradGroup st_fn;                                    // forward states of all (block, fn, sample)
  WgradGroup wg_fnkv;                                  // weight grads of all key/value projections
  std::vector<LinearArgs> fwd_kv_jobs;                 // key/value projections of all (block, fn)
  std::vector<AttnKVBwdArgs> kvbwd_jobs;               // dK/dV of all (block, fn)
  std::vector<std::vector<LinearArgs>> dfn_jobs;       // d(fn encoding): launches of <= kMaxSeg segments
  LinearArgs* d_fwd_kv_jobs = nullptr;
  AttnKVBwdArgs* d_kvbwd_jobs = nullptr;
  std::vector<LinearArgs*> d_dfn_jobs;
  std::vector<WgradGroup> st_s, dst_s;                 // [l]
  size_t table_bytes = 0;
  size_t slab_wgrad_floats = 0, slab_state_floats = 0;

  // weight-gradient groups run on the caller's stream after the chain backward that produced their dZ,
  // or forked onto the side stream; every buffer a forked group reads is double-buffered and guarded
  // by the event of its last side-stream reader.  Measured, one box each, interleaved x2
  // (profiles/r04_wgrad_overlap_ab.txt): configs[2] (262,144 points) 235.3 / 236.2 ms per step serial
  // against 236.8 / 236.7 forked -- the chains and GEMMs fill every CU, so overlapping them buys
  // nothing; configs[1] (10,000 points, d = 128) 4.12 / 4.12 serial against 3.64 / 3.72 forked and
  // configs[0] (16,384 points) 9.62 / 9.65 against 9.56 / 9.55 -- small launches leave CUs idle that
  // the concurrent GEMMs fill.  So plans below kWgradSerialPoints fork, larger ones run serially; env
  // GNOT_WGRAD_OVERLAP = 0 / 1 (read when the plan is created) forces either form (bitwise equal).
  static constexpr long kWgradSerialPoints = 65536;
  hipStream_t side = nullptr;
  hipStream_t side2 = nullptr;          // input-function branch, concurrent with the query branch
  int wgrad_overlap_env = -1;
  bool serial_wgrad() const { return wgrad_overlap_env >= 0 ? wgrad_overlap_env == 0 : P >= kWgradSerialPoints; }
  std::vector<hipEvent_t> evs;
  size_t ev_next = 0;
  // pinned staging ring for the table uploads of gnot_plan_bind_workspace_async: slot k is rewritten
  // only after the copy that last read it has executed (stage_ev[k])
  static constexpr int kStageSlots = 4;
  void* stage[kStageSlots] = {};
  size_t stage_cap[kStageSlots] = {};
  hipEvent_t stage_ev[kStageSlots] = {};
  bool stage_used[kStageSlots] = {};
  int stage_next = 0;
  std::map<const float*, hipEvent_t> readers;
  // forked weight-gradient groups whose side-stream launch waits until the caller's stream has enqueued
  // its next kernel (run_wgrad_side / flush_deferred)
  struct DeferredWgrad {
    const WgradGroup* G;
    std::vector<const float*> reads;
    hipEvent_t fork;
  };
  std::vector<DeferredWgrad> deferred;
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
  bool bwd_done = false;      // a gnot_backward ran after the last gnot_forward (gnot_input_grads needs it)
  bool ig_reduced = false;    // sharded: the input-function gradients of that backward are rank sums already

  // point sharding (gnot_plan_set_shard): sample b's points are split over `world` ranks
  int world = 1, rank = 0;
  gnot_comm comm{};
  // gradient all-reduce overlapped with the backward (gnot_plan_set_grad_comm): each weight-gradient
  // group's (dW, db) ranges are summed over the ranks on `comm_stream` as soon as the group is written
  gnot_comm grad_comm{};
  bool grad_comm_on = false;
  hipStream_t comm_stream = nullptr;
  std::vector<long> nglob;                 // [B] global points per sample (sharded batches)
  bool sharded = false;                    // world > 1 for the current batch
  // MoE activation recompute (gnot_plan_set_moe_recompute): training keeps only each MoE call's
  // input; the backward re-runs that call's expert forward into ONE shared save buffer ("mrsave")
  // just before its chain backward -- E*NL*P*D floats once instead of per MoE call
  bool moe_recompute = false;
  // input gradients (gnot_plan_set_input_grads): the x / gating / input-function encoders' first Linears
  // also run their backward-data into dxin / dxg / dfnin<i>
  bool input_grads = false;
  // operand pieces of the d = 256 bf16-MFMA kernels (chain2, linear2, wide weight gradients):
  // 3 = bf16x6 (fp32-exact, default), 1 = bf16 arithmetic mode (gnot_plan_set_precision)
  int np = 3;
  // bf16 mode stores the soft-MoE chains' saves and dZ as bf16 (ChainArgs::b16s): one [P, 256] bf16 layer
  // is P * D / 2 four-byte units, a chain's 2 * NL save slots take what NL fp32 layers did
  bool b16s() const { return np == 1 && D == 256; }
  // operand pieces of the kernels this plan runs: the bf16 mode covers every width up to 256 (chain.hip /
  // linear.hip / the 128-tile weight gradients at d <= 192 as well); above 256 (chainw.hip) the fp32 path
  int npk() const { return D <= 256 ? np : 3; }
  // linear.hip's image kind of the attention projections (LinearArgs::img): d <= 192 one-piece (bf16 mode) or
  // x6 (kLinearX6), else fp32 fragment images (also d > 256)
  int lin_img() const { return D > 192 ? 0 : npk() == 1 ? 1 : kLinearX6 ? 3 : 0; }
  std::string msave(int l, bool m1) const {
    return moe_recompute ? std::string("mrsave") : "b" + std::to_string(l) + (m1 ? ".m1save" : ".m2save");
  }
  std::vector<CopySeg> xsend, xrecv;       // scramble all-to-all: hm -> send buffer, recv buffer -> tokens
  std::vector<int> xsend_prefix, xrecv_prefix;   // prefix sums in copy units (xunit floats) for the copy kernel
  int xunit = 4;                                  // 4 (float4 runs), 1 with padded heads (runs of dhr floats)
  std::vector<int64_t> xsend_counts, xrecv_counts;
  CopySeg* d_xsend = nullptr;
  CopySeg* d_xrecv = nullptr;
  int* d_xsend_prefix = nullptr;
  int* d_xrecv_prefix = nullptr;

  // live kernel timing (bench roofline): hipEvents around every launch of one kernel class
  std::string prof_kind;
  std::vector<hipEvent_t> prof_events;   // pool, pairs
  size_t prof_used = 0;
  double prof_flops = 0.0;
  long prof_launches = 0;

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
  // double-buffer slots, fixed by the (static) backward order
  std::string dz_buf(int chain_call) const { return "dz" + std::to_string(chain_call & 1); }
  int k_out() const { return 0; }
  int k_m2(int l) const { return 1 + 2 * (L - 1 - l); }
  int k_m1(int l) const { return 2 + 2 * (L - 1 - l); }
  int k_fn(int i) const { return 1 + 2 * L + i; }
  int k_x() const { return 1 + 2 * L + I; }
  int k_gate() const { return 2 + 2 * L + I; }
  std::string dsum_buf(bool m1) const { return m1 ? "dsum1" : "dsum0"; }
  // input-function encoder chains run on side2 with their own dZ buffer; the others alternate dz0/dz1
  std::string dz_name(int kcall) const { return (kcall >= k_fn(0) && kcall < k_fn(0) + I) ? "dzf" : dz_buf(kcall); }
  std::string dqkv_buf(bool cross) const { return cross ? "dqkv1" : "dqkv0"; }
  std::string dkv_buf(int l, int i) const { return "dkv" + std::to_string(l) + "_" + std::to_string(i); }
  std::string dstate_fn(int l, int i) const { return "dstate" + std::to_string(l) + "_" + std::to_string(i); }
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
  const int Dr = c.n_attn_hidden_dim;
  if (c.n_head <= 0 || Dr <= 0 || Dr % c.n_head != 0)
    return fail(GNOT_E_INVALID, "n_embed should be divisible by head");   // model.py:41
  const int dhr = Dr / c.n_head;
  // the attention passes take head widths that are a multiple of 4 (4-aligned lane slices up to 64, 4-feature
  // quads over 16 lanes above, attn.hip; the fp32-MFMA forms at 16 / 32 / 64); any other runs on heads padded
  // to the next multiple of 4 (gnot_plan::head_padded): q / k / v rows at h * dh, H * dh internal columns
  const int dh = (dhr + 3) / 4 * 4;
  if (dh > 256)
    return fail(GNOT_E_INVALID, "head width d/n_head must be at most 256 on the MI355X kernels");
  // the internal width D (Dr real columns + exact-zero pad columns): chain.hip / linear.hip run any multiple of
  // 16 up to 192 (whole 16-wide MFMA tiles, activations in registers); chain2.hip / linear2.hip d = 256 with
  // unpadded heads of 16 / 32 / 64 / 128 / 256 (the projections' softmax head groups); everything else up to
  // 512 runs at the next multiple of 64 from 320 on chainw.hip (one Linear at a time on linear.hip, whose
  // whole-row tilings keep any head in one workgroup)
  const int need = std::max(Dr, c.n_head * dh);
  const bool l2_heads = dh == dhr && (dh == 16 || dh == 32 || dh == 64 || dh == 128 || dh == 256);
  // Above 512 the internal width is the next multiple of 128 up to 1024: the projections then contract in two
  // halves of 320 .. 512 (launch_linear's K-split, half images PackJob::kh)
  int D;
  if (need <= 192) D = (need + 15) / 16 * 16;
  else if (need <= 256 && l2_heads) D = 256;
  else if (need <= 512) D = std::max(320, (need + 63) / 64 * 64);
  else D = (need + 127) / 128 * 128;
  if (D > 1024)
    return fail(GNOT_E_INVALID, "hidden width must be at most 1024 on the MI355X kernels (n_head times the head "
                                "width rounded up to a multiple of 4, with padded heads)");
  if (D > 512 && 64 % dh != 0)
    return fail(GNOT_E_INVALID, "above an internal width of 512 the head width must divide 64 on the MI355X "
                                "kernels");
  if ((D != 256 && (linear_oc(D, 3 * D, 2 * D, dh) < 0 || linear_oc(D, D, D, dh) < 0)) || linear_oc(D, 2 * D, 1, dh) < 0)
    return fail(GNOT_E_INVALID, "no projection tiling keeps whole heads of this head width on the MI355X kernels");
  if (c.n_expert < 1 || c.n_attn_layers < 0 || c.n_input_functions < 0 || c.n_input_functions > 8)
    return fail(GNOT_E_INVALID, "bad n_expert / n_attn_layers / n_input_functions");
  if (c.input_dim + c.theta_dim > Dr || c.input_dim > Dr || c.input_func_dim > Dr || c.out_dim > Dr ||
      c.n_expert > Dr || c.input_dim < 1 || c.out_dim < 1)
    return fail(GNOT_E_INVALID, "input/output widths must be in [1, hidden width]");
  gnot_plan* p = new gnot_plan();
  p->c = c;
  p->D = D; p->Dr = Dr; p->H = c.n_head; p->dh = dh; p->dhr = dhr; p->E = c.n_expert; p->L = c.n_attn_layers;
  p->I = c.n_input_functions; p->KI = std::max(p->I, 1); p->DT = D / 16;
  p->NL = std::max(c.n_mlp_num_layers, 1) + 1;   // MLP(nl) has max(nl,1)+1 Linears (model.py:9-14)
  p->in = c.input_dim; p->th = c.theta_dim; p->F = c.input_func_dim; p->out = c.out_dim;
  const int NL = p->NL;
  // canonical Linears at the model's width Dr (= named_parameters() shapes)
  auto mlp = [&](int in, int outd) {
    for (int j = 0; j < NL; ++j) add_linear(p, j == NL - 1 ? outd : Dr, j == 0 ? in : Dr);
  };
  mlp(p->in + p->th, Dr);                                  // x
  mlp(p->in, p->E);                                        // gating
  for (int i = 0; i < p->I; ++i) mlp(p->F, Dr);            // input_func_mlps
  for (int l = 0; l < p->L; ++l) {
    for (int k = 0; k < 2 + 2 * p->KI; ++k) add_linear(p, Dr, Dr);   // cross q, fc_out, keys, values
    for (int k = 0; k < 4; ++k) add_linear(p, Dr, Dr);               // self q, fc_out, key, value
    for (int e = 0; e < 2 * p->E; ++e) mlp(Dr, Dr);                  // ffn1, ffn2 experts
  }
  mlp(Dr, p->out);                                         // out
  if ((int)p->lin_o.size() != p->n_lin()) {
    delete p;
    return fail(GNOT_E_INVALID, "internal: linear count mismatch");
  }
  p->W.assign(p->n_lin(), nullptr);
  p->b.assign(p->n_lin(), nullptr);
  if (const char* ov = std::getenv("GNOT_WGRAD_OVERLAP")) p->wgrad_overlap_env = ov[0] == '1' ? 1 : 0;
  *out = p;
  return GNOT_OK;
}

extern "C" void gnot_plan_destroy(gnot_plan* plan) {
  if (!plan) return;
  for (hipEvent_t e : plan->prof_events) (void)hipEventDestroy(e);
  for (hipEvent_t e : plan->evs) (void)hipEventDestroy(e);
  for (int k = 0; k < gnot_plan::kStageSlots; ++k) {
    if (plan->stage_ev[k]) {
      (void)hipEventSynchronize(plan->stage_ev[k]);
      (void)hipEventDestroy(plan->stage_ev[k]);
    }
    if (plan->stage[k]) (void)hipHostFree(plan->stage[k]);
  }
  if (plan->side) (void)hipStreamDestroy(plan->side);
  if (plan->comm_stream) (void)hipStreamDestroy(plan->comm_stream);
  if (plan->side2) (void)hipStreamDestroy(plan->side2);
  delete plan;
}

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
  // bf16x6 image (chain kernels): OT x ceil(KT/2) blocks of `np` pieces x 64 lanes x 16 B
  auto new_img_x6 = [&](int OT, int KT, int np = 3) {
    Img im;
    im.off4 = p->packed4;
    im.OT = OT;
    im.KT = KT;
    p->packed4 += (size_t)OT * ((KT + 1) / 2) * np * 64;
    return im;
  };
  auto new_bias = [&](int n) {
    const size_t o = p->pbias;
    p->pbias += (size_t)((n + 63) / 64) * 64;
    return o;
  };
  // job: linear li into image im at tile offsets (o0, t0); transposed flag; bias destination
  // heads: a q / k / v projection (padded heads: its rows placed in heads of dh, PackJob::hr / hp)
  auto job = [&](int li, const Img& im, int o0, int t0, int OTp, int KTp, int tr, long bias_off, int x6 = 0,
                 bool heads = false) {
    PackJob J{};
    J.x6 = x6;
    J.out = p->lin_o[li];
    J.in = p->lin_i[li];
    if (heads && p->head_padded()) {
      J.hr = p->dhr;
      J.hp = p->dh;
      J.out = p->hd();
    }
    J.transposed = tr;
    J.o0 = o0; J.t0 = t0; J.ktot = im.KT; J.otot = im.OT;
    // internal widths above 512: a full-width contraction packed as two half images (launch_linear's K-split)
    if (x6 == 0 && p->D > 512 && im.KT == p->DT) J.kh = p->DT / 2;
    J.OTp = OTp; J.KTp = KTp;
    p->pack_jobs.push_back(J);
    p->pack_dst_off4.push_back(im.off4);
    p->pack_bias_off.push_back(bias_off < 0 ? (size_t)-1 : (size_t)bias_off);
    // remember which linear: encode in W/b later
    p->pack_jobs.back().W = reinterpret_cast<const float*>((intptr_t)li);
  };
  // d = 256: chain2.hip, bf16x6 output-major images in both directions; else chain.hip, k-major x6
  // forward image + exact fp32 backward-data image (bf16 mode: k-major one-piece images both ways, and the
  // projections on output-major one-piece images, linear.hip)
  const bool c2 = p->D == 256;
  const int c2np = c2 ? p->np : 3;                 // pieces of the output-major images
  const int c2x6 = c2np == 1 ? 3 : 2;              // their pack mode
  // d > 256 (chainw.hip: each Linear on linear.hip): fp32 fragment images in both directions
  const bool cw = p->D > 256;
  const bool b1 = !c2 && !cw && p->npk() == 1;      // d <= 192 in the bf16 mode
  auto chain_imgs = [&](int first, int KT0, int OTL) {
    for (int j = 0; j < NL; ++j) {
      const int li = first + j;
      const int KTp = (j == 0) ? KT0 : DT;
      const int OTp = (j == NL - 1) ? OTL : DT;
      Img f = cw ? new_img(OTp, KTp) : new_img_x6(OTp, KTp, c2 ? c2np : b1 ? 1 : 3);
      const size_t bo = new_bias(16 * OTp);
      job(li, f, 0, 0, OTp, KTp, 0, (long)bo, cw ? 0 : c2 ? c2x6 : b1 ? 4 : 1);
      // backward-data image: d <= 192 k-major x6 or one-piece (bf16 mode), else fp32 tiles
      const bool tx6 = !c2 && !cw;
      Img t = c2 ? new_img_x6(KTp, OTp, c2np) : tx6 ? new_img_x6(KTp, OTp, b1 ? 1 : 3) : new_img(KTp, OTp);
      job(li, t, 0, 0, KTp, OTp, 1, -1, c2 ? c2x6 : tx6 ? (b1 ? 4 : 1) : 0);
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
  // attention projections: at d = 256 the q | q|k|v | fc_out images and the backward-data images that
  // linear2.hip uses are output-major bf16x6; the input-function K/V images and their backward-data
  // images stay fp32 for the batched linear.hip kernel
  auto attn_imgs = [&](gnot_plan::AttnImgs& A, int iq, int io, const std::vector<int>& ik,
                       const std::vector<int>& iv, bool selftype) {
    const int D = p->D;
    const bool lx6 = p->lin_img() == 3;   // fp32 mode at d <= 192 (kLinearX6): output-major x6
    const int x6 = c2 ? c2x6 : b1 ? 3 : lx6 ? 2 : 0;
    auto img = [&](int OT, int KT) {
      return c2 ? new_img_x6(OT, KT, c2np) : b1 ? new_img_x6(OT, KT, 1) : lx6 ? new_img_x6(OT, KT, 3) : new_img(OT, KT);
    };
    if (selftype) {
      A.qkv = img(3 * DT, DT);
      A.bqkv = new_bias(3 * D);
      job(iq, A.qkv, 0, 0, DT, DT, 0, (long)A.bqkv, x6, true);
      job(ik[0], A.qkv, DT, 0, DT, DT, 0, (long)(A.bqkv + D), x6, true);
      job(iv[0], A.qkv, 2 * DT, 0, DT, DT, 0, (long)(A.bqkv + 2 * D), x6, true);
    } else {
      A.q = img(DT, DT);
      A.bq = new_bias(D);
      job(iq, A.q, 0, 0, DT, DT, 0, (long)A.bq, x6, true);
      for (size_t i = 0; i < ik.size(); ++i) {
        Img kv = new_img(2 * DT, DT);
        const size_t bkv = new_bias(2 * D);
        job(ik[i], kv, 0, 0, DT, DT, 0, (long)bkv, 0, true);
        job(iv[i], kv, DT, 0, DT, DT, 0, (long)(bkv + D), 0, true);
        A.kv.push_back(kv);
        A.bkv.push_back(bkv);
      }
    }
    A.o = img(DT, DT);
    A.bo = new_bias(D);
    job(io, A.o, 0, 0, DT, DT, 0, (long)A.bo, x6);
    std::vector<int> mine = {iq, io};
    if (selftype) { mine.push_back(ik[0]); mine.push_back(iv[0]); }
    for (int li : mine) {
      Img t = img(DT, DT);
      job(li, t, 0, 0, DT, DT, 1, -1, x6, li != io);
      p->T_img[li] = t;
    }
    if (!selftype)                          // input-function keys/values: batched fp32 kernel
      for (size_t i = 0; i < ik.size(); ++i)
        for (int li : {ik[i], iv[i]}) {
          Img t = new_img(DT, DT);
          job(li, t, 0, 0, DT, DT, 1, -1, 0, true);
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
    acc += pack_tiles(J);
  }
  p->pack_tiles = acc;
}

// ====================================================================== point-reduction GEMM groups
// split-K target of the 128-wide kernel
constexpr long kWide128Wgs = 128;
// balanced point ranges for a wide group (finish_group) when a per-job split count would leave CUs idle and
// every job has a point range of its own (no zero-point jobs)
static bool balanced_wgrad(const WgradGroup& G) {
  if (G.jobs.size() < 2) return false;
  for (const auto& J : G.jobs)
    if (J.P <= 0) return false;
  return 256 % (long)G.jobs.size() != 0;
}
static void finish_group(gnot_plan* p, WgradGroup& G) {
  G.x6 = true;
  for (const auto& J : G.jobs)
    if (J.w != nullptr || J.state_dh > 0 || J.diag_only) G.x6 = false;
  // the x6 kernel holds ~240 registers per lane: one workgroup per CU leaves the other half of
  // every SIMD's register file to the concurrent main-stream kernels
  constexpr long x6_wgs = 256;
  // d = 256: every job's whole 256 x 256 gradient in one workgroup (8 waves, 96 KiB LDS: one per CU).
  // The split-K target is fixed (r02bh: 192-512 all within noise), so the split counts the parity
  // tests exercise are the ones every run uses
  // plans below kWgradSerialPoints fork their weight gradients beside the caller's stream (serial_wgrad): a
  // group holding every CU's register file (the 256 x 256 kernel: 8 waves of 256 registers per CU) leaves the
  // concurrent critical-path kernels no room, so such plans' groups take fewer workgroups.  Keyed on the plan
  // size, not on the fork itself, so a plan gives bitwise the same gradients forked or serial
  // (GNOT_WGRAD_OVERLAP, tests/test_gpu_recompute.py).  Measured (round 6, interleaved sweeps
  // `profiles/r06sw*`): configs[0] (d = 256) 128 workgroups in fp32 (9.54 -> 9.00 ms per step against 256),
  // 64 in the bf16 mode (5.88 -> 5.47); configs[1] (the 128 x 128 kernel) 192 in fp32 (3.28 -> 3.21), 128 in
  // the bf16 mode (the round-5 value)
  const bool small = p->P < gnot_plan::kWgradSerialPoints;
  const long wide_wgs = !small ? 256 : p->npk() == 1 ? 64 : 128;
  const long w128_wgs = small && p->npk() != 1 ? 192 : kWide128Wgs;
  G.wide = G.x6 && p->D == 256 && !G.jobs.empty();
  for (const auto& J : G.jobs)
    if (J.out > 256 || J.in > 256) G.wide = false;
  G.tw = 256;
  // d <= 128 (configs[1]): the wide kernel's design at a 128 x 128 output (4 waves, staging interleaved with
  // the MFMAs, raw rows by LDS-DMA) instead of the 128-tile kernel (round 5: configs[1] 3.44 -> 3.37 ms)
  if (G.x6 && !G.wide && p->D <= 128 && !G.jobs.empty()) {
    bool fits = true;
    for (const auto& J : G.jobs)
      if (J.out > 128 || J.in > 128) fits = false;
    if (fits) { G.wide = true; G.tw = 128; }
  }
  if (G.b16) G.wide = true;          // the bf16-storage kernel has the wide kernel's geometry
  const long target = G.wide ? (G.tw == 128 ? w128_wgs : wide_wgs) : G.x6 ? x6_wgs : kTargetWGs;
  long tiles = 0;
  for (auto& J : G.jobs) {
    J.tiles_o = (J.out + kPTile - 1) / kPTile;
    J.tiles_i = (J.in + kPTile - 1) / kPTile;
    tiles += G.wide ? 1 : J.diag_only ? J.tiles_o : J.tiles_o * J.tiles_i;
  }
  // floor, not ceil: never more than `target` workgroups, so no CU runs one more than planned
  const long want = std::max<long>(1, target / std::max<long>(tiles, 1));
  G.wg_prefix.clear();
  G.red_prefix.clear();
  G.segs.clear();
  G.seg_start.clear();
  G.slab_floats = 0;
  if (G.wide && G.tw == 256 && balanced_wgrad(G)) {
    // the 256 x 256 kernel holds one workgroup per CU: a per-job split count leaves target % jobs CUs idle
    // (the 40 soft-MoE jobs of configs[2]: 6 splits each = 240 of 256), so cut the group's concatenated
    // points into `target` equal ranges instead (a range crossing a job boundary runs as two segments)
    long T = 0, maxrow = 1;
    for (const auto& J : G.jobs) {
      T += J.P;
      maxrow = std::max<long>(maxrow, G.b16 ? 512L : 4L * std::max<long>(std::max<long>(J.lddz, J.ldx), 1));
    }
    long C = std::max<long>((T + target - 1) / target, kMinSplitPoints);
    C = (C + 31) / 32 * 32;                                 // whole stages (kWStage 16, kBStage 32 points)
    C = std::min<long>(C, ((1L << 31) - 1) / maxrow - 64);  // a range's rows stay below 2^31 bytes
    std::vector<long> jstart(G.jobs.size() + 1, 0);
    for (size_t j = 0; j < G.jobs.size(); ++j) jstart[j + 1] = jstart[j] + G.jobs[j].P;
    std::vector<int> nslots(G.jobs.size(), 0);
    size_t jj = 0;
    for (long w0 = 0; w0 < T; w0 += C) {
      const long w1 = std::min(T, w0 + C);
      G.seg_start.push_back((int)G.segs.size());
      while (jj < G.jobs.size() && jstart[jj + 1] <= w0) ++jj;
      for (size_t j = jj; j < G.jobs.size() && jstart[j] < w1; ++j) {
        const long b = std::max(w0, jstart[j]) - jstart[j], e = std::min(w1, jstart[j + 1]) - jstart[j];
        if (e > b) G.segs.push_back(int4{(int)j, nslots[j]++, (int)b, (int)e});
      }
    }
    G.seg_start.push_back((int)G.segs.size());
    int red = 0;
    for (size_t j = 0; j < G.jobs.size(); ++j) {
      auto& J = G.jobs[j];
      J.splits = std::max(1, nslots[j]);
      const int nt = J.tiles_o * J.tiles_i;
      J.slab_off = (long)G.slab_floats;
      G.slab_floats += (size_t)J.splits * nt * kPTile * (kPTile + 1);
      G.wg_prefix.push_back(0);
      G.red_prefix.push_back(red);
      red += nt * kPTile * (kPTile + 1);
    }
    G.total_wgs = (int)G.seg_start.size() - 1;
    G.total_red = red;
    size_t& slab = p->slab_wgrad_floats;
    slab = std::max(slab, G.slab_floats);
    return;
  }
  int wg = 0, red = 0;
  for (auto& J : G.jobs) {
    const long minpts = kMinSplitPoints;   // >= 4 LDS stages per workgroup: bounds the split-K slab traffic
    const long maxs = std::max<long>(1, (J.P + minpts - 1) / minpts);
    J.splits = (int)std::min<long>(std::min<long>(want, maxs), 256);
    // the wide / bf16-row kernels address one split through a buffer resource based at its first row
    // with 32-bit offsets: a split's rows (+ the stage loaded past its end) stay below 2^31 bytes
    const long row_bytes = G.b16 ? 512L : 4L * std::max<long>(std::max<long>(J.lddz, J.ldx), 1);
    const long max_pts = ((1L << 31) - 1) / row_bytes - 64;
    J.splits = (int)std::max<long>(J.splits, (J.P + max_pts - 1) / max_pts);
    const int nt = J.diag_only ? J.tiles_o : J.tiles_o * J.tiles_i;
    J.slab_off = (long)G.slab_floats;
    G.slab_floats += (size_t)J.splits * nt * kPTile * (kPTile + 1);
    G.wg_prefix.push_back(wg);
    wg += (G.wide ? 1 : nt) * J.splits;
    G.red_prefix.push_back(red);
    red += nt * kPTile * (kPTile + 1);
  }
  G.total_wgs = wg;
  G.total_red = red;
  size_t& slab = (!G.jobs.empty() && G.jobs[0].state_dh > 0) ? p->slab_state_floats : p->slab_wgrad_floats;
  slab = std::max(slab, G.slab_floats);
}

// attention-state group (state.hip): one job per sample, ceil(P / kStatePts) partial states each
static void finish_state_group(gnot_plan* p, WgradGroup& G) {
  if (!G.jobs.empty()) {
    const int d = G.jobs[0].out;
    const int dh = G.jobs[0].state_dh;
    long total = 0;
    for (const auto& J : G.jobs) total += J.P;
    G.state_mfma = state_mfma_ok(d, dh) && total >= state_mfma_min_points();
    G.state_pts = state_pts(G.state_mfma, d);
    G.state_nw = 0;
    for (const auto& J : G.jobs)
      if (J.w != nullptr) G.state_nw = d / J.state_dh;
  }
  G.wg_prefix.clear();
  G.red_prefix.clear();
  G.slab_floats = 0;
  int wg = 0, red = 0;
  for (auto& J : G.jobs) {
    const int per = J.out / J.state_dh * (J.state_dh * J.state_dh + J.state_dh);
    J.splits = std::max(1, (J.P + G.state_pts - 1) / G.state_pts);
    J.slab_off = (long)G.slab_floats;
    G.slab_floats += (size_t)J.splits * per;
    G.wg_prefix.push_back(wg);
    wg += J.splits;
    G.red_prefix.push_back(red);
    red += per;
  }
  G.total_wgs = wg;
  G.total_red = red;
  p->slab_state_floats = std::max(p->slab_state_floats, G.slab_floats);
}

template <typename F>
static void for_each_group(gnot_plan* p, F&& f) {
  if (p->training) {
    f(p->wg_out); f(p->wg_x); f(p->wg_gate);
    for (auto& G : p->wg_fn) f(G);
    for (int l = 0; l < p->L; ++l) { f(p->wg_m1[l]); f(p->wg_m2[l]); f(p->wg_self[l]); f(p->wg_cross[l]); }
    f(p->wg_fnkv);
  }
  f(p->st_fn);
  for (int l = 0; l < p->L; ++l) {
    for (auto& G : p->st_c[l]) f(G);
    f(p->st_s[l]);
    if (p->training) {
      for (auto& G : p->dst_c[l]) f(G);
      f(p->dst_s[l]);
    }
  }
}

// (Re)build every job list from the current buffer pointers (null before bind: sizing only).
static void build_groups(gnot_plan* p) {
  p->slab_wgrad_floats = 0;
  p->slab_state_floats = 0;
  const long P = p->P;
  const int D = p->D, NL = p->NL, E = p->E, I = p->I, KI = p->KI, dh = p->dh;
  const bool tr = p->training;
  const long per_state = (long)p->H * (dh * dh + dh);
  p->wg_out = {}; p->wg_x = {}; p->wg_gate = {};
  p->wg_fn.assign(I, {});
  p->wg_m1.assign(p->L, {}); p->wg_m2.assign(p->L, {});
  p->wg_self.assign(p->L, {}); p->wg_cross.assign(p->L, {});
  p->st_c.assign(p->L, std::vector<WgradGroup>(KI));
  p->dst_c.assign(p->L, std::vector<WgradGroup>(KI));
  p->st_s.assign(p->L, {}); p->dst_s.assign(p->L, {});

  auto lin_job = [&](WgradGroup& G, int li, const float* dz, long lddz, const float* x, long ldx, int gelu,
                     long rows) {
    float* grads = p->P_("grads");
    WgradJob J{};
    J.dz = dz; J.lddz = lddz; J.x = x; J.ldx = ldx; J.x_gelu = gelu;
    J.out = p->lin_o[li]; J.in = p->lin_i[li];
    J.dW = grads + p->grad_off[2 * li];
    J.db = grads + p->grad_off[2 * li + 1];
    J.P = (int)rows;
    G.jobs.push_back(J);
    G.lins.push_back(li);
  };
  // a q / k / v projection's gradients: dz in heads of dh; padded heads: one job per head (its dhr real
  // rows of the canonical dW / db)
  auto lin_job_heads = [&](WgradGroup& G, int li, const float* dz, long lddz, const float* x, long ldx, long rows) {
    if (!p->head_padded()) {
      lin_job(G, li, dz, lddz, x, ldx, 0, rows);
      return;
    }
    float* grads = p->P_("grads");
    const int in = p->lin_i[li];
    for (int h = 0; h < p->H; ++h) {
      WgradJob J{};
      J.dz = dz ? dz + (long)h * dh : nullptr; J.lddz = lddz; J.x = x; J.ldx = ldx; J.x_gelu = 0;
      J.out = p->dhr; J.in = in;
      J.dW = grads + p->grad_off[2 * li] + (long)h * p->dhr * in;
      J.db = grads + p->grad_off[2 * li + 1] + (long)h * p->dhr;
      J.P = (int)rows;
      G.jobs.push_back(J);
    }
    G.lins.push_back(li);
  };
  // chain c of a group: Linear j reads dZ_j from dz[(c*NL + j)*rows*D] and its input from the
  // chain input (j = 0) or gelu(saved pre-activation j-1)
  auto chain_group = [&](WgradGroup& G, int kcall, const std::vector<int>& firsts, long rows, const float* x0,
                         long ldx0, const float* save) {
    const float* dz = p->P_(p->dz_name(kcall));
    for (size_t c = 0; c < firsts.size(); ++c)
      for (int j = 0; j < NL; ++j) {
        const float* dzp = dz + ((long)c * NL + j) * rows * D;
        if (j == 0) lin_job(G, firsts[c] + j, dzp, D, x0, ldx0, 0, rows);
        else lin_job(G, firsts[c] + j, dzp, D, save + ((long)c * NL + j - 1) * rows * D, D, 1, rows);
      }
    finish_group(p, G);
  };
  // bf16-storage soft-MoE group (bf16 mode): dZ_j of chain c at dz + (c NL + j) lay, the input of Linear
  // j > 0 in save slot NL + j of chain c, Linear 0's (the shared MoE input) in chain 0's slot NL
  auto moe_group_b16 = [&](WgradGroup& G, int kcall, const std::vector<int>& firsts, const float* save) {
    const float* dz = p->P_(p->dz_name(kcall));
    const long lay = P * D / 2;
    for (size_t c = 0; c < firsts.size(); ++c)
      for (int j = 0; j < NL; ++j) {
        const float* x = j == 0 ? save + NL * lay : save + ((long)c * 2 * NL + NL + j) * lay;
        lin_job(G, firsts[c] + j, dz + ((long)c * NL + j) * lay, D, x, D, 0, P);
      }
    G.b16 = true;
    finish_group(p, G);
  };
  auto state_group = [&](WgradGroup& G, const float* A, long lda, const float* Bm, long ldb, const float* w,
                         long ldw, const std::vector<long>& off, float* state) {
    for (int b = 0; b < p->B; ++b) {
      WgradJob J{};
      J.dz = A + off[b] * lda; J.lddz = lda;
      J.x = Bm + off[b] * ldb; J.ldx = ldb;
      J.out = p->hd(); J.in = p->hd();            // H heads of dh (the internal head width)
      J.dW = state + b * per_state;
      J.db = J.dW;
      J.w = w ? w + off[b] * ldw : nullptr; J.ldw = ldw; J.wdh = dh;
      J.state_dh = dh; J.diag_only = 1;
      J.P = (int)(off[b + 1] - off[b]);
      G.jobs.push_back(J);
    }
    finish_state_group(p, G);
  };

  for (int l = 0; l < p->L; ++l) {
    const std::string s = "b" + std::to_string(l) + ".";
    // forward states
    if (I > 0) {
      // (all blocks' input-function states are one group: st_fn, below)
    } else {
      float* qkv = p->P_(s + "cq");
      state_group(p->st_c[l][0], qkv + D, 3 * D, qkv + 2 * D, 3 * D, nullptr, 0, p->xoff, p->P_(s + "cstate0"));
    }
    {
      float* qkv = p->P_(s + "sq");
      state_group(p->st_s[l], qkv + D, 3 * D, qkv + 2 * D, 3 * D, nullptr, 0, p->xoff, p->P_(s + "sstate"));
    }
    if (!tr) continue;
    // backward states dS = sum q^T du, dz = sum dden q
    for (int i = 0; i < KI; ++i) {
      const std::string si = std::to_string(i);
      const long ldq = I > 0 ? D : 3 * D;
      state_group(p->dst_c[l][i], p->P_(s + "cq"), ldq, p->P_("du" + si), D, p->P_("dden" + si), p->H, p->xoff,
                  p->P_(I > 0 ? p->dstate_fn(l, i) : std::string("dstate0")));
    }
    state_group(p->dst_s[l], p->P_(s + "sq"), 3 * D, p->P_("du0"), D, p->P_("dden0"), p->H, p->xoff,
                p->P_("dstate0"));
  }
  p->st_fn = {};
  if (I > 0) {
    // one job per (block, fn, sample): S = k^T v, z = sum k over that sample's input-function points
    for (int l = 0; l < p->L; ++l)
      for (int i = 0; i < I; ++i) {
        const std::string s = "b" + std::to_string(l) + ".", si = std::to_string(i);
        float* kv = p->P_(s + "ckv" + si);
        float* st = p->P_(s + "cstate" + si);
        for (int b = 0; b < p->B; ++b) {
          WgradJob J{};
          const long o = p->fnoff[i][b];
          J.dz = kv + o * 2 * D; J.lddz = 2 * D; J.x = kv + D + o * 2 * D; J.ldx = 2 * D;
          J.out = p->hd(); J.in = p->hd(); J.dW = st + b * per_state; J.db = J.dW; J.wdh = dh;
          J.state_dh = dh; J.diag_only = 1; J.P = (int)(p->fnoff[i][b + 1] - o);
          p->st_fn.jobs.push_back(J);
        }
      }
    finish_state_group(p, p->st_fn);
  }
  if (!tr) return;

  p->wg_fnkv = {};
  if (I > 0) {
    for (int l = 0; l < p->L; ++l)
      for (int i = 0; i < I; ++i) {
        float* dkv = p->P_(p->dkv_buf(l, i));
        const float* enc = p->P_("fnenc" + std::to_string(i));
        lin_job_heads(p->wg_fnkv, p->lin_ck(l, i), dkv, 2 * D, enc, D, p->Q[i]);
        lin_job_heads(p->wg_fnkv, p->lin_cv(l, i), dkv + D, 2 * D, enc, D, p->Q[i]);
      }
    finish_group(p, p->wg_fnkv);
  }

  chain_group(p->wg_out, p->k_out(), {p->lin_out(0)}, P, p->P_(p->final_query()), D, p->P_("out_save"));
  chain_group(p->wg_x, p->k_x(), {p->lin_x(0)}, P, p->P_("xin"), p->bufs.at("xin").ld, p->P_("x_save"));
  chain_group(p->wg_gate, p->k_gate(), {p->lin_g(0)}, P, p->P_("x"), p->bufs.at("x").ld, p->P_("gate_save"));
  for (int i = 0; i < I; ++i) {
    const std::string si = std::to_string(i);
    chain_group(p->wg_fn[i], p->k_fn(i), {p->lin_fn(i, 0)}, p->Q[i], p->P_("fn" + si), p->bufs.at("fn" + si).ld,
                p->P_("fn_save" + si));
  }
  for (int l = 0; l < p->L; ++l) {
    const std::string s = "b" + std::to_string(l) + ".";
    std::vector<int> f1, f2;
    for (int e = 0; e < E; ++e) { f1.push_back(p->lin_f1(l, e, 0)); f2.push_back(p->lin_f2(l, e, 0)); }
    if (p->b16s()) {
      moe_group_b16(p->wg_m1[l], p->k_m1(l), f1, p->P_(p->msave(l, true)));
      moe_group_b16(p->wg_m2[l], p->k_m2(l), f2, p->P_(p->msave(l, false)));
    } else {
      chain_group(p->wg_m1[l], p->k_m1(l), f1, P, p->P_(s + "a"), D, p->P_(p->msave(l, true)));
      chain_group(p->wg_m2[l], p->k_m2(l), f2, P, p->P_(s + "bb"), D, p->P_(p->msave(l, false)));
    }
    {
      float* dsum = p->P_(p->dsum_buf(false));
      float* dqkv = p->P_(p->dqkv_buf(false));
      WgradGroup& G = p->wg_self[l];
      const float* q1 = p->P_(s + "query1");
      lin_job(G, p->lin_so(l), dsum, D, p->P_(s + "sres"), p->Dr, 0, P);
      lin_job_heads(G, p->lin_sq(l), dqkv, 3 * D, q1, D, P);
      lin_job_heads(G, p->lin_sk(l), dqkv + D, 3 * D, q1, D, P);
      lin_job_heads(G, p->lin_sv(l), dqkv + 2 * D, 3 * D, q1, D, P);
      finish_group(p, G);
    }
    {
      float* dsum = p->P_(p->dsum_buf(true));
      float* dqkv = p->P_(p->dqkv_buf(true));
      WgradGroup& G = p->wg_cross[l];
      const float* qin = p->P_(p->block_query(l));
      lin_job(G, p->lin_co(l), dsum, D, p->P_(s + "cres"), p->Dr, 0, P);
      if (I > 0) {
        lin_job_heads(G, p->lin_cq(l), dqkv, D, qin, D, P);   // key/value grads: wg_fnkv
      } else {
        lin_job_heads(G, p->lin_cq(l), dqkv, 3 * D, qin, D, P);
        lin_job_heads(G, p->lin_ck(l, 0), dqkv + D, 3 * D, qin, D, P);
        lin_job_heads(G, p->lin_cv(l, 0), dqkv + 2 * D, 3 * D, qin, D, P);
      }
      finish_group(p, G);
    }
  }
}

// internal widths above 512: a batched projection job's segments as K-halves (launch_linear's K-split done on
// the host: the batched kernel reads its jobs from device memory and runs at D / 2)
static void ksplit_job(const gnot_plan* p, LinearArgs& a) {
  if (p->D <= 512) return;
  const int Kh = p->D / 2;
  const long half4 = (long)(a.NO / 16) * (Kh / 16) * 64;   // the second half image (64 float4 per tile)
  LinearArgs b = a;
  b.nseg = 2 * a.nseg;
  for (int k = 0; k < b.nseg; ++k) {
    b.X[k] = a.X[k / 2] + (k % 2) * Kh;
    b.Wp[k] = a.Wp[k / 2] + (k % 2) * half4;
  }
  b.K = Kh;
  b.dblk = p->D;
  a = b;
}

// Device job tables of the batched input-function side of cross attention (pointers are null
// before bind: sizing only).
static void build_attn_tables(gnot_plan* p) {
  const int D = p->D, I = p->I, L = p->L;
  p->fwd_kv_jobs.clear();
  p->kvbwd_jobs.clear();
  p->dfn_jobs.clear();
  if (I == 0 || L == 0) return;
  float* pbias = p->P_("pbias");
  for (int l = 0; l < L; ++l)
    for (int i = 0; i < I; ++i) {
      const std::string s = "b" + std::to_string(l) + ".", si = std::to_string(i);
      const gnot_plan::AttnImgs& A = p->cross_img[l];
      LinearArgs a{};
      a.nseg = 1; a.X[0] = p->P_("fnenc" + si); a.ldx = D; a.Wp[0] = A.kv[i].p; a.nsum = 1; a.K = D;
      a.bias = pbias + A.bkv[i]; a.Y = p->P_(s + "ckv" + si); a.ldy = 2 * D; a.NO = 2 * D; a.P = (int)p->Q[i];
      a.epi = EPI_STORE; a.nsoft = D; a.dh = p->dh; a.dreal = p->attn_dreal();
      a.dhr = p->head_padded() ? p->dhr : 0;
      ksplit_job(p, a);
      p->fwd_kv_jobs.push_back(a);
    }
  if (!p->training) return;
  for (int l = 0; l < L; ++l)
    for (int i = 0; i < I; ++i) {
      const std::string s = "b" + std::to_string(l) + ".";
      const float* kv = p->P_(s + "ckv" + std::to_string(i));
      float* dkv = p->P_(p->dkv_buf(l, i));
      AttnKVBwdArgs kb{};
      kb.k = kv; kb.v = kv + D; kb.ldkv = 2 * D; kb.dstate = p->P_(p->dstate_fn(l, i));
      kb.chunks = p->d_fchunks.empty() ? nullptr : p->d_fchunks[i];
      kb.nchunks = (int)p->fchunks[i].size(); kb.H = p->H; kb.dh = p->dh;
      kb.dk = dkv; kb.dv = dkv + D; kb.lddkv = 2 * D;
      p->kvbwd_jobs.push_back(kb);
    }
  // d(fn encoding i) = sum_l dK_{l,i} Wk_{l,i} + dV_{l,i} Wv_{l,i}: 2L K-segments, <= kMaxSeg per launch (half
  // as many above an internal width of 512, each then two K-halves)
  const int nseg = 2 * L;
  const int per = D > 512 ? kMaxSeg / 2 : kMaxSeg;
  for (int k0 = 0; k0 < nseg; k0 += per) {
    std::vector<LinearArgs> launch;
    for (int i = 0; i < I; ++i) {
      LinearArgs a{};
      a.nseg = std::min(per, nseg - k0);
      for (int sg = 0; sg < a.nseg; ++sg) {
        const int l = (k0 + sg) / 2, kv = (k0 + sg) % 2;
        a.X[sg] = p->P_(p->dkv_buf(l, i)) + kv * D;
        a.Wp[sg] = p->T_img[kv ? p->lin_cv(l, i) : p->lin_ck(l, i)].p;
      }
      a.ldx = 2 * D; a.nsum = 1; a.K = D; a.bias = nullptr; a.Y = p->P_("dfn" + std::to_string(i)); a.ldy = D;
      a.NO = D; a.P = (int)p->Q[i]; a.epi = k0 == 0 ? EPI_STORE : EPI_ACCUM; a.nsoft = 0; a.dh = p->dh;
      ksplit_job(p, a);
      launch.push_back(a);
    }
    p->dfn_jobs.push_back(launch);
  }
}

// ====================================================================== point sharding
static void shard_range(long n, int rank, int world, long& lo, long& hi) {
  lo = n * rank / world;
  hi = n * (rank + 1) / world;
}

// The scramble all-to-all of one rank (see gnot_hip.h).  Flat row r = h*N_b + n of sample b's
// head-major [H, N_b, dh] apply output belongs to output token r / H.  Rank s computes the rows of
// its points n in [lo_s, hi_s) (local head-major layout: loff_s*d + (h*cnt_s + n - lo_s)*dh); rank t
// owns the tokens [lo_t, hi_t), i.e. flat rows [lo_t*H, hi_t*H), stored in token order at
// loff_t*d + (r - lo_t*H)*dh.  For every (peer, sample, head) the intersection is ONE contiguous run
// on both sides; packets are ordered (peer, sample, head) on both sides.
static void build_exchange(int B, const std::vector<long>& nglob, int H, int dh, int me, int world,
                           std::vector<CopySeg>& send, std::vector<CopySeg>& recv, std::vector<int64_t>& send_counts,
                           std::vector<int64_t>& recv_counts) {
  const long d = (long)H * dh;
  std::vector<std::vector<long>> lo(world, std::vector<long>(B)), hi = lo, loff = lo;
  for (int r = 0; r < world; ++r) {
    long acc = 0;
    for (int b = 0; b < B; ++b) {
      shard_range(nglob[b], r, world, lo[r][b], hi[r][b]);
      loff[r][b] = acc;
      acc += hi[r][b] - lo[r][b];
    }
  }
  send.clear(); recv.clear();
  send_counts.assign(world, 0);
  recv_counts.assign(world, 0);
  long scur = 0, rcur = 0;
  auto run = [&](int s, int t, int b, int h, long& r0, long& r1) {
    const long N = nglob[b];
    r0 = std::max((long)h * N + lo[s][b], lo[t][b] * H);
    r1 = std::min((long)h * N + hi[s][b], hi[t][b] * H);
    return r0 < r1;
  };
  for (int t = 0; t < world; ++t)          // me = source
    for (int b = 0; b < B; ++b)
      for (int h = 0; h < H; ++h) {
        long r0, r1;
        if (!run(me, t, b, h, r0, r1)) continue;
        const long cnt = hi[me][b] - lo[me][b];
        const long len = (r1 - r0) * dh;
        send.push_back(CopySeg{loff[me][b] * d + (h * cnt + (r0 - (long)h * nglob[b] - lo[me][b])) * dh, scur, len});
        scur += len;
        send_counts[t] += len;
      }
  for (int s = 0; s < world; ++s)          // me = destination
    for (int b = 0; b < B; ++b)
      for (int h = 0; h < H; ++h) {
        long r0, r1;
        if (!run(s, me, b, h, r0, r1)) continue;
        const long len = (r1 - r0) * dh;
        recv.push_back(CopySeg{rcur, loff[me][b] * d + (r0 - lo[me][b] * H) * dh, len});
        rcur += len;
        recv_counts[s] += len;
      }
}

static std::vector<int> seg_prefix(const std::vector<CopySeg>& segs, int unit) {
  std::vector<int> pre;
  int acc = 0;
  for (const auto& sg : segs) {
    pre.push_back(acc);
    acc += (int)(sg.len / unit);
  }
  pre.push_back(acc);
  return pre;
}

extern "C" int gnot_shard_range(int64_t n, int rank, int world, int64_t* lo, int64_t* hi) {
  if (world < 1 || rank < 0 || rank >= world || n < 0 || !lo || !hi) return fail(GNOT_E_INVALID, "bad shard range");
  long l, h;
  shard_range(n, rank, world, l, h);
  *lo = l;
  *hi = h;
  return GNOT_OK;
}

extern "C" int gnot_shard_exchange(int B, const int64_t* n_global, int n_head, int head_dim, int rank, int world,
                                   int64_t* send_counts, int64_t* recv_counts, int64_t* segs, int64_t cap,
                                   int64_t* nseg) {
  if (B <= 0 || !n_global || n_head <= 0 || head_dim <= 0 || world < 1 || rank < 0 || rank >= world || !nseg)
    return fail(GNOT_E_INVALID, "bad shard exchange arguments");
  std::vector<long> ng(n_global, n_global + B);
  std::vector<CopySeg> snd, rcv;
  std::vector<int64_t> sc, rc;
  build_exchange(B, ng, n_head, head_dim, rank, world, snd, rcv, sc, rc);
  if (send_counts) std::copy(sc.begin(), sc.end(), send_counts);
  if (recv_counts) std::copy(rc.begin(), rc.end(), recv_counts);
  *nseg = (int64_t)(snd.size() + rcv.size());
  int64_t k = 0;
  for (int dir = 0; dir < 2; ++dir)
    for (const auto& sg : dir == 0 ? snd : rcv) {
      if (segs && k < cap) {
        segs[4 * k] = dir;
        segs[4 * k + 1] = dir == 0 ? sg.a : sg.b;    // local offset (hm for send, tokens for recv)
        segs[4 * k + 2] = dir == 0 ? sg.b : sg.a;    // buffer offset
        segs[4 * k + 3] = sg.len;
      }
      ++k;
    }
  return GNOT_OK;
}

extern "C" int gnot_plan_set_shard(gnot_plan* p, int rank, int world, int B, const int64_t* n_global,
                                   const gnot_comm* comm) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  if (world <= 1 || !comm) {
    p->world = 1; p->rank = 0; p->nglob.clear(); p->comm = gnot_comm{};
    return GNOT_OK;
  }
  if (rank < 0 || rank >= world || B <= 0 || !n_global || !comm->allreduce_sum || !comm->alltoallv)
    return fail(GNOT_E_INVALID, "bad shard arguments");
  p->world = world;
  p->rank = rank;
  p->comm = *comm;
  p->nglob.assign(n_global, n_global + B);
  return GNOT_OK;
}

extern "C" int gnot_plan_set_grad_comm(gnot_plan* p, const gnot_comm* comm) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  if (comm && !comm->allreduce_sum) return fail(GNOT_E_INVALID, "gnot_comm.allreduce_sum is required");
  p->grad_comm_on = comm != nullptr;
  p->grad_comm = comm ? *comm : gnot_comm{};
  return GNOT_OK;
}

extern "C" int gnot_plan_set_precision(gnot_plan* p, int bf16) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  const int np = bf16 ? 1 : 3;
  if (p->np != np) {
    p->np = np;
    p->batch_set = false;          // image sizes change: set_batch + bind again
    p->ws_bound = false;
    p->packed = false;
  }
  return GNOT_OK;
}

extern "C" int gnot_plan_set_moe_recompute(gnot_plan* p, int on) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  if (p->moe_recompute != (on != 0)) {
    p->moe_recompute = on != 0;
    p->batch_set = false;          // the workspace layout changes: set_batch + bind again
    p->ws_bound = false;
  }
  return GNOT_OK;
}

extern "C" int gnot_plan_set_input_grads(gnot_plan* p, int on) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  if (p->input_grads != (on != 0)) {
    p->input_grads = on != 0;
    p->batch_set = false;          // the workspace layout changes: set_batch + bind again
    p->ws_bound = false;
  }
  return GNOT_OK;
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
  // point / chunk indices are 32-bit in the kernels' job tables (the buffer resources of the streaming
  // kernels are based per workgroup or per split, so no activation array size bounds a plan)
  if (p->P >= (1L << 31) / 4) return fail(GNOT_E_INVALID, "batch too large for 32-bit segment indices");
  for (int i = 0; i < p->I; ++i)
    if (p->Q[i] >= (1L << 31) / 4) return fail(GNOT_E_INVALID, "input functions too large for 32-bit segment indices");
  p->training = training != 0;
  p->sharded = p->world > 1;
  if (p->sharded) {
    if ((int)p->nglob.size() != B) return fail(GNOT_E_INVALID, "gnot_plan_set_shard was declared for another B");
    for (int b = 0; b < B; ++b) {
      long lo, hi;
      shard_range(p->nglob[b], p->rank, p->world, lo, hi);
      if (p->xoff[b + 1] - p->xoff[b] != hi - lo)
        return fail(GNOT_E_INVALID, "x_off does not match this rank's shard of n_global (gnot_shard_range)");
    }
    build_exchange(B, p->nglob, p->H, p->dhr, p->rank, p->world, p->xsend, p->xrecv, p->xsend_counts,
                   p->xrecv_counts);
    // the runs are multiples of the real head width (offsets too): float4 copies unless it is not a multiple of 4
    p->xunit = p->dhr % 4 == 0 ? 4 : 1;
    p->xsend_prefix = seg_prefix(p->xsend, p->xunit);
    p->xrecv_prefix = seg_prefix(p->xrecv, p->xunit);
  } else {
    p->xsend.clear(); p->xrecv.clear(); p->xsend_prefix.clear(); p->xrecv_prefix.clear();
  }

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
    C.add(s + "cres", P * D, p->Dr);   // scramble rows: Dr floats per token (attn_forward)
    C.add(s + "a", P * D, D);
    if (tr && !p->moe_recompute) C.add(s + "m1save", E * NL * P * D, D);
    C.add(s + "query1", P * D, D);
    C.add(s + "sq", P * 3 * D, 3 * D);
    C.add(s + "sstate", p->B * per_state, per_state);
    C.add(s + "sres", P * D, p->Dr);
    C.add(s + "bb", P * D, D);
    if (tr && !p->moe_recompute) C.add(s + "m2save", E * NL * P * D, D);
    C.add(s + "query2", P * D, D);
  }
  C.add("stage", E * P * D, D);
  if (D > 256) {                             // chainw.hip scratch: query-branch chains / input-function branch
    C.add("lw_scr", 2 * P * D, D);
    if (I > 0) C.add("lw_scr2", 2 * Qmax * D, D);
  }
  if (tr && p->moe_recompute && p->L > 0) C.add("mrsave", E * NL * P * D, D);
  if (p->sharded) {                          // scramble exchange scratch: head-major rows / packed peers
    C.add("xa", P * D, p->Dr);
    C.add("xb", P * D, p->Dr);
  }
  // attention segments
  make_chunks(p->xoff, p->qchunks, p->qchunk_off);
  p->fchunks.assign(I, {});
  p->fchunk_off.assign(I, {});
  for (int i = 0; i < I; ++i) make_chunks(p->fnoff[i], p->fchunks[i], p->fchunk_off[i]);
  if (tr) {
    C.add("dout", P * r4(p->out), r4(p->out));
    C.add("dquery", P * D, D);
    C.add("dsum0", P * D, D);
    C.add("dsum1", P * D, D);
    C.add("dres", P * D, p->Dr);
    C.add("dqkv0", P * 3 * D, 3 * D);
    C.add("dqkv1", P * 3 * D, 3 * D);
    for (int i = 0; i < KI; ++i) {
      C.add("du" + std::to_string(i), P * D, D);
      C.add("dden" + std::to_string(i), P * H, H);
    }
    C.add("dstate0", p->B * per_state, per_state);
    for (int l = 0; l < p->L; ++l)
      for (int i = 0; i < I; ++i) {
        C.add(p->dstate_fn(l, i), p->B * per_state, per_state);
        C.add(p->dkv_buf(l, i), p->Q[i] * 2 * D, 2 * D);
      }
    for (int i = 0; i < I; ++i) {
      C.add("dfn" + std::to_string(i), p->Q[i] * D, D);
    }
    if (p->input_grads) {
      C.add("dtheta_ws", (long)p->B * std::max(p->th, 1), std::max(p->th, 1));   // d theta before the copy out
      C.add("dxin", P * r4(p->in + p->th), r4(p->in + p->th));
      C.add("dxg", P * r4(p->in), r4(p->in));
      for (int i = 0; i < I; ++i) C.add("dfnin" + std::to_string(i), p->Q[i] * r4(p->F), r4(p->F));
    }
    C.add("dz0", E * NL * std::max(P, Qmax) * D, D);
    C.add("dz1", E * NL * P * D, D);
    if (I > 0) C.add("dzf", NL * Qmax * D, D);
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
    T.host.assign(firsts.size() * NL, ChainLayer{nullptr, nullptr, nullptr});   // filled at bind
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
  tbl(p->xsend.size() * sizeof(CopySeg)); tbl(p->xrecv.size() * sizeof(CopySeg));
  tbl(p->xsend_prefix.size() * sizeof(int)); tbl(p->xrecv_prefix.size() * sizeof(int));

  // point-reduction GEMM groups: built with null buffer pointers now (sizes only), rebuilt with
  // real pointers at bind
  build_groups(p);
  auto tbl_group = [&](const WgradGroup& G) {
    tbl(G.jobs.size() * sizeof(WgradJob));
    tbl(G.jobs.size() * sizeof(int) * 2);
    tbl(G.segs.size() * sizeof(int4));
    tbl(G.seg_start.size() * sizeof(int));
  };
  for_each_group(p, tbl_group);
  build_attn_tables(p);
  tbl(p->fwd_kv_jobs.size() * sizeof(LinearArgs));
  tbl(p->kvbwd_jobs.size() * sizeof(AttnKVBwdArgs));
  for (auto& v : p->dfn_jobs) tbl(v.size() * sizeof(LinearArgs));
  C.add("slab_wgrad", p->slab_wgrad_floats, 0);
  if (I > 0 && tr) C.add("slab_wgrad2", p->slab_wgrad_floats, 0);   // weight grads on side2
  C.add("slab_state", p->slab_state_floats, 0);
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
extern "C" int gnot_plan_bind_workspace_async(gnot_plan* p, void* workspace, size_t bytes, void* stream);
extern "C" int gnot_plan_bind_workspace(gnot_plan* p, void* workspace, size_t bytes) {
  const int rc = gnot_plan_bind_workspace_async(p, workspace, bytes, nullptr);
  if (rc != GNOT_OK) return rc;
  GNOT_CK(hipStreamSynchronize(nullptr));
  return GNOT_OK;
}

// Stream-ordered bind: the table image goes through a pinned staging slot and one hipMemcpyAsync on
// `stream`, so a new batch geometry costs no host synchronisation (the copy is ordered after the
// previous step's kernels on that stream, which have joined every side stream by then).
extern "C" int gnot_plan_bind_workspace_async(gnot_plan* p, void* workspace, size_t bytes, void* stream) {
  if (!p || !p->batch_set) return fail(GNOT_E_STATE, "set_batch first");
  if (!p->params_bound) return fail(GNOT_E_STATE, "bind_params first");
  if (!workspace || bytes < p->ws_need) return fail(GNOT_E_WORKSPACE, "workspace missing or too small");
  if (reinterpret_cast<uintptr_t>(workspace) & 255) return fail(GNOT_E_WORKSPACE, "workspace must be 256-byte aligned");
  p->ws = static_cast<char*>(workspace);
  for (auto& kv : p->bufs) kv.second.p = reinterpret_cast<float*>(p->ws + kv.second.off);
  const int NL = p->NL;

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
  // point-reduction GEMM groups with real pointers
  {
    const size_t slab_need = p->slab_wgrad_floats, slab_state_need = p->slab_state_floats;
    build_groups(p);
    if (p->slab_wgrad_floats != slab_need || p->slab_state_floats != slab_state_need)
      return fail(GNOT_E_INVALID, "internal: slab size changed at bind");
    for_each_group(p, [&](WgradGroup& G) {
      G.d_jobs = static_cast<WgradJob*>(put(G.jobs.data(), G.jobs.size() * sizeof(WgradJob)));
      std::vector<int> pre(G.wg_prefix);
      pre.insert(pre.end(), G.red_prefix.begin(), G.red_prefix.end());
      int* d = static_cast<int*>(put(pre.data(), pre.size() * sizeof(int)));
      G.d_wg_prefix = d;
      G.d_red_prefix = d + G.jobs.size();
      G.d_segs = G.segs.empty() ? nullptr : static_cast<int4*>(put(G.segs.data(), G.segs.size() * sizeof(int4)));
      G.d_seg_start = G.segs.empty() ? nullptr : static_cast<int*>(put(G.seg_start.data(), G.seg_start.size() * sizeof(int)));
    });
  }
  build_attn_tables(p);
  p->d_fwd_kv_jobs = static_cast<LinearArgs*>(put(p->fwd_kv_jobs.data(), p->fwd_kv_jobs.size() * sizeof(LinearArgs)));
  p->d_kvbwd_jobs = static_cast<AttnKVBwdArgs*>(put(p->kvbwd_jobs.data(), p->kvbwd_jobs.size() * sizeof(AttnKVBwdArgs)));
  p->d_dfn_jobs.clear();
  for (auto& v : p->dfn_jobs) p->d_dfn_jobs.push_back(static_cast<LinearArgs*>(put(v.data(), v.size() * sizeof(LinearArgs))));
  p->d_xsend = static_cast<CopySeg*>(put(p->xsend.data(), p->xsend.size() * sizeof(CopySeg)));
  p->d_xrecv = static_cast<CopySeg*>(put(p->xrecv.data(), p->xrecv.size() * sizeof(CopySeg)));
  p->d_xsend_prefix = static_cast<int*>(put(p->xsend_prefix.data(), p->xsend_prefix.size() * sizeof(int)));
  p->d_xrecv_prefix = static_cast<int*>(put(p->xrecv_prefix.data(), p->xrecv_prefix.size() * sizeof(int)));
  if (cur > p->table_bytes) return fail(GNOT_E_INVALID, "internal: table overflow");
  {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const int k = p->stage_next;
    p->stage_next = (k + 1) % gnot_plan::kStageSlots;
    if (!p->stage_ev[k]) GNOT_CK(hipEventCreateWithFlags(&p->stage_ev[k], hipEventDisableTiming));
    if (p->stage_used[k]) GNOT_CK(hipEventSynchronize(p->stage_ev[k]));   // only when the ring wraps in flight
    if (p->stage_cap[k] < cur) {
      if (p->stage[k]) GNOT_CK(hipHostFree(p->stage[k]));
      p->stage[k] = nullptr;
      p->stage_cap[k] = 0;
      const size_t cap = cur + cur / 2 + 4096;                           // headroom: growth is rare
      GNOT_CK(hipHostMalloc(&p->stage[k], cap, hipHostMallocDefault));
      p->stage_cap[k] = cap;
    }
    std::memcpy(p->stage[k], host.data(), cur);
    GNOT_CK(hipMemcpyAsync(tp, p->stage[k], cur, hipMemcpyHostToDevice, s));
    GNOT_CK(hipEventRecord(p->stage_ev[k], s));
    p->stage_used[k] = true;
  }
  // a padded width: the pad columns of rows that kernels write per head only (the attention backward's
  // dq / dk / dv, du) are read as exact zeros by the next backward-data products: clear the activation
  // part of the workspace once per bind (the tables follow it, uploaded after this on the same stream)
  if (p->padded())
    GNOT_CK(hipMemsetAsync(p->ws, 0, p->bufs["__tables"].off, static_cast<hipStream_t>(stream)));
  if (!p->side2) GNOT_CK(hipStreamCreateWithFlags(&p->side2, hipStreamNonBlocking));
  if (!p->side) {
    // same priority as the caller's stream: measured on MI355X, a low- (or high-) priority side
    // stream serialises against the main one and the step takes ~1.9x longer (round 1)
    GNOT_CK(hipStreamCreateWithPriority(&p->side, hipStreamNonBlocking, 0));
  }
  while (p->evs.size() < 256) {
    hipEvent_t e;
    GNOT_CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p->evs.push_back(e);
  }
  p->ws_bound = true;
  p->packed = false;
  p->fwd_done = false;
  p->bwd_done = false;
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

// records a start/stop event pair around one launch when `kind` is the profiled kernel class
struct ProfScope {
  Ctx& c;
  bool on = false;
  size_t idx = 0;
  hipStream_t st;
  ProfScope(Ctx& c_, const char* kind, double flops, hipStream_t stream = nullptr) : c(c_), st(stream ? stream : c_.s) {
    gnot_plan* p = c.p;
    if (p->prof_kind.empty() || p->prof_kind != kind) return;
    while (p->prof_events.size() < p->prof_used + 2) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      p->prof_events.push_back(e);
    }
    idx = p->prof_used;
    p->prof_used += 2;
    p->prof_flops += flops;
    p->prof_launches += 1;
    on = hipEventRecord(p->prof_events[idx], st) == hipSuccess;
  }
  ~ProfScope() {
    if (on) (void)hipEventRecord(c.p->prof_events[idx + 1], st);
  }
};

// ncol > 0: store only output columns [0, ncol) (a row pitch below NO: the attention's head-major
// scramble rows of the real width, attn_backward)
int run_linear(Ctx& c, const float* X, long ldx, int K, const Img& A, const float* bias, float* Y, long ldy,
               int NO, long P, int epi, int nsoft, int ncol = 0) {
  LinearArgs a{};
  a.nseg = 1; a.X[0] = X; a.Wp[0] = A.p; a.ldx = ldx; a.nsum = 1; a.sum_stride = 0; a.K = K;
  a.bias = bias; a.Y = Y; a.ldy = ldy; a.NO = NO; a.P = (int)P;
  a.epi = epi; a.nsoft = nsoft; a.dh = c.p->dh; a.np = c.p->npk(); a.img = c.p->lin_img();
  a.dreal = nsoft > 0 ? c.p->attn_dreal() : 0;
  a.dhr = (nsoft > 0 && c.p->head_padded()) ? c.p->dhr : 0;
  a.ncol = ncol;
  GNOT_CK(c.p->D == 256 ? launch_linear2(a, c.s) : launch_linear(a, c.p->D, c.s));
  return GNOT_OK;
}

// Y (+)= sum_s X_s A_s over K-segments that share one row pitch (backward-data of several Linears)
int run_linear_seg(Ctx& c, std::initializer_list<std::pair<const float*, const Img*>> segs, long ldx, float* Y,
                   long ldy, long P, int epi) {
  LinearArgs a{};
  a.nseg = 0;
  for (const auto& sg : segs) {
    a.X[a.nseg] = sg.first;
    a.Wp[a.nseg] = sg.second->p;
    ++a.nseg;
  }
  a.ldx = ldx; a.nsum = 1; a.K = c.p->D; a.bias = nullptr; a.Y = Y; a.ldy = ldy; a.NO = c.p->D; a.P = (int)P;
  a.epi = epi; a.nsoft = 0; a.dh = c.p->dh; a.np = c.p->npk(); a.img = c.p->lin_img();
  GNOT_CK(c.p->D == 256 ? launch_linear2(a, c.s) : launch_linear(a, c.p->D, c.s));
  return GNOT_OK;
}

// d > 256: the chainw.hip scratch of the stream a chain call runs on (the input-function branch on side2
// runs concurrently with the query branch)
ChainArgs& cw_scratch(gnot_plan* p, ChainArgs& a, hipStream_t s) {
  if (p->D > 256) a.scratch = p->P_(s == p->side2 ? "lw_scr2" : "lw_scr");
  return a;
}

ChainArgs chain_args(gnot_plan* p, const ChainTable& T, long P) {
  ChainArgs a{};
  a.D = p->D; a.KT0 = T.KT0; a.OTL = T.OTL; a.nlin = p->NL;
  a.layers_host = T.host.data();
  a.in_dim = T.in_dim; a.out_dim = T.out_dim; a.P = (int)P; a.nchains = T.nchains; a.layers = T.dev;
  a.np = p->npk();
  return a;
}

double group_flops(const WgradGroup& G) {
  double fl = 0.0;
  for (const auto& J : G.jobs) fl += 2.0 * J.P * (double)J.out * J.in;
  return fl;
}

// attention-state reductions: on the main stream (they are on the critical path)
int run_state(Ctx& c, const WgradGroup& G) {
  if (G.jobs.empty()) return GNOT_OK;
  ProfScope ps(c, "state", group_flops(G));
  GNOT_CK(launch_state(G.d_jobs, G.d_wg_prefix, (int)G.jobs.size(), G.total_wgs, G.d_red_prefix,
                       G.total_red, c.p->P_("slab_state"), G.jobs[0].out, G.jobs[0].state_dh, G.state_pts,
                       G.state_nw, G.state_mfma, c.s));
  return GNOT_OK;
}

hipEvent_t next_event(gnot_plan* p) {
  hipEvent_t e = p->evs[p->ev_next];
  p->ev_next = (p->ev_next + 1) % p->evs.size();
  return e;
}

// before the main stream overwrites `buf`, wait for the side-stream group that last read it
int flush_deferred(Ctx& c);
int guard_write(Ctx& c, const float* buf) {
  // a deferred group reads buf: launch it (and register) first.  flush_deferred empties the vector, so
  // decide before calling it
  const auto& dq = c.p->deferred;
  if (std::any_of(dq.begin(), dq.end(), [buf](const gnot_plan::DeferredWgrad& d) {
        return std::find(d.reads.begin(), d.reads.end(), buf) != d.reads.end();
      })) {
    const int rc = flush_deferred(c);
    if (rc != GNOT_OK) return rc;
  }
  auto it = c.p->readers.find(buf);
  if (it != c.p->readers.end()) {
    GNOT_CK(hipStreamWaitEvent(c.s, it->second, 0));
    c.p->readers.erase(it);
  }
  return GNOT_OK;
}

#define GNOT_RUN(expr)              \
  do {                              \
    const int rc_ = (expr);         \
    if (rc_ != GNOT_OK) return rc_; \
  } while (0)

// one weight-gradient group's launches (point-reduction GEMM + split-K reduce)
int launch_group(gnot_plan* p, const WgradGroup& G, float* slab, hipStream_t s) {
  if (G.b16)
    GNOT_CK(launch_wgrad_b16(G.d_jobs, G.d_wg_prefix, (int)G.jobs.size(), G.total_wgs, G.d_red_prefix, G.total_red,
                             slab, s, G.d_segs, G.d_seg_start));
  else
    GNOT_CK(launch_wgrad(G.d_jobs, G.d_wg_prefix, (int)G.jobs.size(), G.total_wgs, G.d_red_prefix, G.total_red, slab,
                         s, G.x6, G.wide, p->npk(), G.tw, G.d_segs, G.d_seg_start));
  return GNOT_OK;
}

// the group's gradient ranges summed over the ranks (gnot_plan_set_grad_comm) on the comm stream, once
// the event `done` (the group's kernels) has passed: consecutive canonical Linears are adjacent in the
// arena ((dW, db) per Linear), so a group is a few contiguous ranges, one collective each
int grad_allreduce(gnot_plan* p, const WgradGroup& G, hipEvent_t done) {
  GNOT_CK(hipStreamWaitEvent(p->comm_stream, done, 0));
  std::vector<int> ls(G.lins);
  std::sort(ls.begin(), ls.end());
  float* grads = p->P_("grads");
  for (size_t k = 0; k < ls.size();) {
    size_t m = k + 1;
    while (m < ls.size() && ls[m] == ls[m - 1] + 1) ++m;
    const long lo = p->grad_off[2 * ls[k]];
    const long hi = p->grad_off[2 * ls[m - 1] + 1] + p->lin_o[ls[m - 1]];
    if (p->grad_comm.allreduce_sum(p->grad_comm.user, grads + lo, hi - lo, p->comm_stream) != 0)
      return fail(GNOT_E_HIP, "gnot_comm.allreduce_sum (gradients) failed");
    k = m;
  }
  return GNOT_OK;
}

// weight gradients: on the caller's stream (plans of >= 65,536 points), or forked onto the side stream;
// `reads` are the main-stream buffers the group consumes, guarded until it finishes
int run_wgrad_side(Ctx& c, const WgradGroup& G, std::initializer_list<const float*> reads) {
  if (G.jobs.empty()) return GNOT_OK;
  gnot_plan* p = c.p;
  const bool serial = p->serial_wgrad();
  // Only the caller's (capture-origin) stream forks to the side stream.  A fork from the forked
  // input-function stream side2 segfaults the HIP runtime in hipStreamEndCapture (ROCm 7.2, torch
  // 2.10), while eager execution of the same sequence is correct.  Four topologies, each run once:
  //   r1   side2 -> side (side already forked from the origin), side joined into the origin only
  //   r2a  the same, side's event also joined back into side2 before side2 joins the origin
  //   r2b  side2 -> side3 (a stream used by nothing else), side3 joined into side2
  //   r2c  r2b + side3 also joined into the origin
  // all crash at the first capture; only first-level forks from the origin capture.  side2's weight
  // gradients therefore run in order on side2 with their own slab: they are the input-function
  // encoders' and the cross K/V Linears' (M ~ 10^3 points: tens of microseconds).  DESIGN.md
  // "capture fault".
  if (serial || c.s == p->side2) {
    float* slab = c.s == p->side2 ? p->P_("slab_wgrad2") : p->P_("slab_wgrad");
    {
      ProfScope ps(c, G.b16 ? "wgrad_b16" : "wgrad", group_flops(G));
      GNOT_RUN(launch_group(c.p, G, slab, c.s));
    }
    if (p->grad_comm_on) {
      hipEvent_t done = next_event(p);
      GNOT_CK(hipEventRecord(done, c.s));
      GNOT_RUN(grad_allreduce(p, G, done));
    }
    return GNOT_OK;
  }
  // forked: the side stream waits for what the caller's stream has issued so far (the fork event is
  // recorded now), but its launches are captured only after the caller's NEXT kernel (flush_deferred).  A
  // captured graph keeps a node's first-captured child on the node's own hardware queue; with the side
  // launch captured first, the main chain hopped to another queue at every fork, ~10 us of cross-queue
  // wait each (configs[1] trace, profiles/r05m_*: 8 MoE calls x 2 forks per step)
  hipEvent_t fork = next_event(p);
  GNOT_CK(hipEventRecord(fork, c.s));
  p->deferred.push_back({&G, std::vector<const float*>(reads), fork});
  return GNOT_OK;
}

// the deferred side-stream weight-gradient groups, in order; `c` is the capture-origin stream's context
int flush_deferred(Ctx& c) {
  gnot_plan* p = c.p;
  std::vector<gnot_plan::DeferredWgrad> pend;
  pend.swap(p->deferred);
  for (const auto& d : pend) {
    GNOT_CK(hipStreamWaitEvent(p->side, d.fork, 0));
    {
      // profiled as its own class: the bf16-row MoE weight gradients are HBM-bound, the others are not
      ProfScope ps(c, d.G->b16 ? "wgrad_b16" : "wgrad", group_flops(*d.G), p->side);
      GNOT_RUN(launch_group(p, *d.G, p->P_("slab_wgrad"), p->side));
    }
    hipEvent_t done = next_event(p);
    GNOT_CK(hipEventRecord(done, p->side));
    for (const float* r : d.reads) p->readers[r] = done;
    if (p->grad_comm_on) GNOT_RUN(grad_allreduce(p, *d.G, done));
  }
  return GNOT_OK;
}

// sum a state buffer over the ranks of a sharded batch
int shard_allreduce(Ctx& c, float* buf, long count) {
  gnot_plan* p = c.p;
  if (!p->sharded || count <= 0) return GNOT_OK;
  if (p->comm.allreduce_sum(p->comm.user, buf, count, c.s) != 0)
    return fail(GNOT_E_HIP, "gnot_comm.allreduce_sum failed");
  return GNOT_OK;
}

// forward scramble: local head-major apply output `hm` -> this rank's output tokens `tok`
// backward (reverse): token-order gradient `tok` -> local head-major `hm`
int shard_exchange(Ctx& c, float* hm, float* tok, bool reverse) {
  gnot_plan* p = c.p;
  float* xa = p->P_("xa");
  float* xb = p->P_("xb");
  const int ns = (int)p->xsend.size(), nr = (int)p->xrecv.size();
  if (!reverse) {
    GNOT_CK(launch_segcopy(p->d_xsend, p->d_xsend_prefix, ns, p->xsend_prefix.back(), hm, xa, false, c.s, p->xunit));
    if (p->comm.alltoallv(p->comm.user, xa, p->xsend_counts.data(), xb, p->xrecv_counts.data(), c.s) != 0)
      return fail(GNOT_E_HIP, "gnot_comm.alltoallv failed");
    GNOT_CK(launch_segcopy(p->d_xrecv, p->d_xrecv_prefix, nr, p->xrecv_prefix.back(), xb, tok, false, c.s, p->xunit));
  } else {
    GNOT_CK(launch_segcopy(p->d_xrecv, p->d_xrecv_prefix, nr, p->xrecv_prefix.back(), tok, xb, true, c.s, p->xunit));
    if (p->comm.alltoallv(p->comm.user, xb, p->xrecv_counts.data(), xa, p->xsend_counts.data(), c.s) != 0)
      return fail(GNOT_E_HIP, "gnot_comm.alltoallv failed");
    GNOT_CK(launch_segcopy(p->d_xsend, p->d_xsend_prefix, ns, p->xsend_prefix.back(), xa, hm, true, c.s, p->xunit));
  }
  return GNOT_OK;
}


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
    // keys/values/states of the input functions were computed for every block up front
    for (int i = 0; i < p->I; ++i) ap.state[i] = p->P_(s + "cstate" + std::to_string(i));
    ap.q = q; ap.ldq = D; ap.nsrc = p->I; ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff;
    ap.H = p->H; ap.dh = p->dh; ap.res = p->sharded ? p->P_("xb") : res_out;
    ap.dhr = p->head_padded() ? p->dhr : 0;
    GNOT_CK(launch_attn_apply_fwd(ap, c.s));
  } else {
    float* qkv = p->P_(cross ? s + "cq" : s + "sq");
    GNOT_RUN(run_linear(c, q_in, D, D, A.qkv, pbias + A.bqkv, qkv, 3 * D, 3 * D, P, EPI_STORE, 2 * D));
    float* st = p->P_(cross ? s + "cstate0" : s + "sstate");
    GNOT_RUN(run_state(c, cross ? p->st_c[l][0] : p->st_s[l]));
    GNOT_RUN(shard_allreduce(c, st, (long)p->B * p->H * (p->dh * p->dh + p->dh)));   // S, z over all ranks
    AttnApplyArgs ap{};
    ap.q = qkv; ap.ldq = 3 * D; ap.nsrc = 1; ap.state[0] = st; ap.chunks = p->d_qchunks; ap.nchunks = nq;
    ap.off = p->d_xoff; ap.H = p->H; ap.dh = p->dh; ap.res = p->sharded ? p->P_("xb") : res_out;
    ap.dhr = p->head_padded() ? p->dhr : 0;
    GNOT_CK(launch_attn_apply_fwd(ap, c.s));
  }
  if (p->sharded) GNOT_RUN(shard_exchange(c, p->P_("xb"), res_out, false));   // the scramble, across ranks
  // fc_out over the scramble rows: Dr columns per token (the head-major apply output viewed as rows of
  // H * dh = Dr floats, model.py:81-83), read zero-filled to the padded width
  GNOT_RUN(run_linear(c, res_out, p->Dr, p->Dr, A.o, pbias + A.bo, out, D, D, P, EPI_STORE, 0));
  return GNOT_OK;
}

// backward of one LinearAttention call; its output gradient is materialised in dsum_buf(cross).
// Accumulates d(query input) into dquery and forks the weight gradients of its 4+ Linears.
int attn_backward(Ctx& c, int l, bool cross) {
  gnot_plan* p = c.p;
  const long P = p->P;
  const int D = p->D;
  const std::string s = "b" + std::to_string(l) + ".";
  const int lo = cross ? p->lin_co(l) : p->lin_so(l);
  const int lq = cross ? p->lin_cq(l) : p->lin_sq(l);
  float* dsum = p->P_(p->dsum_buf(cross));
  float* dres = p->P_("dres");
  float* dquery = p->P_("dquery");
  float* dqkv = p->P_(p->dqkv_buf(cross));
  const int nq = (int)p->qchunks.size();
  GNOT_RUN(guard_write(c, dqkv));
  // fc_out backward-data: dres = dout W_o (token order); sharded: back to this rank's head-major rows
  GNOT_RUN(run_linear(c, dsum, D, D, p->T_img[lo], nullptr, dres, p->Dr, D, P, EPI_STORE, 0, p->Dr));
  if (p->sharded) {
    GNOT_RUN(shard_exchange(c, p->P_("xb"), dres, true));
    dres = p->P_("xb");
  }
  if (cross && p->I > 0) {
    const float* q = p->P_(s + "cq");
    AttnApplyArgs ap{};
    ap.q = q; ap.ldq = D; ap.nsrc = p->I; ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff;
    ap.H = p->H; ap.dh = p->dh; ap.dres = dres; ap.dq_pre = dqkv; ap.lddq = D; ap.lddu = D;
    ap.dhr = p->head_padded() ? p->dhr : 0;
    for (int i = 0; i < p->I; ++i) {
      const std::string si = std::to_string(i);
      ap.state[i] = p->P_(s + "cstate" + si);
      ap.du[i] = p->P_("du" + si);
      ap.dden[i] = p->P_("dden" + si);
    }
    GNOT_CK(launch_attn_apply_bwd(ap, c.s));
    // dS, dz per input function (kept per block: the dK/dV side of every block runs batched later)
    for (int i = 0; i < p->I; ++i) GNOT_RUN(run_state(c, p->dst_c[l][i]));
    GNOT_RUN(run_linear(c, dqkv, D, D, p->T_img[lq], nullptr, dquery, D, D, P, EPI_ACCUM, 0));
    GNOT_RUN(run_wgrad_side(c, p->wg_cross[l], {dsum, dqkv}));
  } else {
    const float* qkv = p->P_(cross ? s + "cq" : s + "sq");
    const int lk = cross ? p->lin_ck(l, 0) : p->lin_sk(l);
    const int lv = cross ? p->lin_cv(l, 0) : p->lin_sv(l);
    AttnApplyArgs ap{};
    ap.q = qkv; ap.ldq = 3 * D; ap.nsrc = 1; ap.state[0] = p->P_(cross ? s + "cstate0" : s + "sstate");
    ap.chunks = p->d_qchunks; ap.nchunks = nq; ap.off = p->d_xoff; ap.H = p->H; ap.dh = p->dh;
    ap.dres = dres; ap.dq_pre = dqkv; ap.lddq = 3 * D; ap.du[0] = p->P_("du0"); ap.lddu = D;
    ap.dden[0] = p->P_("dden0");
    ap.dhr = p->head_padded() ? p->dhr : 0;
    GNOT_CK(launch_attn_apply_bwd(ap, c.s));
    float* dst = p->P_("dstate0");
    GNOT_RUN(run_state(c, cross ? p->dst_c[l][0] : p->dst_s[l]));
    GNOT_RUN(shard_allreduce(c, dst, (long)p->B * p->H * (p->dh * p->dh + p->dh)));   // dS, dz over all ranks
    AttnKVBwdArgs kb{};
    kb.k = qkv + D; kb.v = qkv + 2 * D; kb.ldkv = 3 * D; kb.dstate = dst; kb.chunks = p->d_qchunks;
    kb.nchunks = nq; kb.H = p->H; kb.dh = p->dh; kb.dk = dqkv + D; kb.dv = dqkv + 2 * D; kb.lddkv = 3 * D;
    GNOT_CK(launch_attn_kv_bwd(kb, c.s));
    GNOT_RUN(run_linear_seg(c, {{dqkv, &p->T_img[lq]}, {dqkv + D, &p->T_img[lk]}, {dqkv + 2 * D, &p->T_img[lv]}},
                            3 * D, dquery, D, P, EPI_ACCUM));
    GNOT_RUN(run_wgrad_side(c, cross ? p->wg_cross[l] : p->wg_self[l], {dsum, dqkv}));
  }
  return GNOT_OK;
}

}  // namespace

// the soft-MoE experts of one call: the expert grid writes the [E, P, d] stage (bf16 mode at d = 256: bf16
// stage rows), a moe_combine pass sums residual + experts in expert order (chain2.hip names the forms that
// were measured slower and removed)
static bool moe_stage_b16(gnot_plan* p) { return p->b16s(); }
// stage_stride: floats between two experts' stage rows (the stage buffer's P * D; the bf16 training forward's
// stage rows are its save slot nl-1, one save chain apart)
static hipError_t launch_moe_pass(gnot_plan* p, const float* base, const float* stage, float* out, hipStream_t s,
                                  long stage_stride = 0) {
  const long P = p->P, D = p->D;
  if (stage_stride == 0) stage_stride = P * D;
  return p->b16s() ? launch_moe_combine_b16(base, stage, stage_stride, p->E, out, P, s)
                   : launch_moe_combine(base, stage, stage_stride, p->E, out, P * D, s);
}
// save (and dZ) layout of a soft-MoE chain call: fp32 [NL][P][D] per expert, or in bf16 mode 2 NL bf16
// layers per expert (ChainArgs::b16s)
static void moe_save_strides(gnot_plan* p, ChainArgs& a) {
  const long P = p->P, D = p->D, NL = p->NL;
  a.b16s = p->b16s() ? 1 : 0;
  a.save_layer_stride = a.b16s ? P * D / 2 : P * D;
  a.save_chain_stride = NL * P * D;
}

static int moe_forward(Ctx& c, const ChainTable& T, const float* in, const float* qin, float* qout, float* save) {
  gnot_plan* p = c.p;
  const long P = p->P;
  const int D = p->D, E = p->E, NL = p->NL;
  ChainArgs a = chain_args(p, T, P);
  a.X = in; a.ldx = D; a.ldy = D;
  a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.mode = CH_MOE;
  moe_save_strides(p, a);                 // bf16 mode: bf16 expert terms with or without saves
  a.save = save;
  a.Y = p->P_("stage"); a.y_chain_stride = P * D;
  if (p->b16s() && save) {
    // bf16 training: the experts' bf16 score-scaled terms are kept in save slot nl-1 (the backward's d score
    // operand), so the stage rows ARE that slot (chain2.hip): no separate stage write
    a.Y = save + (NL - 1) * a.save_layer_stride;
    a.y_chain_stride = a.save_chain_stride;
  }
  a.stage_b16 = moe_stage_b16(p) ? 1 : 0;
  {
    ProfScope ps(c, "moe_fwd", 2.0 * E * P * NL * (double)D * D);
    GNOT_CK(launch_chain_fwd(cw_scratch(p, a, c.s), c.s));
  }
  GNOT_CK(launch_moe_pass(p, qin, a.Y, qout, c.s, a.y_chain_stride));
  return GNOT_OK;
}

// A call that fails part-way through a stream capture (e.g. a collective callback refused) leaves the side
// streams it forked into the capture unjoined, and hipStreamEndCapture then fails with "unjoined work" and
// leaves the caller's stream capturing.  Every side stream still in the capture joins the caller's stream
// again before the error returns, so the capture ends (the caller discards the graph); eager calls skip it.
static void rejoin_side_streams(gnot_plan* p, hipStream_t origin) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(origin, &st) != hipSuccess || st != hipStreamCaptureStatusActive) return;
  for (hipStream_t s : {p->side, p->side2, p->comm_stream}) {
    hipStreamCaptureStatus ss = hipStreamCaptureStatusNone;
    if (!s || hipStreamIsCapturing(s, &ss) != hipSuccess || ss != hipStreamCaptureStatusActive) continue;
    hipEvent_t e = next_event(p);
    if (hipEventRecord(e, s) == hipSuccess) (void)hipStreamWaitEvent(origin, e, 0);
  }
}

static int forward_impl(gnot_plan* p, const float* x, const float* theta, const float* const* fns, float* out,
                        void* stream);
static int backward_impl(gnot_plan* p, const float* dout, void* stream);
extern "C" int gnot_forward(gnot_plan* p, const float* x, const float* theta, const float* const* fns,
                            float* out, void* stream) {
  const int rc = forward_impl(p, x, theta, fns, out, stream);
  if (rc != GNOT_OK && p) rejoin_side_streams(p, static_cast<hipStream_t>(stream));
  return rc;
}
extern "C" int gnot_backward(gnot_plan* p, const float* dout, void* stream) {
  const int rc = backward_impl(p, dout, stream);
  if (rc != GNOT_OK && p) rejoin_side_streams(p, static_cast<hipStream_t>(stream));
  return rc;
}

static int forward_impl(gnot_plan* p, const float* x, const float* theta, const float* const* fns, float* out,
                        void* stream) {
  if (!p || !p->ws_bound) return fail(GNOT_E_STATE, "bind_workspace first");
  if (!p->packed) return fail(GNOT_E_STATE, "gnot_pack_weights must run before gnot_forward");
  if (!x || !theta || !out || (p->I > 0 && !fns)) return fail(GNOT_E_INVALID, "null input");
  Ctx c{p, static_cast<hipStream_t>(stream)};
  const long P = p->P;
  const int D = p->D, NL = p->NL;
  const bool tr = p->training;
  // the input-function branch (encoders, every block's K/V projections and states) depends only on
  // the input functions: it runs on side2 while the query branch (gating, x encoder) runs here.  The
  // query branch is issued first (graph replay dispatches in capture order).
  const bool br = p->I > 0;
  Ctx cf{p, br ? p->side2 : c.s};
  if (br) {
    hipEvent_t fork = next_event(p);
    GNOT_CK(hipEventRecord(fork, c.s));
    GNOT_CK(hipStreamWaitEvent(cf.s, fork, 0));
  }
  // inputs into the workspace (row pitch rounded to 16 B)
  GNOT_CK(hipMemcpy2DAsync(p->P_("x"), p->bufs["x"].ld * 4, x, p->in * 4, p->in * 4, P, hipMemcpyDeviceToDevice, c.s));
  GNOT_CK(hipMemcpyAsync(p->P_("theta"), theta, (size_t)p->B * p->th * 4, hipMemcpyDeviceToDevice, c.s));
  GNOT_CK(launch_concat_theta(p->P_("x"), p->bufs["x"].ld, p->in, p->P_("theta"), p->th, p->d_xoff, p->B,
                              p->P_("xin"), p->bufs["xin"].ld, (int)P, c.s));
  // gating (model.py:155-156)
  {
    ChainArgs a = chain_args(p, p->ch_gate, P);
    a.X = p->P_("x"); a.ldx = p->bufs["x"].ld;
    a.Y = p->P_("scores"); a.ldy = p->bufs["scores"].ld; a.mode = CH_SOFTMAX;
    if (tr) { a.save = p->P_("gate_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(cw_scratch(p, a, c.s), c.s));
  }
  // query encoder (model.py:158-161)
  {
    ChainArgs a = chain_args(p, p->ch_x, P);
    a.X = p->P_("xin"); a.ldx = p->bufs["xin"].ld;
    a.Y = p->P_("query0"); a.ldy = D; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("x_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(cw_scratch(p, a, c.s), c.s));
  }
  for (int i = 0; i < p->I; ++i) {
    const std::string n = "fn" + std::to_string(i);
    if (p->Q[i] > 0)
      GNOT_CK(hipMemcpy2DAsync(p->P_(n), p->bufs[n].ld * 4, fns[i], p->F * 4, p->F * 4, p->Q[i],
                               hipMemcpyDeviceToDevice, cf.s));
  }
  // input-function encoders (model.py:164-166)
  for (int i = 0; i < p->I; ++i) {
    const std::string si = std::to_string(i);
    ChainArgs a = chain_args(p, p->ch_fn[i], p->Q[i]);
    a.X = p->P_("fn" + si); a.ldx = p->bufs["fn" + si].ld;
    a.Y = p->P_("fnenc" + si); a.ldy = D; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("fn_save" + si); a.save_layer_stride = p->Q[i] * D; a.save_chain_stride = NL * p->Q[i] * D; }
    GNOT_CK(launch_chain_fwd(cw_scratch(p, a, cf.s), cf.s));
  }
  // key/value projections (model.py:67-75) and states (model.py:77-79) of every (block, input
  // function): they depend only on the input-function encodings, so all L*I of them run batched here
  if (p->I > 0 && p->L > 0) {
    long Qmax = 0;
    for (long q : p->Q) Qmax = std::max(Qmax, q);
    GNOT_CK(launch_linear_batch(p->d_fwd_kv_jobs, (int)p->fwd_kv_jobs.size(), (int)Qmax, 2 * D, D > 512 ? D / 2 : D,
                                p->dh, cf.s));
    GNOT_RUN(run_state(cf, p->st_fn));
  }
  if (br) {                                // join the input-function branch
    hipEvent_t join = next_event(p);
    GNOT_CK(hipEventRecord(join, cf.s));
    GNOT_CK(hipStreamWaitEvent(c.s, join, 0));
  }
  // blocks (model.py:126-139)
  for (int l = 0; l < p->L; ++l) {
    const std::string s = "b" + std::to_string(l) + ".";
    const float* qin = p->P_(p->block_query(l));
    GNOT_RUN(attn_forward(c, l, true, qin, p->P_(s + "cres"), p->P_(s + "a")));
    // ffn1 experts: query1 = query + sum_e s_e ffn1_e(a)   (model.py:128-131)
    GNOT_RUN(moe_forward(c, p->ch_m1[l], p->P_(s + "a"), qin, p->P_(s + "query1"),
                         tr && !p->moe_recompute ? p->P_(s + "m1save") : nullptr));
    GNOT_RUN(attn_forward(c, l, false, p->P_(s + "query1"), p->P_(s + "sres"), p->P_(s + "bb")));
    // ffn2 experts: query2 = query1 + sum_e s_e ffn2_e(bb)   (model.py:134-137)
    GNOT_RUN(moe_forward(c, p->ch_m2[l], p->P_(s + "bb"), p->P_(s + "query1"), p->P_(s + "query2"),
                         tr && !p->moe_recompute ? p->P_(s + "m2save") : nullptr));
  }
  // decoder (model.py:171)
  {
    ChainArgs a = chain_args(p, p->ch_out, P);
    a.X = p->P_(p->final_query()); a.ldx = D; a.Y = out; a.ldy = p->out; a.mode = CH_STORE;
    if (tr) { a.save = p->P_("out_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D; }
    GNOT_CK(launch_chain_fwd(cw_scratch(p, a, c.s), c.s));
  }
  p->fwd_done = true;
  p->bwd_done = false;
  return GNOT_OK;
}

static int backward_impl(gnot_plan* p, const float* dout, void* stream) {
  if (!p || !p->ws_bound || !p->fwd_done) return fail(GNOT_E_STATE, "gnot_forward must run before gnot_backward");
  if (!p->training) return fail(GNOT_E_STATE, "plan was set up with training = 0");
  if (!dout) return fail(GNOT_E_INVALID, "null dout");
  Ctx c{p, static_cast<hipStream_t>(stream)};
  const long P = p->P;
  const int D = p->D, E = p->E, NL = p->NL;
  float* dquery = p->P_("dquery");
  float* stage = p->P_("stage");
  p->readers.clear();
  p->deferred.clear();
  if (p->grad_comm_on) {                   // the comm stream joins here (a first-level fork of the caller's)
    if (!p->comm_stream) GNOT_CK(hipStreamCreateWithFlags(&p->comm_stream, hipStreamNonBlocking));
    hipEvent_t fork = next_event(p);
    GNOT_CK(hipEventRecord(fork, c.s));
    GNOT_CK(hipStreamWaitEvent(p->comm_stream, fork, 0));
  }
  GNOT_CK(hipMemcpy2DAsync(p->P_("dout"), p->bufs["dout"].ld * 4, dout, p->out * 4, p->out * 4, P,
                           hipMemcpyDeviceToDevice, c.s));
  GNOT_CK(hipMemsetAsync(p->P_("dscore"), 0, P * p->bufs["dscore"].ld * 4, c.s));
  // one chain backward: dZ of every Linear into the chain call's dz slot, then its weight gradients
  // are forked to the side stream
  auto chain_bwd_on = [&](Ctx& cc, ChainArgs& a, int kcall, long rows, const WgradGroup& G, const char* prof) -> int {
    float* dz = p->P_(p->dz_name(kcall));
    GNOT_RUN(guard_write(cc, dz));
    a.dz = dz; a.dz_layer_stride = rows * D; a.dz_chain_stride = NL * rows * D;
    if (a.b16s) { a.dz_layer_stride /= 2; a.dz_chain_stride /= 2; }   // bf16 dZ layers
    {
      ProfScope ps(cc, prof, 2.0 * a.nchains * rows * NL * (double)D * D);
      GNOT_CK(launch_chain_bwd(cw_scratch(p, a, cc.s), cc.s));
    }
    if (cc.s == c.s) GNOT_RUN(flush_deferred(cc));   // earlier groups' side launches after this kernel
    // the weight gradients read the saved pre-activations too: a recomputed (shared) save buffer
    // must not be overwritten by the next MoE's recompute before they finish.  That guard is the
    // readers map, which only run_wgrad_side from the capture-origin stream registers (side2 runs its
    // groups in order without it): the MoE chains must therefore stay on the origin stream
    if (p->moe_recompute && a.mode == CH_MOE) {
      if (cc.s != c.s) return fail(GNOT_E_STATE, "internal: MoE recompute backward off the origin stream");
      return run_wgrad_side(cc, G, {dz, a.save});
    }
    return run_wgrad_side(cc, G, {dz});
  };
  auto chain_bwd = [&](ChainArgs& a, int kcall, long rows, const WgradGroup& G, const char* prof) -> int {
    return chain_bwd_on(c, a, kcall, rows, G, prof);
  };
  // decoder (model.py:171)
  {
    ChainArgs a = chain_args(p, p->ch_out, P);
    a.dY = p->P_("dout"); a.lddy = p->bufs["dout"].ld; a.mode = CH_STORE;
    a.save = p->P_("out_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    a.dX = dquery; a.lddx = D; a.dx_chain_stride = 0;
    GNOT_RUN(chain_bwd(a, p->k_out(), P, p->wg_out, "chain_bwd"));
  }
  for (int l = p->L - 1; l >= 0; --l) {
    const std::string s = "b" + std::to_string(l) + ".";
    // ffn2 experts: query2 = query1 + sum_e s_e ffn2_e(bb)   (model.py:134-137)
    for (int m = 2; m >= 1; --m) {
      const bool m1 = (m == 1);
      if (p->moe_recompute) {
        // re-run this call's expert forward (inputs kept: "a" / "bb") into the shared save buffer
        float* mr = p->P_("mrsave");
        GNOT_RUN(guard_write(c, mr));
        ChainArgs f = chain_args(p, m1 ? p->ch_m1[l] : p->ch_m2[l], P);
        f.X = p->P_(s + (m1 ? "a" : "bb")); f.ldx = D; f.ldy = D;
        f.scores = p->P_("scores"); f.ldsc = (int)p->bufs["scores"].ld; f.mode = CH_MOE;
        f.save = mr; moe_save_strides(p, f);
        // only the saves are needed: no output (Y = null), no combine
        f.Y = nullptr; f.y_chain_stride = P * D;
        ProfScope ps(c, "moe_recompute", 2.0 * E * P * NL * (double)D * D);
        GNOT_CK(launch_chain_fwd(cw_scratch(p, f, c.s), c.s));
      }
      ChainArgs a = chain_args(p, m1 ? p->ch_m1[l] : p->ch_m2[l], P);
      a.dY = dquery; a.lddy = D; a.mode = CH_MOE;
      a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld; a.dscore = p->P_("dscore");
      a.save = p->P_(p->msave(l, m1)); moe_save_strides(p, a);
      float* dsum = p->P_(p->dsum_buf(m1));
      // d(MoE input) = sum_e W_e0^T dz_e0: each expert's term into the stage, summed by moe_combine
      GNOT_RUN(guard_write(c, dsum));
      a.dX = stage; a.lddx = D; a.dx_chain_stride = P * D;
      a.stage_b16 = moe_stage_b16(p) ? 1 : 0;
      GNOT_RUN(chain_bwd(a, m1 ? p->k_m1(l) : p->k_m2(l), P, m1 ? p->wg_m1[l] : p->wg_m2[l], "moe_bwd"));
      GNOT_CK(launch_moe_pass(p, nullptr, stage, dsum, c.s));
      GNOT_RUN(flush_deferred(c));            // the chain's weight gradients: side launch after the pass
      // m2: self attention (model.py:133) ; m1: cross attention (model.py:127)
      GNOT_RUN(attn_backward(c, l, m1));
    }
  }
  // the input-function branch again runs on side2, concurrently with the query encoder and gating
  const bool br = p->I > 0;
  Ctx cf{p, br ? p->side2 : c.s};
  // ranks issue their gradient collectives in one host order whatever serial_wgrad() says (it is chosen
  // per rank from the local point count): a forked rank still holds the last attention call's groups
  // (wg_cross[0]) deferred here, and side2 issues its groups' all-reduces at once -- flush first
  if (p->grad_comm_on) GNOT_RUN(flush_deferred(c));
  if (br) {
    hipEvent_t fork = next_event(p);
    GNOT_CK(hipEventRecord(fork, c.s));
    GNOT_CK(hipStreamWaitEvent(cf.s, fork, 0));
  }
  // dK, dV of every (block, input function), the encodings' gradient and the key/value weight
  // gradients, batched over blocks
  if (p->I > 0 && p->L > 0) {
    long Qmax = 0;
    int maxch = 0;
    for (int i = 0; i < p->I; ++i) {
      Qmax = std::max(Qmax, p->Q[i]);
      maxch = std::max(maxch, (int)p->fchunks[i].size());
    }
    GNOT_CK(launch_attn_kv_bwd_batch(p->d_kvbwd_jobs, (int)p->kvbwd_jobs.size(), maxch, p->H, p->dh, cf.s));
    for (size_t k = 0; k < p->d_dfn_jobs.size(); ++k)
      GNOT_CK(launch_linear_batch(p->d_dfn_jobs[k], p->I, (int)Qmax, D, D > 512 ? D / 2 : D, p->dh, cf.s));
    GNOT_RUN(run_wgrad_side(cf, p->wg_fnkv, {}));
  }
  if (p->I > 0 && p->L == 0)   // encodings unused by the output: zero gradients
    for (int i = 0; i < p->I; ++i)
      GNOT_CK(hipMemsetAsync(p->P_("dfn" + std::to_string(i)), 0, p->Q[i] * D * 4, cf.s));
  // input-function encoders (their inputs need no gradient)
  for (int i = 0; i < p->I; ++i) {
    const std::string si = std::to_string(i);
    ChainArgs a = chain_args(p, p->ch_fn[i], p->Q[i]);
    a.dY = p->P_("dfn" + si); a.lddy = D; a.mode = CH_STORE;
    a.save = p->P_("fn_save" + si); a.save_layer_stride = p->Q[i] * D; a.save_chain_stride = NL * p->Q[i] * D;
    if (p->input_grads) { a.dX = p->P_("dfnin" + si); a.lddx = p->bufs["dfnin" + si].ld; a.dx_chain_stride = 0; }
    GNOT_RUN(chain_bwd_on(cf, a, p->k_fn(i), p->Q[i], p->wg_fn[i], "chain_bwd"));
  }
  // query encoder
  {
    ChainArgs a = chain_args(p, p->ch_x, P);
    a.dY = dquery; a.lddy = D; a.mode = CH_STORE;
    a.save = p->P_("x_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    if (p->input_grads) { a.dX = p->P_("dxin"); a.lddx = p->bufs["dxin"].ld; a.dx_chain_stride = 0; }
    GNOT_RUN(chain_bwd(a, p->k_x(), P, p->wg_x, "chain_bwd"));
  }
  // gating: d scores accumulated over every MoE above -> softmax backward -> chain.  With the weight
  // gradients forked and an input-function branch, the gating's own group runs HERE after the branch has
  // joined, on the branch's slab (free by then): forked, it queued behind the query encoder's group on the
  // side stream and ended the step ~45 us later (configs[1] trace); its all-reduce keeps its place, last
  const bool gate_here = br && !p->serial_wgrad();
  {
    ChainArgs a = chain_args(p, p->ch_gate, P);
    a.mode = CH_SOFTMAX; a.scores = p->P_("scores"); a.ldsc = (int)p->bufs["scores"].ld;
    a.dscore = p->P_("dscore");
    a.save = p->P_("gate_save"); a.save_layer_stride = P * D; a.save_chain_stride = NL * P * D;
    if (p->input_grads) { a.dX = p->P_("dxg"); a.lddx = p->bufs["dxg"].ld; a.dx_chain_stride = 0; }
    if (gate_here) {
      float* dz = p->P_(p->dz_name(p->k_gate()));
      GNOT_RUN(guard_write(c, dz));
      a.dz = dz; a.dz_layer_stride = P * D; a.dz_chain_stride = NL * P * D;
      {
        ProfScope ps(c, "chain_bwd", 2.0 * a.nchains * P * NL * (double)D * D);
        GNOT_CK(launch_chain_bwd(cw_scratch(p, a, c.s), c.s));
      }
      GNOT_RUN(flush_deferred(c));           // the query encoder's group: side launch after this kernel
    } else {
      GNOT_RUN(chain_bwd(a, p->k_gate(), P, p->wg_gate, "chain_bwd"));
    }
  }
  if (br) {                                // join the input-function branch
    hipEvent_t joinf = next_event(p);
    GNOT_CK(hipEventRecord(joinf, cf.s));
    GNOT_CK(hipStreamWaitEvent(c.s, joinf, 0));
  }
  if (gate_here && !p->wg_gate.jobs.empty()) {
    {
      ProfScope ps(c, "wgrad", group_flops(p->wg_gate));
      GNOT_RUN(launch_group(p, p->wg_gate, p->P_("slab_wgrad2"), c.s));
    }
    if (p->grad_comm_on) {
      hipEvent_t done = next_event(p);
      GNOT_CK(hipEventRecord(done, c.s));
      GNOT_RUN(grad_allreduce(p, p->wg_gate, done));
    }
  }
  GNOT_RUN(flush_deferred(c));
  // join the side stream: every gradient is complete when the caller's stream moves on
  hipEvent_t join = next_event(p);
  GNOT_CK(hipEventRecord(join, p->side));
  GNOT_CK(hipStreamWaitEvent(c.s, join, 0));
  if (p->grad_comm_on) {                   // ... and summed over the ranks
    hipEvent_t joinc = next_event(p);
    GNOT_CK(hipEventRecord(joinc, p->comm_stream));
    GNOT_CK(hipStreamWaitEvent(c.s, joinc, 0));
  }
  p->readers.clear();
  p->bwd_done = true;
  p->ig_reduced = false;
  return GNOT_OK;
}

// reference autograd's gradients of x, theta and the input functions (model.py:155-166), from the
// encoders' input gradients of the last gnot_backward
extern "C" int gnot_input_grads(gnot_plan* p, float* dx, float* dtheta, float* const* dfns, void* stream) {
  if (!p || !p->input_grads || !p->ws_bound || !p->training)
    return fail(GNOT_E_STATE, "gnot_plan_set_input_grads(plan, 1) and a training batch are required");
  if (!p->bwd_done)
    return fail(GNOT_E_STATE, "gnot_input_grads reads the encoders' input gradients of a gnot_backward, which must "
                              "follow the last gnot_forward");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const Buf& xin = p->bufs.at("dxin");
  const Buf& xg = p->bufs.at("dxg");
  if (dx) GNOT_CK(launch_add_cols(xin.p, xin.ld, xg.p, xg.ld, p->in, dx, p->P, s));
  // point-sharded: x's rows are local, but theta (broadcast over ALL points of a sample) and the input
  // functions (replicated on every rank, reached through every rank's attention states) get one partial
  // gradient per rank -- summed over the ranks (every rank must call this: the sums are collectives)
  float* dth = p->P_("dtheta_ws");
  if (dtheta || p->sharded) GNOT_CK(launch_seg_colsum(xin.p, xin.ld, p->in, p->th, p->d_xoff, p->B, dth, s));
  if (p->sharded && p->th > 0) {
    Ctx c{p, s};
    GNOT_RUN(shard_allreduce(c, dth, (long)p->B * p->th));
  }
  if (dtheta && p->th > 0)
    GNOT_CK(hipMemcpyAsync(dtheta, dth, (size_t)p->B * p->th * 4, hipMemcpyDeviceToDevice, s));
  for (int i = 0; i < p->I; ++i) {
    const Buf& f = p->bufs.at("dfnin" + std::to_string(i));
    if (p->sharded && !p->ig_reduced) {
      Ctx c{p, s};
      GNOT_RUN(shard_allreduce(c, f.p, p->Q[i] * f.ld));
    }
    if (dfns && dfns[i]) GNOT_CK(launch_add_cols(f.p, f.ld, nullptr, 0, p->F, dfns[i], p->Q[i], s));
  }
  p->ig_reduced = true;
  return GNOT_OK;
}

extern "C" int gnot_profile_enable(gnot_plan* p, const char* kind) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  p->prof_kind = kind ? kind : "";
  p->prof_used = 0;
  p->prof_flops = 0.0;
  p->prof_launches = 0;
  return GNOT_OK;
}

extern "C" int gnot_profile_read(gnot_plan* p, double* ms_total, int64_t* launches, double* flops_total) {
  if (!p) return fail(GNOT_E_INVALID, "null plan");
  double ms = 0.0;
  for (size_t k = 0; k + 1 < p->prof_used; k += 2) {
    GNOT_CK(hipEventSynchronize(p->prof_events[k + 1]));
    float t = 0.f;
    GNOT_CK(hipEventElapsedTime(&t, p->prof_events[k], p->prof_events[k + 1]));
    ms += t;
  }
  if (ms_total) *ms_total = ms;
  if (launches) *launches = p->prof_launches;
  if (flops_total) *flops_total = p->prof_flops;
  p->prof_used = 0;
  p->prof_flops = 0.0;
  p->prof_launches = 0;
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

// ====================================================================== training step
extern "C" size_t gnot_rel_l2_work_floats(const int64_t* off_host, int B, int C) {
  if (!off_host || B <= 0 || C <= 0) return 0;
  std::vector<long> off(off_host, off_host + B + 1);
  return (size_t)B * rel_l2_splits(off.data(), B) * 2 * C + (size_t)B * C;
}

extern "C" int gnot_rel_l2_loss(const float* pred, const float* tgt, const int64_t* off_dev, const int64_t* off_host,
                                int B, int C, float* work, float* loss, float* dpred, void* stream) {
  if (!pred || !tgt || !off_dev || !off_host || B <= 0 || C <= 0 || !work || !loss)
    return fail(GNOT_E_INVALID, "bad rel_l2 arguments");
  std::vector<long> off(off_host, off_host + B + 1);
  if (off[0] != 0) return fail(GNOT_E_INVALID, "off[0] must be 0");
  for (int b = 0; b < B; ++b)
    if (off[b + 1] < off[b]) return fail(GNOT_E_INVALID, "offsets must be non-decreasing");
  GNOT_CK(launch_rel_l2(pred, tgt, reinterpret_cast<const long*>(off_dev), B, C, rel_l2_splits(off.data(), B),
                        off[B], work, loss, dpred, static_cast<hipStream_t>(stream)));
  return GNOT_OK;
}

extern "C" int gnot_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                               const float* hyper, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || n < 0 || !hyper) return fail(GNOT_E_INVALID, "bad adamw arguments");
  GNOT_CK(launch_adamw(param, grad, exp_avg, exp_avg_sq, n, hyper, static_cast<hipStream_t>(stream)));
  return GNOT_OK;
}

extern "C" const char* gnot_last_error(void) { return g_err.c_str(); }
extern "C" const char* gnot_version(void) { return "gnot-mi355x 0.1 (gfx950, fp32 MFMA)"; }
