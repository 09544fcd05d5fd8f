// Internal (C++) launcher interface between the engine and the HIP kernels.
// The public C-ABI lives in include/gnot_hip.h; nothing here crosses the library boundary.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gnot {

// ------------------------------------------------------------------ weight packing (pack.hip)
// One Linear (W [out, in] row-major, bias [out]) written into the fragment-order image used as the
// MFMA A operand (see gnot_common.h).  transposed=0: A = W   (forward, out = x W^T + b)
//                                       transposed=1: A = W^T (backward data, dx = dy W)
// Tile (o, T) of this matrix lands at dst[((o0 + o) * ktot + t0 + T) * 64 + lane] (float4 units), so
// several Linears can be concatenated along either dimension of one packed matrix.
struct PackJob {
  const float* W;
  const float* b;      // may be null; only used when bias_dst != null
  float4* dst;
  float* bias_dst;     // padded bias copy (16*OTp floats, zero filled), or null
  int out, in;
  int transposed;
  int o0, t0, ktot;
  int OTp, KTp;        // tile counts of this job's image (>= what out/in need; the rest is zero)
  int x6;              // 1: bf16x6 image (3 bf16 pieces per 16x32 block, k-major, gnot_common.h); 2: the
                       //    same output-major (chain2.hip); 3: output-major, 1 RNE bf16 piece; 4: k-major,
                       //    1 RNE bf16 piece (chain.hip in the bf16 mode); 0: fp32
  int otot;            // x6: output tiles of the whole image (its k-major block stride)
  // padded heads (a head width d / H that is not a multiple of 4): W's rows come in H heads of hr real rows,
  // the image holds them in heads of hp >= hr (row h * hp + j <- W row h * hr + j, j < hr; the rest zero).
  // out is then H * hp.  Applies to the image rows (forward) or the contraction index (transposed) and to
  // the bias copy.  0: rows map 1:1
  int hr = 0, hp = 0;
  // internal widths above 512 (fp32 images): the contraction in two halves of kh tiles, each half a whole
  // image of its own -- tile (o, T) at ((T / kh) * otot + o) * kh + T % kh -- so that a projection runs as two
  // K-segments of the 320 .. 512-wide kernels (launch_linear).  0: one image, ktot tiles deep
  int kh = 0;
};
// pack tiles of a job: fp32 images have OTp*KTp tiles, x6 images OTp*ceil(KTp/2) blocks
inline int pack_tiles(const PackJob& J) { return J.x6 ? J.OTp * ((J.KTp + 1) / 2) : J.OTp * J.KTp; }
hipError_t launch_pack(const PackJob* jobs_dev, const int* tile_prefix_dev, int njobs,
                       int total_tiles, hipStream_t s);

// ------------------------------------------------------------------ projections (linear.hip)
enum LinearEpi { EPI_STORE = 0, EPI_ACCUM = 1 };
constexpr int kMaxSeg = 8;
struct LinearArgs {
  int nseg;                          // K-segments: Y = sum_s X[s] . A_s (+ bias)
  const float* X[kMaxSeg];           // segment input rows X[s] + p*ldx, K columns each
  const float4* Wp[kMaxSeg];         // segment packed A images (NO/16 x ceil(K/16) tiles)
  long ldx;
  int nsum;                          // segment 0 only: input = sum_{t<nsum} X[0][t*sum_stride + ...]
  long sum_stride;
  int K;                             // real input columns (<= D)
  const float* bias;                 // padded bias or null
  float* Y;
  long ldy;
  int NO;                            // output columns (multiple of D)
  int P;                             // rows
  int epi;                           // LinearEpi
  int nsoft;                         // feature-softmax on output columns [0, nsoft)
  int dh;                            // head width for that softmax
  int np = 3;                        // linear2: operand pieces (3 = bf16x6, 1 = bf16 mode)
  // linear.hip (d <= 192): 0 = fp32 fragment images on the fp32 MFMA; 1 / 3 = output-major bf16-piece images
  // (the bf16 mode / the fp32 mode's bf16x6, kLinearX6)
  int img = 0;
  // padded hidden width (the plan runs a real width dr < D in tiles of D, engine.cpp gnot_plan_create):
  // output column c with c % D >= dreal is written as 0 (the softmax of a head's features must not leak
  // into the pad columns, which the next kernels read as exact zeros); 0 = no pad columns
  int dreal = 0;
  // padded heads: heads of dh internal features of which the first dhr are real; the feature softmax
  // excludes (and writes 0 to) the others.  0: every feature of a head is real
  int dhr = 0;
  int ncol = 0;                      // store only output columns [0, ncol) (row pitch ldy < NO); 0 = all NO
  // the width of the output blocks dreal / dhr repeat in (the internal width); 0 = the kernel's K width D.
  // Set by launch_linear's K-split, whose kernels run at half the internal width
  int dblk = 0;
  int kcols[kMaxSeg] = {};           // per-segment input columns when they differ (K-split); 0 = K
};
// D: the K width the kernel is instantiated at (the internal width for the projections, a layer's input
// tiles x 16 for the chains).  D in (512, 1024] (a multiple of 128): the contraction runs as two K-halves of
// every segment on the D / 2 kernels -- X[s] + D / 2 for the second half and an image made of two half
// images (PackJob::kh), the second (NO / 16) x (D / 32) tiles after the first -- in launches of at most
// kMaxSeg segments (later ones accumulate; a softmax epilogue must fit one launch); a.K must then be D
hipError_t launch_linear(const LinearArgs& a, int D, hipStream_t s);
// output tiles per workgroup of linear.hip for an NO-column projection with a softmax epilogue over its
// first nsoft columns in heads of dh (-1: no tiling keeps whole heads per workgroup)
int linear_oc(int D, int NO, int nsoft, int dh);
// d = 256 projections on bf16x6 MFMA (linear2.hip): Wp[s] are OUTPUT-MAJOR x6 images (pack x6 = 2)
bool linear2_supported(const LinearArgs& a, int D);
hipError_t launch_linear2(const LinearArgs& a, hipStream_t s);
// jobs_dev: device array of independent LinearArgs (same D and NO), one per grid.z
hipError_t launch_linear_batch(const LinearArgs* jobs_dev, int njobs, int maxP, int NO, int D, int dh, hipStream_t s);

// ------------------------------------------------------------------ fused MLP chains (chain.hip)
enum ChainMode { CH_STORE = 0, CH_SOFTMAX = 1, CH_MOE = 2 };
// points per workgroup of the d = 256 chain kernels (chain2.hip: 16 per wave): one block of the soft-MoE
// expert grid
constexpr int kC2Rows = 128;
struct ChainLayer {
  const float4* Wp;    // packed forward weights of this layer
  const float4* WpT;   // packed transposed weights (backward)
  const float* bias;   // padded bias
};
struct ChainArgs {
  int D;               // hidden width
  int KT0, OTL;        // input / last-output tile counts (1 or D/16)
  int nlin;            // number of Linears (>= 2)
  int in_dim, out_dim;
  int P;
  int nchains;         // grid.y
  const ChainLayer* layers;          // device table [nchains * nlin]
  // d > 256 (chainw.hip, one Linear at a time): the same table in host memory and 2 * P * D floats of
  // scratch (the activations between two Linears)
  const ChainLayer* layers_host = nullptr;
  float* scratch = nullptr;
  // forward
  const float* X; long ldx;          // chain input (shared by all chains)
  float* Y; long ldy; long y_chain_stride;   // output (CH_STORE/CH_SOFTMAX) or MoE stage
  const float* scores; int ldsc;     // CH_MOE: expert weights scores[p*ldsc + chain]; CH_SOFTMAX bwd: s
  int mode;
  float* save; long save_layer_stride; long save_chain_stride;  // pre-activations [P, D] per layer (ld D)
  // backward
  const float* dY; long lddy;        // incoming grad (CH_STORE: [P,out]; CH_MOE: dquery [P,D]);
  float* dscore;                     // CH_MOE: dscore[p*ldsc + chain] += dq . y ; CH_SOFTMAX: d(scores)
  float* dz; long dz_layer_stride; long dz_chain_stride;          // per layer dZ [P, D] for wgrad
  float* dX; long lddx; long dx_chain_stride;                     // chain input grad or null
  int np = 3;                        // d = 256: operand pieces (3 = bf16x6 fp32-exact, 1 = bf16 mode)
#ifdef GNOT_DIAG_STAMP
  unsigned long long* dbg = nullptr;  // diagnostic builds: per-wave stamp sums (x6_core.h C2Pipe)
#endif
  int grid_mode = 0;                 // set by the launcher (chain2.hip c2_grid_pos)
  // CH_MOE, d = 256, np = 1 (bf16 mode): bf16 activation storage.  Saves and dZ are bf16 "pair-
  // interleaved" rows (gnot_common.h, 512 B per point; strides above then count 4-byte units, so a
  // [P, 256] bf16 layer is P * 128 of them).  Per chain, save slots 0 .. nlin-2 hold gelu'(h_l) of the
  // GELU layers (the backward's factor, computed with gelu(h_l) in the forward), slot nlin-1 the expert's
  // bf16 score-scaled term s y (the stage row the combine sums; the backward's d score = dq . (s y) / s),
  // slots nlin + l the RNE bf16 input of Linear l (= gelu(h_{l-1}), the
  // MFMA operand the forward used), written for the weight gradients; slot nlin + 0 (the shared MoE
  // input) only in chain 0.
  int b16s = 0;
  // b16s expert grid: the stage terms (forward s_e y_e, backward dX_e) go to the [E, P, d] stage as bf16
  // pair-interleaved rows (the strides are the fp32 stage's), summed by launch_moe_combine_b16
  int stage_b16 = 0;
};
// d <= 192 projections in the fp32 mode: bf16x6 on output-major 3-piece images (pack x6 = 2), as linear2.hip
// at d = 256 (round 5; exact fp32 MFMA on fp32 fragment images before -- the form d > 192 keeps).
// configs[1] (d = 128), one box, interleaved x2: 3.37 / 3.35 ms per step against 3.44 / 3.44 (profiles/r05o*)
constexpr bool kLinearX6 = true;
// d > 256: chains one Linear at a time (linear.hip + elementwise passes, chainw.hip)
hipError_t launch_chainw(const ChainArgs& a, bool bwd, hipStream_t s);
hipError_t launch_chain_fwd(const ChainArgs& a, hipStream_t s);
hipError_t launch_chain_bwd(const ChainArgs& a, hipStream_t s);
// d = 256 chains (chain2.hip): bf16x6 in both directions, output-major x6 images (pack x6 = 2) for Wp
// AND WpT
hipError_t launch_chain2(const ChainArgs& a, bool bwd, hipStream_t s);

// ------------------------------------------------------------------ point-reduction GEMM (wgrad.hip)
// C[out, in] = sum_p dz[p, :out]^T x[p, :in] over a point range, plus column sums of dz.
struct WgradJob {
  const float* dz; long lddz;        // A rows [P, out]
  const float* x;  long ldx;         // B rows [P, in]
  int x_gelu;                        // 1: B = gelu(x) (x is a saved pre-activation)
  int out, in;
  float* dW;                         // [out, in] row-major, or the state [H][dh*dh + dh] (state_dh > 0)
  float* db;                         // [out] column sums of A, or null
  const float* w; long ldw; int wdh; // optional per-(point, column/wdh) weight of the column sums
  int state_dh;                      // > 0: keep only dh x dh diagonal blocks, state layout
  int diag_only;                     // compute only the diagonal 128x128 tiles
  int P;
  int tiles_o, tiles_i;              // 128x128 output tiles
  int splits;                        // split-K count over points
  long slab_off;                     // offset (floats) of this job's partial slabs
  int accumulate;                    // 1: dW += result
};
// one workgroup per (job, tile, split); wg_prefix / red_prefix: per-job prefix sums of workgroups and
// of reduce elements (ntile * 128 * 129)
// x6: plain weight-gradient jobs only (no w, state_dh, diag_only) on the bf16x6 MFMA kernel
// wide: the same on the 256 x 256-tile kernel (out, in <= 256; ONE workgroup per (job, split), so
//       wg_prefix counts splits only)
// tw: the wide kernel's output edge, 256 (d = 256) or 128 (d <= 128: every job within 128 x 128)
// segs / seg_start (wide kernel only, optional): the balanced form -- workgroup w runs the point ranges
// segs[seg_start[w] .. seg_start[w+1]) = {job, slab slot, first point, end point}; each job's J.splits
// then counts the ranges that touch it (slots 0 .. splits-1)
hipError_t launch_wgrad(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                        const int* red_prefix_dev, int total_red, float* slab, hipStream_t s, bool x6 = false,
                        bool wide = false, int np = 3, int tw = 256,    // np: operand pieces (1 = bf16 mode)
                        const int4* segs = nullptr, const int* seg_start = nullptr);
// bf16-storage jobs (ChainArgs::b16s): dz and x point at bf16 pair-interleaved rows [P, 256] (x already
// the Linear's input, no GELU), out = in = 256, one workgroup per (job, split) as the wide kernel
hipError_t launch_wgrad_b16(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                            const int* red_prefix_dev, int total_red, float* slab, hipStream_t s,
                            const int4* segs = nullptr, const int* seg_start = nullptr);

// ------------------------------------------------------------------ attention states (state.hip)
// Jobs are WgradJobs with state_dh > 0: A = dz/lddz, B = x/ldx, optional w/ldw, out = dW as
// [H][dh*dh + dh], `splits` partials of state_pts(d) points each at slab + slab_off.
// Two kernels: state_mfma (fp32 MFMA, rows straight from HBM, dh = 16/32/64 with H % 4 == 0;
// below GNOT_STATE_MFMA_MIN points the VALU form) and the VALU state_partial (LDS-staged rows, any width).
// (the instantiated state_mfma_kernel<DH, HPW> forms, HPW = heads per wave = d / dh / 4: 1 / 2 / 4 at dh 16 and
// 32, 1 / 2 at 64; any other head count runs the VALU kernel -- round 6: 12 heads of 16 at d = 192 used to pass
// this test and fail the launch on meshes past GNOT_STATE_MFMA_MIN)
inline bool state_mfma_ok(int d, int dh) {
  if (!((dh == 16 || dh == 32 || dh == 64) && d % dh == 0 && (d / dh) % 4 == 0)) return false;
  const int hpw = d / dh / 4;
  return hpw == 1 || hpw == 2 || (hpw == 4 && dh <= 32);
}
// points per partial-state workgroup: 256 on MFMA (4 waves per SIMD at 262k points, partials ~6 % of
// the row bytes); VALU: the workgroup's A and B rows fill <= 32 KiB of LDS each (64 at d <= 128,
// 8192 / d above; measured: 32 and 16 are slower at cfg2)
inline int state_pts(bool mfma, int d) { return mfma ? 256 : d <= 128 ? 64 : 8192 / d; }
// MFMA only from this many points in the group (env GNOT_STATE_MFMA_MIN, read per plan): below it the
// 256-point MFMA workgroups leave most CUs idle and the 64-point VALU kernel is faster (configs[1],
// 10k points: 3.60 vs 3.94 ms per step)
inline long state_mfma_min_points() {
  const char* e = std::getenv("GNOT_STATE_MFMA_MIN");
  return e ? std::atol(e) : 65536;
}
hipError_t launch_state(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                        const int* red_prefix_dev, int total_red, float* slab, int d, int dh, int pts, int nw,
                        bool mfma, hipStream_t s);   // d: row width, pts: points per workgroup, nw: per-point
                                                     // weights (0 or H), mfma: state_mfma_kernel (state_mfma_ok)

// ------------------------------------------------------------------ attention (attn.hip)
struct AttnApplyArgs {
  const float* q; long ldq;          // post-softmax q, point-major
  int nsrc;                          // number of (S, z) sets to average (I, or 1 for self)
  const float* state[8];             // [B][H][dh*dh + dh] per source
  const int4* chunks; int nchunks;
  const long* off;                   // [B+1] sample offsets (device)
  int H, dh;
  float* res;                        // [P, d] head-major per sample (the scramble)
  // padded heads: the scramble holds heads of dhr real features (element (h, n, j) at (h N_b + n) dhr + j,
  // j < dhr), while q / states / du / dq run heads of dh (pad features zero).  0: dhr = dh
  int dhr = 0;
  // backward
  const float* dres;                 // [P, d] head-major per sample
  float* dq_pre; long lddq;          // grad wrt pre-softmax q, point-major
  float* du[8]; long lddu;           // per source du, point-major
  float* dden[8];                    // per source [P, H]
};
hipError_t launch_attn_apply_fwd(const AttnApplyArgs& a, hipStream_t s);
hipError_t launch_attn_apply_bwd(const AttnApplyArgs& a, hipStream_t s);
// fp32-MFMA variants (attn_mfma.hip, dh = 16/32/64); hipErrorNotSupported when not applicable
hipError_t launch_attn_apply_mfma(const AttnApplyArgs& a, bool bwd, hipStream_t s);

struct AttnKVBwdArgs {
  const float* k; const float* v; long ldkv;   // post-softmax k, v (point-major)
  const float* dstate;               // [B][H][dh*dh + dh]  (dS, dz)
  const int4* chunks; int nchunks;
  int H, dh;
  float* dk; float* dv; long lddkv;  // pre-softmax dK, dV
};
hipError_t launch_attn_kv_bwd(const AttnKVBwdArgs& a, hipStream_t s);
// independent K/V backward jobs (every block x input function) in one launch, job = grid.y
hipError_t launch_attn_kv_bwd_batch(const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks, int H, int dh,
                                    hipStream_t s);
// fp32-MFMA K/V backward (attn_mfma.hip): one job (a) or the batched jobs; hipErrorNotSupported
// when not applicable
hipError_t launch_attn_kv_bwd_mfma(const AttnKVBwdArgs* a, const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks,
                                   int H, int dh, hipStream_t s);

// ------------------------------------------------------------------ small elementwise (misc.hip)
hipError_t launch_concat_theta(const float* x, long ldx, int in_dim, const float* theta, int th_dim,
                               const long* off, int B, float* xin, long ldxin, int P, hipStream_t s);
// out = (base ? base : 0) + sum_e stage[e]
hipError_t launch_moe_combine(const float* base, const float* stage, long stage_stride, int E,
                              float* out, long n, hipStream_t s);
// the same over bf16 pair-interleaved stage rows (ChainArgs::stage_b16: 512 B per point at the start of each
// expert's fp32-sized region, stage_stride in floats); base / out fp32 [P, 256]
hipError_t launch_moe_combine_b16(const float* base, const float* stage, long stage_stride, int E, float* out,
                                  long P, hipStream_t s);
// out[r][c] = a[r][c] + b[r][c] (b null: a copy), c < cols, out dense [rows, cols]
hipError_t launch_add_cols(const float* a, long lda, const float* b, long ldb, int cols, float* out, long rows,
                           hipStream_t s);
// out[b][t] = sum over rows [off[b], off[b+1]) of a[row][c0 + t], t < ncols (fixed order)
hipError_t launch_seg_colsum(const float* a, long lda, int c0, int ncols, const long* off, int B, float* out,
                             hipStream_t s);
// segmented copy: dst[seg.dst + i] = src[seg.src + i], i < seg.len (floats); reverse swaps the roles of
// src/dst offsets.  unit 4: every offset and length a multiple of 4 (float4 copies), unit 1: any.  prefix:
// prefix sums of the lengths in units [nseg + 1], total = prefix[nseg].
struct CopySeg {
  long a, b, len;      // a = source offset, b = destination offset (forward direction)
};
hipError_t launch_segcopy(const CopySeg* segs, const int* prefix, int nseg, int total, const float* src, float* dst,
                          bool reverse, hipStream_t s, int unit = 4);

// ------------------------------------------------------------------ training step (train.hip)
int rel_l2_splits(const long* off_host, int B);
// work: B*nsplit*2C + B*C floats
hipError_t launch_rel_l2(const float* pred, const float* tgt, const long* off_dev, int B, int C, int nsplit,
                         long rows, float* work, float* loss, float* dpred, hipStream_t s);
hipError_t launch_adamw(float* param, const float* grad, float* m, float* v, long n, const float* hyper,
                        hipStream_t s);

}  // namespace gnot
