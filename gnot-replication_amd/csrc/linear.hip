// Projection kernel: Y[p, :NO] (=|+=) epi( sum_s X_s[p, :K] . A + bias )
//
// Used for the attention projections (reference model.py:56, 67-68, 89-90: query/key/value, with
// the feature softmax of model.py:59/72/93 fused into the epilogue), fc_out (model.py:106) and every
// backward-data product dX = dY W of those Linears.  One wave = 16 points held in point form
// (gnot_common.h), the input row block is loaded ONCE and reused for all NO output columns; the
// A operand is the packed weight image streamed from L2 (one 1 KiB load per 4 MFMAs).
// The input may be a sum of `nsum` equally strided buffers (the per-expert dX stage of the MoE
// backward), and the contraction may run over several K-segments with their own input rows and
// weight images (backward-data of the q/k/v projections: dX = dQ Wq + dK Wk + dV Wv in one pass).
// A batched variant runs independent jobs (e.g. the key/value projections of every block and
// input function) in one launch.
#include <algorithm>
#include <cstdlib>

#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

// NP-piece forms (round 5): the images are OUTPUT-MAJOR bf16 pieces (pack x6 = 3 for one RNE piece, the
// bf16 arithmetic mode; x6 = 2 for the exact three-piece split of the fp32 mode, kLinearX6, as linear2.hip's): block (o, kb) = 16 outputs x 32 contraction slots, piece q at Wg[((o * KB + kb) * NP + q) *
// 64 + lane], so a workgroup's OC output tiles are one contiguous run of OC * KB blocks.  Chunks of OCH tiles
// (OCH * KB * NP KiB <= the buffer) stream through two LDS buffers; the input is split once per segment (bp,
// NP 16x16x32 B operands per k-block); per block one v_mfma_f32_16x16x32_bf16 (NP = 1) or the six order <= 2
// piece products (NP = 3, smallest first)
template <int NP>
constexpr int bx_buf_kb() { return NP == 1 ? kChunkKB : 24; }
template <int NP>
constexpr int bx_och(int KB, int OC) {
  int c = OC;
  while (c > 1 && (c * KB * NP > bx_buf_kb<NP>() || OC % c != 0)) --c;
  return c;
}
template <int NP>
constexpr int bx_chunk_f4(int KB, int OC) { return bx_och<NP>(KB, OC) * KB * NP * WAVE; }
template <int KB, int OC, int NP, typename Hook = NoHook>
GNOT_DEV void mm_tiles_pipe_bx(const float4* __restrict__ Wg, const float4* __restrict__ next_W, int next_f4,
                               float4* lds, int& cnt, const u32x4 (&bp)[KB][NP], f32x4 (&acc)[OC], int nwaves,
                               int wave, int lane, Hook hook = Hook()) {
  constexpr int OCH = bx_och<NP>(KB, OC);
  constexpr int NC = OC / OCH;
  constexpr int CH4 = OCH * KB * NP * WAVE;
  constexpr int BUF4 = bx_buf_kb<NP>() * WAVE;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    lds_dma_wait();                                    // this chunk's DMA (issued one chunk ago) has landed
    __syncthreads();
    float4* nb = lds + ((cnt + 1) & 1) * BUF4;
    if (c + 1 < NC) stage_image(nb, Wg + (c + 1) * CH4, CH4, nwaves, wave, lane);
    else if (next_W) stage_image(nb, next_W, next_f4, nwaves, wave, lane);
    if (c == 0) hook();
    const u32x4* cb = reinterpret_cast<const u32x4*>(lds + (cnt & 1) * BUF4);
#pragma unroll
    for (int o = 0; o < OCH; ++o) {
      f32x4 r = acc[c * OCH + o];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const u32x4* blk = cb + (o * KB + kb) * NP * WAVE + lane;
        if constexpr (NP == 3) {
          r = mfma_bf16(blk[2 * WAVE], bp[kb][0], r);
          r = mfma_bf16(blk[WAVE], bp[kb][1], r);
          r = mfma_bf16(blk[0], bp[kb][2], r);
          r = mfma_bf16(blk[WAVE], bp[kb][0], r);
          r = mfma_bf16(blk[0], bp[kb][1], r);
        }
        r = mfma_bf16(blk[0], bp[kb][0], r);
      }
      acc[c * OCH + o] = r;
    }
    ++cnt;
  }
}

// NP: 0 = fp32 fragment images on the exact fp32 MFMA; 1 / 3 = the output-major bf16-piece forms above
template <int D, int OC, int NP = 0>   // OC: output tiles per workgroup (grid.y splits NO)
GNOT_DEV void linear_body(const LinearArgs& a, float4* wlds) {
  constexpr int KT = D / 16, KB = (KT + 1) / 2;
  constexpr bool B1 = NP > 0;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const long p = ((long)blockIdx.x * 4 + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int c = blockIdx.y;                       // output chunk of this workgroup
  // chunk offset inside every segment's image (fp32 tiles of KT x 1 KiB, or KB one-piece blocks per tile)
  const long wchunk = (long)c * OC * (B1 ? KB * NP : KT) * WAVE;
  const int cf4 = B1 ? bx_chunk_f4<B1 ? NP : 1>(KB, OC) : chunk_f4(KT, OC);
  int cnt = 0;
  stage_image(wlds, a.Wp[0] + wchunk, cf4, 4, wave, lane);

  auto kcol = [&](int sg) { return a.kcols[sg] > 0 ? a.kcols[sg] : a.K; };
  // segment 0 input (optionally the sum of nsum equally strided buffers)
  float in[KT][4];
  load_rows<KT>(in, a.X[0], a.ldx, p, valid, kcol(0), lane);
  for (int s = 1; s < a.nsum; ++s) {
    float t[KT][4];
    load_rows<KT>(t, a.X[0] + s * a.sum_stride, a.ldx, p, valid, kcol(0), lane);
#pragma unroll
    for (int T = 0; T < KT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) in[T][r] += t[T][r];
  }

  f32x4 acc[OC];
  init_bias<OC>(acc, a.bias ? a.bias + c * 16 * OC : nullptr, lane);
  // K-segments: acc += X_s W_s for s < nseg; segment s+1's rows are fetched during segment s's MFMAs
  for (int sg = 0; sg < a.nseg; ++sg) {
    const bool more = sg + 1 < a.nseg;
    float nx[KT][4];
    auto pre = [&]() {
      if (more) load_rows<KT>(nx, a.X[sg + 1], a.ldx, p, valid, kcol(sg + 1), lane);
    };
    if constexpr (B1) {
      u32x4 bp[KB][NP];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) split_block_x6<KT, NP>(in, kb, bp[kb]);
      mm_tiles_pipe_bx<KB, OC, NP>(a.Wp[sg] + wchunk, more ? a.Wp[sg + 1] + wchunk : nullptr, cf4, wlds, cnt, bp, acc,
                                   4, wave, lane, pre);
    } else {
      mm_tiles_pipe<KT, OC>(a.Wp[sg] + wchunk, more ? a.Wp[sg + 1] + wchunk : nullptr, cf4, wlds, cnt, in, acc, 4,
                            wave, lane, pre);
    }
    if (more) {
#pragma unroll
      for (int T = 0; T < KT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) in[T][r] = nx[T][r];
    }
  }
  float h[OC][4];
  acc_to_regs<OC>(acc, h);
  const int DB = a.dblk > 0 ? a.dblk : D;          // the width of the output blocks (pad columns, heads)
  if (c * 16 * OC < a.nsoft) {
    if (a.dhr > 0) {
      // padded heads: the pad features of every head (j >= dhr) take no part in its softmax (exp -> 0)
#pragma unroll
      for (int T = 0; T < OC; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if ((c * 16 * OC + 16 * T + 4 * (lane >> 4) + r) % DB % a.dh >= a.dhr) h[T][r] = -INFINITY;
    }
    softmax_heads<OC>(h, a.dh, lane >> 4);
  }
  if (a.dreal > 0) {
    // pad columns of a padded width (D is the tile width; features dreal .. D-1 of each D-block)
#pragma unroll
    for (int T = 0; T < OC; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((c * 16 * OC + 16 * T + 4 * (lane >> 4) + r) % DB >= a.dreal) h[T][r] = 0.f;
  }
  const int ncols = a.ncol > 0 ? min(16 * OC, a.ncol - c * 16 * OC) : 16 * OC;
  if (ncols <= 0) return;
  float* Y = a.Y + c * 16 * OC;
  if (a.epi == EPI_ACCUM) {
    float old[OC][4];
    load_rows<OC>(old, Y, a.ldy, p, valid, ncols, lane);
#pragma unroll
    for (int T = 0; T < OC; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) h[T][r] += old[T][r];
  }
  store_rows<OC>(h, Y, a.ldy, p, valid, ncols, lane);
}

template <int D, int OC, int NP = 0>
__global__ void __launch_bounds__(256) linear_kernel(LinearArgs a) {
  __shared__ __attribute__((aligned(16))) float4 wlds[2 * (NP == 3 ? bx_buf_kb<3>() * WAVE : pipe_buf_f4<D / 16>())];
  linear_body<D, OC, NP>(a, wlds);
}

// several independent projections in one launch: job = blockIdx.z (jobs live in device memory)
template <int D, int OC>
__global__ void __launch_bounds__(256) linear_batch_kernel(const LinearArgs* __restrict__ jobs) {
  __shared__ __attribute__((aligned(16))) float4 wlds[2 * pipe_buf_f4<D / 16>()];
  const LinearArgs a = jobs[blockIdx.z];
  if ((long)blockIdx.x * 64 >= a.P) return;        // whole workgroup: no barrier is skipped unevenly
  linear_body<D, OC>(a, wlds);
}

// Output tiles per workgroup.  Fewer tiles per wave means more waves per launch (a 10k-point d=128
// projection is ~1,250 waves at 4 tiles, 2,500 at 2), but the input rows are re-read once per chunk
// and the extra waves compete with the side-stream weight-gradient GEMMs: measured at cfg2, 4 tiles
// 3.57 ms/step, 8 tiles 3.74, 2 tiles 3.75, 1 tile 4.00.
// Chunks of a softmax epilogue must hold whole heads (16 * oc a multiple of dh): oc = D / 16 (the whole
// row) always does, so every (D, dh) the plan accepts has a valid choice (e.g. d = 144 with 4 heads of
// 36: the divisors 1 and 3 of 9 tiles split a head, 9 does not).  GNOT_LINEAR_OC overrides the choice
// (experiments); a choice that does not tile D and NO, or would split a head, falls back to the widest
// valid one; -1 when none exists (the launch then fails instead of skipping the softmax).
int linear_oc(int D, int NO, int nsoft, int dh) {
  static const int env = [] {
    const char* e = getenv("GNOT_LINEAR_OC");
    return e ? atoi(e) : 0;
  }();
  const int kt = D / 16;
  auto ok = [&](int oc) {
    // the whole row (oc == kt) always keeps whole heads, also at a padded width (D % dh != 0: the heads
    // tile the first dr features, the pad columns after them are zeroed, LinearArgs::dreal)
    return oc >= 1 && (oc <= 8 || oc == kt) && kt % oc == 0 && NO % (16 * oc) == 0 &&
           (nsoft == 0 || (16 * oc) % dh == 0 || oc == kt);
  };
  int want = env > 0 ? env : 4;
  if (ok(want)) return want;
  for (int oc = kt; oc >= 1; --oc)
    if (ok(oc)) return oc;
  return -1;
}

// every (D, oc) linear_oc can return: oc a divisor of D / 16 (<= 8, or D / 16 itself: the whole row, which
// keeps any head in one workgroup -- d = 256's batched input-function K / V with one head of 256, the d > 256
// projections with heads that do not divide 64)
#define GNOT_LIN_CASES                                                                                  \
  GNOT_LIN(16, 1) GNOT_LIN(32, 1) GNOT_LIN(32, 2) GNOT_LIN(48, 1) GNOT_LIN(48, 3) GNOT_LIN(64, 1)         \
  GNOT_LIN(64, 2) GNOT_LIN(64, 4) GNOT_LIN(80, 1) GNOT_LIN(80, 5) GNOT_LIN(96, 1) GNOT_LIN(96, 2)         \
  GNOT_LIN(96, 3) GNOT_LIN(96, 6) GNOT_LIN(112, 1) GNOT_LIN(112, 7) GNOT_LIN(128, 1) GNOT_LIN(128, 2)     \
  GNOT_LIN(128, 4) GNOT_LIN(128, 8) GNOT_LIN(144, 1) GNOT_LIN(144, 3) GNOT_LIN(144, 9) GNOT_LIN(160, 1)   \
  GNOT_LIN(160, 2) GNOT_LIN(160, 5) GNOT_LIN(160, 10) GNOT_LIN(176, 1) GNOT_LIN(176, 11) GNOT_LIN(192, 1) \
  GNOT_LIN(192, 2) GNOT_LIN(192, 3) GNOT_LIN(192, 4) GNOT_LIN(192, 6) GNOT_LIN(192, 12) GNOT_LIN(256, 1)  \
  GNOT_LIN(256, 2) GNOT_LIN(256, 4) GNOT_LIN(256, 8) GNOT_LIN(256, 16) GNOT_LIN(320, 1) GNOT_LIN(320, 2) GNOT_LIN(320, 4)   \
  GNOT_LIN(384, 1) GNOT_LIN(384, 2) GNOT_LIN(384, 4) GNOT_LIN(448, 1) GNOT_LIN(448, 2) GNOT_LIN(448, 4)   \
  GNOT_LIN(512, 1) GNOT_LIN(512, 2) GNOT_LIN(512, 4) GNOT_LIN(320, 20) GNOT_LIN(384, 24) GNOT_LIN(448, 28) \
  GNOT_LIN(512, 32)
// the d <= 192 cases of GNOT_LIN_CASES (the bf16 mode's one-piece kernels)
#define GNOT_LIN_B1_CASES                                                                                         \
  GNOT_LIN_B1(16, 1) GNOT_LIN_B1(32, 1) GNOT_LIN_B1(32, 2) GNOT_LIN_B1(48, 1) GNOT_LIN_B1(48, 3) GNOT_LIN_B1(64, 1)   \
  GNOT_LIN_B1(64, 2) GNOT_LIN_B1(64, 4) GNOT_LIN_B1(80, 1) GNOT_LIN_B1(80, 5) GNOT_LIN_B1(96, 1) GNOT_LIN_B1(96, 2)   \
  GNOT_LIN_B1(96, 3) GNOT_LIN_B1(96, 6) GNOT_LIN_B1(112, 1) GNOT_LIN_B1(112, 7) GNOT_LIN_B1(128, 1)                   \
  GNOT_LIN_B1(128, 2) GNOT_LIN_B1(128, 4) GNOT_LIN_B1(128, 8) GNOT_LIN_B1(144, 1) GNOT_LIN_B1(144, 3)                  \
  GNOT_LIN_B1(144, 9) GNOT_LIN_B1(160, 1) GNOT_LIN_B1(160, 2) GNOT_LIN_B1(160, 5) GNOT_LIN_B1(160, 10)                \
  GNOT_LIN_B1(176, 1) GNOT_LIN_B1(176, 11) GNOT_LIN_B1(192, 1) GNOT_LIN_B1(192, 2) GNOT_LIN_B1(192, 3)                 \
  GNOT_LIN_B1(192, 4) GNOT_LIN_B1(192, 6) GNOT_LIN_B1(192, 12)

// internal widths above 512: every segment's contraction in two halves on the D / 2 kernels (see gnot_kernels.h)
static hipError_t launch_linear_ksplit(const LinearArgs& a, int D, hipStream_t s) {
  const int Kh = D / 2;
  // a.K <= D / 2 (an input narrower than the internal width, e.g. a chain's first layer): the first halves only;
  // otherwise the second halves take the K - D / 2 columns past the first (the real width of a padded input)
  const int halves = a.K <= Kh ? 1 : 2;
  if (D > 1024 || D % 128 != 0 || a.K > D || a.nsum != 1 || a.NO % 16 != 0) return hipErrorInvalidValue;
  for (int sg = 0; sg < a.nseg; ++sg)
    if (a.kcols[sg] > 0) return hipErrorInvalidValue;     // already split
  const long half4 = (long)(a.NO / 16) * (Kh / 16) * WAVE;   // the second half image, in float4
  const int nseg2 = halves * a.nseg;
  if (a.nsoft > 0 && nseg2 > kMaxSeg) return hipErrorInvalidValue;   // a softmax needs the whole sum at once
  for (int s0 = 0; s0 < nseg2; s0 += kMaxSeg) {
    LinearArgs b = a;
    b.nseg = std::min(kMaxSeg, nseg2 - s0);
    for (int k = 0; k < b.nseg; ++k) {
      const int sg = (s0 + k) / halves, h = (s0 + k) % halves;
      b.X[k] = a.X[sg] + h * Kh;
      b.Wp[k] = a.Wp[sg] + h * half4;
      b.kcols[k] = h == 0 ? std::min(a.K, Kh) : a.K - Kh;
    }
    for (int k = b.nseg; k < kMaxSeg; ++k) b.kcols[k] = 0;
    b.K = std::min(a.K, Kh);
    b.dblk = a.dblk > 0 ? a.dblk : D;
    if (s0 > 0) { b.epi = EPI_ACCUM; b.bias = nullptr; }
    const hipError_t r = launch_linear(b, Kh, s);
    if (r != hipSuccess) return r;
  }
  return hipSuccess;
}

hipError_t launch_linear(const LinearArgs& a, int D, hipStream_t s) {
  if (a.P <= 0) return hipSuccess;
  if (a.nseg < 1 || a.nseg > kMaxSeg) return hipErrorInvalidValue;
  if (D > 512) return launch_linear_ksplit(a, D, s);
  const int oc = linear_oc(D, a.NO, a.nsoft, a.dh);
  const dim3 grid((a.P + 63) / 64, a.NO / (16 * oc)), block(256);
#define GNOT_LIN(DD, OO) \
  if (D == DD && oc == OO) { hipLaunchKernelGGL((linear_kernel<DD, OO>), grid, block, 0, s, a); return hipGetLastError(); }
  // d <= 192 on output-major bf16-piece images (LinearArgs::img): the bf16 mode (1) and the fp32 mode's bf16x6
  // (3, kLinearX6); the d = 256 projections are linear2.hip's
#define GNOT_LIN_B1(DD, OO)                                                                              \
  if (D == DD && oc == OO) {                                                                              \
    if (a.img == 1) hipLaunchKernelGGL((linear_kernel<DD, OO, 1>), grid, block, 0, s, a);                 \
    else hipLaunchKernelGGL((linear_kernel<DD, OO, 3>), grid, block, 0, s, a);                            \
    return hipGetLastError();                                                                             \
  }
  if (a.img == 1 || a.img == 3) {
    if (D > 192) return hipErrorInvalidValue;
    GNOT_LIN_B1_CASES
    return hipErrorInvalidValue;
  }
  GNOT_LIN_CASES
#undef GNOT_LIN
#undef GNOT_LIN_B1
  return hipErrorInvalidValue;
}

// jobs may carry a softmax epilogue: the tile choice keeps whole heads (dh) in one workgroup
hipError_t launch_linear_batch(const LinearArgs* jobs_dev, int njobs, int maxP, int NO, int D, int dh, hipStream_t s) {
  if (njobs <= 0 || maxP <= 0) return hipSuccess;
  const int oc = linear_oc(D, NO, 1, dh);
  const dim3 grid((maxP + 63) / 64, NO / (16 * oc), njobs), block(256);
#define GNOT_LIN(DD, OO)                                                                     \
  if (D == DD && oc == OO) {                                                                 \
    hipLaunchKernelGGL((linear_batch_kernel<DD, OO>), grid, block, 0, s, jobs_dev);          \
    return hipGetLastError();                                                                \
  }
  GNOT_LIN_CASES
#undef GNOT_LIN
  return hipErrorInvalidValue;
}

}  // namespace gnot
