// Fused MLP chains (reference MLP, model.py:5-18) — forward and backward.
//
// One wave carries 16 points through ALL nl+1 Linears of one MLP with the activations resident in
// VGPRs (point form, gnot_common.h): Linear -> +bias -> exact-erf GELU -> next Linear ... The
// MFMA output of a layer is directly the B operand of the next one, so a chain touches HBM only
// for its input rows, its output rows and (training) the saved pre-activations.  grid.y selects
// the chain, which is how the E experts of a soft-MoE (model.py:123-137) run side by side on the
// same input; the three epilogues cover every MLP of GNOT:
//   CH_STORE   plain output (x / input-function encoders, decoder: model.py:146, 149, 152)
//   CH_SOFTMAX softmax over the outputs (gating over experts, model.py:148, 155-156)
//   CH_MOE     expert output scaled by its per-point gate weight into a per-expert stage
//              (model.py:128-130; the residual add + sum over experts is moe_combine / the consumer)
// The backward kernel walks the same chain in reverse with the transposed weight images,
// re-applying GELU'(saved pre-activation), and writes each layer's dZ for the weight-gradient pass.
#include <type_traits>

#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

// waves (16 points each) per workgroup; the workgroup shares one LDS weight stream.  Two waves give
// ~5 workgroups per CU at 10k-point meshes instead of 2-3 (less tail imbalance, better MFMA fill)
// for twice the L2->LDS weight traffic.
constexpr int kChainWaves = 4;

// 3 waves per SIMD (<= 168 VGPRs + AGPRs) at d <= 128: a 10k-point MoE launch (2,500 waves) is then
// ONE round on the 1,024 SIMDs instead of a full round plus a 20 % tail round at 2 waves per SIMD.
// NP: operand pieces, 3 = bf16x6 (fp32-exact, k-major x6 images, pack x6 = 1), 1 = the bf16 arithmetic
// mode (one RNE bf16 piece, pack x6 = 4)
template <int D, int KT0, int OTL, int NP>
__global__ void __launch_bounds__(64 * kChainWaves) __attribute__((amdgpu_waves_per_eu(D <= 128 ? 3 : 1)))
chain_fwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const long p = ((long)blockIdx.x * kChainWaves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int e = blockIdx.y;
  const int nl = a.nlin;
  const ChainLayer* L = a.layers + e * nl;
  float* save = a.save ? a.save + e * a.save_chain_stride : nullptr;
  __shared__ __attribute__((aligned(16))) float4 wlds[2 * x6_buf_f4(D)];
  int cnt = 0;
  // the weight stream: layer 0 | hidden layers | last layer, one chunk always in flight
  stage_image(wlds, L[0].Wp, x6_chunk_f4<D, NP>(KT0, DT), kChainWaves, wave, lane);
  auto next_f4 = [&](int l) { return (l == nl - 1) ? x6_chunk_f4<D, NP>(DT, OTL) : x6_chunk_f4<D, NP>(DT, DT); };

  float h[DT][4];
  {
    float x0[KT0][4];
    load_rows<KT0>(x0, a.X, a.ldx, p, valid, a.in_dim, lane);
    f32x4 acc[DT];
    init_bias<DT>(acc, L[0].bias, lane);
    mm_tiles_pipe_x6<D, KT0, DT, NP>(L[0].Wp, L[1].Wp, next_f4(1), wlds, cnt, x0, acc, kChainWaves, wave, lane);
    acc_to_regs<DT>(acc, h);
  }
  if (save) store_rows<DT>(h, save, D, p, valid, D, lane);
#pragma unroll
  for (int T = 0; T < DT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) h[T][r] = gelu(h[T][r]);

  for (int l = 1; l < nl - 1; ++l) {
    f32x4 acc[DT];
    init_bias<DT>(acc, L[l].bias, lane);
    mm_tiles_pipe_x6<D, DT, DT, NP>(L[l].Wp, L[l + 1].Wp, next_f4(l + 1), wlds, cnt, h, acc, kChainWaves, wave,
                                    lane);
    acc_to_regs<DT>(acc, h);
    if (save) store_rows<DT>(h, save + l * a.save_layer_stride, D, p, valid, D, lane);
#pragma unroll
    for (int T = 0; T < DT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) h[T][r] = gelu(h[T][r]);
  }

  float y[OTL][4];
  {
    f32x4 acc[OTL];
    init_bias<OTL>(acc, L[nl - 1].bias, lane);
    mm_tiles_pipe_x6<D, DT, OTL, NP>(L[nl - 1].Wp, nullptr, 0, wlds, cnt, h, acc, kChainWaves, wave, lane);
    acc_to_regs<OTL>(acc, y);
  }
  if (save) store_rows<OTL>(y, save + (nl - 1) * a.save_layer_stride, D, p, valid, 16 * OTL, lane);

  const int g = lane >> 4;
  if (a.mode == CH_SOFTMAX) {
    // softmax over the first out_dim outputs (features 16T + 4g + r); padded features excluded
    float m = -INFINITY;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 * T + 4 * g + r < a.out_dim) m = fmaxf(m, y[T][r]);
    m = fmaxf(m, shfl_xor(m, 16));
    m = fmaxf(m, shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool in = 16 * T + 4 * g + r < a.out_dim;
        y[T][r] = in ? __expf(y[T][r] - m) : 0.f;
        sum += y[T][r];
      }
    sum += shfl_xor(sum, 16);
    sum += shfl_xor(sum, 32);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[T][r] *= inv;
    store_rows<OTL>(y, a.Y + e * a.y_chain_stride, a.ldy, p, valid, a.out_dim, lane);
  } else if (a.mode == CH_MOE) {
    const float s = valid ? a.scores[p * a.ldsc + e] : 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[T][r] *= s;
    if (a.Y != nullptr)   // null: MoE recompute (the saves only)
      store_rows<OTL>(y, a.Y + e * a.y_chain_stride, a.ldy, p, valid, a.out_dim, lane);
  } else {
    store_rows<OTL>(y, a.Y + e * a.y_chain_stride, a.ldy, p, valid, a.out_dim, lane);
  }
}

// NP = 3: bf16x6 on k-major 3-piece images of W^T (pack x6 = 1), as the forward (round 5; the exact fp32
// MFMA on fp32 fragment images before); NP = 1 (bf16 mode): one RNE bf16 piece per operand on k-major
// one-piece images of W^T (pack x6 = 4), fp32 accumulation
// three waves per SIMD at d <= 128 (as the forward): 162-165 VGPRs without spills at d = 128, where the
// compiler's own choice (132 VGPRs + 48 AGPRs) allowed two, so a configs[1] launch (2,500 waves) ran in two
// rounds.  d = 112 would spill at three
template <int D, int KT0, int OTL, int NP>
__global__ void __launch_bounds__(64 * kChainWaves)
__attribute__((amdgpu_waves_per_eu((D <= 128 && D != 112) ? 3 : 1)))
chain_bwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int wave = threadIdx.x >> 6;
  const long p = ((long)blockIdx.x * kChainWaves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int e = blockIdx.y;
  const int nl = a.nlin;
  const ChainLayer* L = a.layers + e * nl;
  const float* save = a.save + e * a.save_chain_stride;
  float* dz = a.dz ? a.dz + e * a.dz_chain_stride : nullptr;
  // k-major NP-piece images of W^T on the bf16 MFMA
  __shared__ __attribute__((aligned(16))) float4 wlds[2 * x6_buf_f4(D)];
  int cnt = 0;
  // chunk of a KT-deep, OT-wide transposed image (NP-piece k-major blocks)
  auto cf4 = [](int KT, int OT) { return x6_chunk_f4<D, NP>(KT, OT); };
  // acc += W^T in over the KT-deep image Wg (the weight stream of the pipe of this arithmetic)
  float gr[DT][4];
  float hs[DT][4];
  // `late` (x6 / one-piece pipes): after the last weight chunk's barrier, before its MFMAs -- the saved
  // pre-activations loaded by `hook` have landed by then, and gelu'(h) evaluates beside the MFMAs instead of
  // as a VALU phase after them (bitwise the same values)
  auto mm = [&](auto KTc, auto OTc, const float4* Wg, const float4* nW, int nf4, const float (&in)[decltype(KTc)::value][4],
                f32x4 (&acc)[decltype(OTc)::value], auto hook, auto late) __attribute__((always_inline)) {
    constexpr int KT = decltype(KTc)::value, OT = decltype(OTc)::value;
    mm_tiles_pipe_x6<D, KT, OT, NP>(Wg, nW, nf4, wlds, cnt, in, acc, kChainWaves, wave, lane, hook, late);
  };
  // hs := gelu'(hs) in place (the factor of the next backward layer)
  auto ggrad = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int T = 0; T < DT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs[T][r] = gelu_grad(hs[T][r]);
  };
  using IOTL = std::integral_constant<int, OTL>;
  using IDT = std::integral_constant<int, DT>;
  using IKT0 = std::integral_constant<int, KT0>;
  // transposed-weight stream in reverse layer order: last | hidden (nl-2 .. 1) | first (if dX)
  stage_image(wlds, L[nl - 1].WpT, cf4(OTL, DT), kChainWaves, wave, lane);
  auto next_W = [&](int l) -> const float4* {      // the layer processed after layer l
    if (l - 1 >= 1) return L[l - 1].WpT;
    return a.dX ? L[0].WpT : nullptr;
  };
  auto next_f4 = [&](int l) { return (l - 1 >= 1) ? cf4(DT, DT) : cf4(DT, KT0); };

  // ---- gradient at the chain output
  float dy[OTL][4];
  if (a.mode == CH_MOE) {
    // query_out = query_in + sum_e s_e * y_e : dy_e = s_e * dq ; ds_e = dq . y_e (model.py:128-131)
    float yv[OTL][4];
    load_rows<OTL>(dy, a.dY, a.lddy, p, valid, 16 * OTL, lane);
    load_rows<OTL>(yv, save + (nl - 1) * a.save_layer_stride, D, p, valid, 16 * OTL, lane);
    float ds = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) ds += dy[T][r] * yv[T][r];
    ds += shfl_xor(ds, 16);
    ds += shfl_xor(ds, 32);
    const float s = valid ? a.scores[p * a.ldsc + e] : 0.f;
    if (valid && g == 0) a.dscore[p * a.ldsc + e] += ds;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dy[T][r] *= s;
  } else if (a.mode == CH_SOFTMAX) {
    // d logits = s * (ds - <s, ds>)   (softmax over experts, model.py:156)
    float sv[OTL][4];
    load_rows<OTL>(sv, a.scores, a.ldsc, p, valid, a.out_dim, lane);
    load_rows<OTL>(dy, a.dscore, a.ldsc, p, valid, a.out_dim, lane);
    float dot = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += sv[T][r] * dy[T][r];
    dot += shfl_xor(dot, 16);
    dot += shfl_xor(dot, 32);
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dy[T][r] = sv[T][r] * (dy[T][r] - dot);
  } else {
    load_rows<OTL>(dy, a.dY, a.lddy, p, valid, a.out_dim, lane);
  }

  // ---- last Linear; the saved pre-activation of Linear nl-2 is prefetched during its MFMAs
  if (dz) store_rows<OTL>(dy, dz + (nl - 1) * a.dz_layer_stride, D, p, valid, 16 * OTL, lane);
  {
    f32x4 acc[DT];
    init_bias<DT>(acc, nullptr, lane);
    auto pre = [&]() { load_rows<DT>(hs, save + (nl - 2) * a.save_layer_stride, D, p, valid, D, lane); };
    mm(IOTL{}, IDT{}, L[nl - 1].WpT, next_W(nl - 1), next_f4(nl - 1), dy, acc, pre, ggrad);
    acc_to_regs<DT>(acc, gr);
  }
  // ---- hidden Linears, reverse
  for (int l = nl - 2; l >= 1; --l) {
#pragma unroll
    for (int T = 0; T < DT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) gr[T][r] *= hs[T][r];     // hs = gelu'(h_l), evaluated during the MFMAs
    if (dz) store_rows<DT>(gr, dz + l * a.dz_layer_stride, D, p, valid, D, lane);
    f32x4 acc[DT];
    init_bias<DT>(acc, nullptr, lane);
    auto pre = [&]() { load_rows<DT>(hs, save + (l - 1) * a.save_layer_stride, D, p, valid, D, lane); };
    mm(IDT{}, IDT{}, L[l].WpT, next_W(l), next_f4(l), gr, acc, pre, ggrad);
    acc_to_regs<DT>(acc, gr);
  }
  // ---- first Linear (hs now holds gelu' of the saved pre-activation of Linear 0)
#pragma unroll
  for (int T = 0; T < DT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[T][r] *= hs[T][r];
  if (dz) store_rows<DT>(gr, dz, D, p, valid, D, lane);
  if (a.dX) {
    f32x4 acc[KT0];
    init_bias<KT0>(acc, nullptr, lane);
    mm(IDT{}, IKT0{}, L[0].WpT, nullptr, 0, gr, acc, NoHook(), NoHook());
    float dx[KT0][4];
    acc_to_regs<KT0>(acc, dx);
    store_rows<KT0>(dx, a.dX + e * a.dx_chain_stride, a.lddx, p, valid, a.in_dim, lane);
  }
}

template <int D, int NP>
static hipError_t launch_chain_np(const ChainArgs& a, bool bwd, hipStream_t s) {
  constexpr int DT = D / 16;
  const dim3 grid((a.P + 16 * kChainWaves - 1) / (16 * kChainWaves), a.nchains), block(64 * kChainWaves);
#define GNOT_CHAIN_CASE(K0, OL)                                                              \
  if (a.KT0 == K0 && a.OTL == OL) {                                                           \
    if (bwd) hipLaunchKernelGGL((chain_bwd_kernel<D, K0, OL, NP>), grid, block, 0, s, a);      \
    else hipLaunchKernelGGL((chain_fwd_kernel<D, K0, OL, NP>), grid, block, 0, s, a);          \
    return hipGetLastError();                                                                 \
  }
  GNOT_CHAIN_CASE(1, 1)
  GNOT_CHAIN_CASE(1, DT)
  GNOT_CHAIN_CASE(DT, 1)
  GNOT_CHAIN_CASE(DT, DT)
#undef GNOT_CHAIN_CASE
  return hipErrorInvalidValue;
}
template <int D>
static hipError_t launch_chain_d(const ChainArgs& a, bool bwd, hipStream_t s) {
  return a.np == 1 ? launch_chain_np<D, 1>(a, bwd, s) : launch_chain_np<D, 3>(a, bwd, s);
}

static hipError_t launch_chain(const ChainArgs& a, bool bwd, hipStream_t s) {
  if (a.P <= 0 || a.nchains <= 0) return hipSuccess;
  if (a.nlin < 2) return hipErrorInvalidValue;
  switch (a.D) {
    case 16: return launch_chain_d<16>(a, bwd, s);
    case 32: return launch_chain_d<32>(a, bwd, s);
    case 48: return launch_chain_d<48>(a, bwd, s);
    case 64: return launch_chain_d<64>(a, bwd, s);
    case 80: return launch_chain_d<80>(a, bwd, s);
    case 96: return launch_chain_d<96>(a, bwd, s);
    case 112: return launch_chain_d<112>(a, bwd, s);
    case 128: return launch_chain_d<128>(a, bwd, s);
    case 144: return launch_chain_d<144>(a, bwd, s);
    case 160: return launch_chain_d<160>(a, bwd, s);
    case 176: return launch_chain_d<176>(a, bwd, s);
    case 192: return launch_chain_d<192>(a, bwd, s);
    default: return hipErrorInvalidValue;
  }
}

// d = 256 runs on chain2.hip (output-major bf16x6 in both directions; the engine packs its images)
hipError_t launch_chain_fwd(const ChainArgs& a, hipStream_t s) {
  return a.D > 256 ? launch_chainw(a, false, s) : a.D == 256 ? launch_chain2(a, false, s) : launch_chain(a, false, s);
}
hipError_t launch_chain_bwd(const ChainArgs& a, hipStream_t s) {
  return a.D > 256 ? launch_chainw(a, true, s) : a.D == 256 ? launch_chain2(a, true, s) : launch_chain(a, true, s);
}

}  // namespace gnot
