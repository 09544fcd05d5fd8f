// Fused MLP chains for hidden width d >= 128 (reference MLP, model.py:5-18): forward and backward on
// bf16x6 MFMA, OUTPUT-MAJOR.
//
// Same point form as chain.hip (a wave carries 16 points through all nl+1 Linears with the
// activations in registers; grid.y = chain, e.g. the E experts of a soft-MoE), but the layer is
// computed one 16-feature OUTPUT tile at a time instead of one input block at a time:
//   * the layer input is held as its exact three-piece bf16 split (gnot_common.h split8_x6), 12
//     registers per 32-feature k-block, so every output tile is 6 x KB v_mfma_f32_16x16x32_bf16 with
//     nothing but the weight pieces read from LDS;
//   * a tile's result is final as soon as its MFMAs retire: bias, save store, GELU (forward) or
//     GELU'(saved pre-activation) and the dZ store (backward) of tile o run beside the MFMAs of tile
//     o+1, instead of a whole-layer VALU burst between two MFMA phases;
//   * the next layer's input accumulates as fp32 (4 registers per tile) and is split once per layer.
// 8 waves (128 points) share one weight stream: one LDS chunk = one output tile's image (KB k-blocks
// x 3 pieces x 1 KiB, output-major pack, pack.hip x6 = 2), double-buffered, the next chunk's DMA
// (next tile, or the next layer's first tile) issued one chunk ahead.  <= 256 registers: two waves per
// SIMD, so one wave's epilogue VALU runs beside its partner's MFMAs.
//   forward : h_l = W_l a_l + b_l, a_{l+1} = gelu(h_l); saves h_l (training); epilogue of the last
//             layer: CH_STORE / CH_SOFTMAX (gating) / CH_MOE (score-scaled expert output)
//   backward: dz_{nl-1} = dy (x score for CH_MOE), g_l = W_l^T dz_l, dz_{l-1} = g_l * gelu'(h_{l-1});
//             writes every dz_l (weight gradients, wgrad.hip) and optionally dX = W_0^T dz_0.
#include "gnot_kernels.h"
#include "x6_core.h"

namespace gnot {

// ------------------------------------------------------------------------------------------ forward
// one forward layer: OT output tiles h = W a + b; saves h (if sv) and returns gelu(h) (GELU) or h in out.
// The epilogue of tile o-1 follows the MFMAs of tile o in program order (independent work the
// scheduler can place between them).
template <int OT, int KBI, bool GELU = true>
GNOT_DEV void c2_fwd_layer(C2Stream& st, const u32x4* W, const u32x4 (&in)[KBI][3], const float* bias, const float* sv,
                           unsigned sv_bytes, int voff, const u32x4* nextW, int next_u4, int g, int lane,
                           float (&out)[OT][4]) {
  // saved pre-activations through a buffer resource: base + bound in SGPRs, the lane's row offset in
  // one VGPR, the tile in the immediate; tail lanes (rows past P) fall outside the bound and are dropped
  const rsrc_t rs = make_rsrc(sv, sv ? sv_bytes : 0u);
  float4 bn = ld4(bias + 4 * g);
  f32x4 prev;
  auto epi = [&](int o, const f32x4& acc) {
    if (sv) buf_store_f32x4(make_float4(acc[0], acc[1], acc[2], acc[3]), rs, voff + 64 * o, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) out[o][r] = GELU ? gelu(acc[r]) : acc[r];
    pin4(out[o]);
  };
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    const float4 bb = bn;
    if (o + 1 < OT) bn = ld4(bias + 16 * (o + 1) + 4 * g);
    const u32x4* cb = st.begin(W, o, OT, c2_tile_u4(KBI), nextW, next_u4);
    const f32x4 acc = c2_tile<KBI, true>(cb, in, f32x4{bb.x, bb.y, bb.z, bb.w}, lane);
    if (o > 0) epi(o - 1, prev);
    prev = acc;
  }
  epi(OT - 1, prev);
}

template <int D, int KT0, int OTL>
__global__ void __launch_bounds__(64 * kC2Waves) chain2_fwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16, KB = DT / 2, KB0 = (KT0 + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const long p = ((long)blockIdx.x * kC2Waves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int e = blockIdx.y, nl = a.nlin;
  const ChainLayer* L = a.layers + e * nl;
  float* save = a.save ? a.save + e * a.save_chain_stride : nullptr;
  const unsigned lay_bytes = (unsigned)min((long)a.P * D * 4, 0xFFFFFFFFL);   // one [P, D] layer
  const int voff = (int)((blockIdx.x * kC2Waves + wave) * 16 + (lane & 15)) * D * 4 + 16 * g;
  const u32x4* W0 = reinterpret_cast<const u32x4*>(L[0].Wp);
  C2Stream st{c2lds, c2_tile_u4(KB), 0, wave, lane};
  stage_image(reinterpret_cast<float4*>(c2lds), reinterpret_cast<const float4*>(W0), c2_tile_u4(KB0), kC2Waves, wave,
              lane);

  float nx[DT][4];                                   // next layer input (fp32), then split
  u32x4 bp[KB][3];
  // ---- layer 0 (input: KT0 tiles of the chain input)
  {
    float x0[KT0][4];
    load_rows<KT0>(x0, a.X, a.ldx, p, valid, a.in_dim, lane);
    u32x4 b0[KB0][3];
    c2_split<KT0>(x0, b0);
    const float* bias = L[0].bias;
    const u32x4* nextW = reinterpret_cast<const u32x4*>(nl > 1 ? L[1].Wp : nullptr);
    const int next_u4 = c2_tile_u4(KB);
    c2_fwd_layer<DT, KB0>(st, W0, b0, bias, save, lay_bytes, voff, nextW, next_u4, g, lane, nx);
  }
  // ---- hidden layers 1 .. nl-2
  for (int l = 1; l < nl - 1; ++l) {
    c2_split<DT>(nx, bp);
    const u32x4* Wl = reinterpret_cast<const u32x4*>(L[l].Wp);
    const u32x4* nextW = reinterpret_cast<const u32x4*>(L[l + 1].Wp);
    const float* bias = L[l].bias;
    float* sv = save ? save + l * a.save_layer_stride : nullptr;
    c2_fwd_layer<DT, KB>(st, Wl, bp, bias, sv, lay_bytes, voff, nextW, c2_tile_u4(KB), g, lane, nx);
  }
  // ---- last layer (OTL output tiles)
  float y[OTL][4];
  {
    c2_split<DT>(nx, bp);
    const u32x4* Wl = reinterpret_cast<const u32x4*>(L[nl - 1].Wp);
    const float* bias = L[nl - 1].bias;
    float* sv = save ? save + (nl - 1) * a.save_layer_stride : nullptr;
    c2_fwd_layer<OTL, KB, false>(st, Wl, bp, bias, sv, lay_bytes, voff, nullptr, 0, g, lane, y);
  }
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
  } else if (a.mode == CH_MOE) {
    const float s = valid ? a.scores[p * a.ldsc + e] : 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[T][r] *= s;
  }
  store_rows<OTL>(y, a.Y + e * a.y_chain_stride, a.ldy, p, valid, a.out_dim, lane);
}

// ------------------------------------------------------------------------------------------ backward
template <int D, int KT0, int OTL>
__global__ void __launch_bounds__(64 * kC2Waves) chain2_bwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16, KB = DT / 2, KBL = (OTL + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const long p = ((long)blockIdx.x * kC2Waves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int e = blockIdx.y, nl = a.nlin;
  const ChainLayer* L = a.layers + e * nl;
  const float* save = a.save + e * a.save_chain_stride;
  float* dz = a.dz ? a.dz + e * a.dz_chain_stride : nullptr;
  const u32x4* WL = reinterpret_cast<const u32x4*>(L[nl - 1].WpT);
  C2Stream st{c2lds, c2_tile_u4(KB), 0, wave, lane};
  stage_image(reinterpret_cast<float4*>(c2lds), reinterpret_cast<const float4*>(WL), c2_tile_u4(KBL), kC2Waves, wave,
              lane);

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
  if (dz) store_rows<OTL>(dy, dz + (nl - 1) * a.dz_layer_stride, D, p, valid, 16 * OTL, lane);

  float nx[DT][4];
  u32x4 bp[KB][3];
  // one backward layer: g = W_l^T dz_l (DT output tiles), dz_{l-1} = g * gelu'(h_{l-1}) stored and kept
  // in nx; the saved pre-activation tile of o+1 is loaded while tile o's MFMAs run
  const unsigned lay_bytes = (unsigned)min((long)a.P * D * 4, 0xFFFFFFFFL);   // one [P, D] layer
  const int voff = (int)((blockIdx.x * kC2Waves + wave) * 16 + (lane & 15)) * D * 4 + 16 * g;
  auto layer = [&](const u32x4* Wt, const auto& in, int l, const u32x4* nextW, int next_u4) {
    constexpr int KBI = std::extent<std::remove_reference_t<decltype(in)>>::value;
    // saved pre-activation h_{l-1} (read, one tile ahead) and dz_{l-1} (written) through buffer
    // resources: rows past P read 0 / are dropped
    const rsrc_t rh = make_rsrc(save + (l - 1) * a.save_layer_stride, lay_bytes);
    const rsrc_t rz = make_rsrc(dz ? dz + (l - 1) * a.dz_layer_stride : nullptr, dz ? lay_bytes : 0u);
    float4 hn = buf_load_f32x4(rh, voff, 0);
    f32x4 prev;
    float4 hp;
    auto epi = [&](int o, const f32x4& acc, const float4& hc) {
      nx[o][0] = acc[0] * gelu_grad(hc.x);
      nx[o][1] = acc[1] * gelu_grad(hc.y);
      nx[o][2] = acc[2] * gelu_grad(hc.z);
      nx[o][3] = acc[3] * gelu_grad(hc.w);
      if (dz) buf_store_f32x4(make_float4(nx[o][0], nx[o][1], nx[o][2], nx[o][3]), rz, voff + 64 * o, 0);
      pin4(nx[o]);
    };
#pragma unroll
    for (int o = 0; o < DT; ++o) {
      const float4 hc = hn;
      if (o + 1 < DT) hn = buf_load_f32x4(rh, voff + 64 * (o + 1), 0);
      const u32x4* cb = st.begin(Wt, o, DT, c2_tile_u4(KBI), nextW, next_u4);
      const f32x4 acc = c2_tile<KBI, false>(cb, in, f32x4{0.f, 0.f, 0.f, 0.f}, lane);
      if (o > 0) epi(o - 1, prev, hp);
      prev = acc;
      hp = hc;
    }
    epi(DT - 1, prev, hp);
  };
  // ---- last Linear (input: dy, OTL tiles)
  {
    u32x4 bl[KBL][3];
    c2_split<OTL>(dy, bl);
    const u32x4* nextW = reinterpret_cast<const u32x4*>(nl - 2 >= 1 ? L[nl - 2].WpT : (a.dX ? L[0].WpT : nullptr));
    const int next_u4 = c2_tile_u4(KB);
    layer(WL, bl, nl - 1, nextW, next_u4);
  }
  // ---- hidden Linears nl-2 .. 1
  for (int l = nl - 2; l >= 1; --l) {
    c2_split<DT>(nx, bp);
    const u32x4* Wt = reinterpret_cast<const u32x4*>(L[l].WpT);
    const u32x4* nextW = reinterpret_cast<const u32x4*>(l - 1 >= 1 ? L[l - 1].WpT : (a.dX ? L[0].WpT : nullptr));
    layer(Wt, bp, l, nextW, c2_tile_u4(KB));
  }
  // ---- first Linear: dX = W_0^T dz_0 (KT0 output tiles)
  if (a.dX) {
    c2_split<DT>(nx, bp);
    const u32x4* W0 = reinterpret_cast<const u32x4*>(L[0].WpT);
    float dx[KT0][4];
#pragma unroll
    for (int o = 0; o < KT0; ++o) {
      const u32x4* cb = st.begin(W0, o, KT0, c2_tile_u4(KB), nullptr, 0);
      f32x4 acc = c2_tile<KB, false>(cb, bp, f32x4{0.f, 0.f, 0.f, 0.f}, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) dx[o][r] = acc[r];
    }
    store_rows<KT0>(dx, a.dX + e * a.dx_chain_stride, a.lddx, p, valid, a.in_dim, lane);
  }
}

template <int D>
static hipError_t launch_chain2_d(const ChainArgs& a, bool bwd, hipStream_t s) {
  constexpr int DT = D / 16;
  const dim3 grid((a.P + 16 * kC2Waves - 1) / (16 * kC2Waves), a.nchains), block(64 * kC2Waves);
  const size_t lds = 2 * (size_t)c2_tile_u4(DT / 2) * 16;
#define GNOT_C2_CASE(K0, OL)                                                                         \
  if (a.KT0 == K0 && a.OTL == OL) {                                                                  \
    static bool attr = false;                                                                        \
    if (!attr) {                                                                                     \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(chain2_bwd_kernel<D, K0, OL>),         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);               \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(chain2_fwd_kernel<D, K0, OL>),         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);               \
      attr = true;                                                                                   \
    }                                                                                                \
    if (bwd) hipLaunchKernelGGL((chain2_bwd_kernel<D, K0, OL>), grid, block, lds, s, a);             \
    else hipLaunchKernelGGL((chain2_fwd_kernel<D, K0, OL>), grid, block, lds, s, a);                 \
    return hipGetLastError();                                                                        \
  }
  GNOT_C2_CASE(1, 1)
  GNOT_C2_CASE(1, DT)
  GNOT_C2_CASE(DT, 1)
  GNOT_C2_CASE(DT, DT)
#undef GNOT_C2_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_chain2(const ChainArgs& a, bool bwd, hipStream_t s) {
  if (a.P <= 0 || a.nchains <= 0) return hipSuccess;
  if (a.nlin < 2) return hipErrorInvalidValue;
  switch (a.D) {
    case 256: return launch_chain2_d<256>(a, bwd, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gnot
