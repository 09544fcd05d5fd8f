// Projection kernel: Y[p, :NO] (=|+=) epi( sum_s X_s[p, :K] . A + bias )
//
// Used for the attention projections (reference model.py:56, 67-68, 89-90: query/key/value, with
// the feature softmax of model.py:59/72/93 fused into the epilogue), fc_out (model.py:106) and every
// backward-data product dX = dY W of those Linears.  One wave = 16 points held in point form
// (gnot_common.h), the input row block is loaded ONCE and reused for all NO output columns; the
// A operand is the packed weight image streamed from L2 (one 1 KiB load per 4 MFMAs).
// The input may be a sum of `nsum` equally strided buffers (the per-expert dX stage of the MoE
// backward), which fuses the expert reduction into the consumer.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

template <int D>
__global__ void __launch_bounds__(256) linear_kernel(LinearArgs a) {
  constexpr int KT = D / 16;
  constexpr int OC = lds_och(KT, (D / 16) < 8 ? (D / 16) : 8);   // output tiles per workgroup chunk
  __shared__ __attribute__((aligned(16))) float4 wlds[2 * kChunkF4];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const long p = ((long)blockIdx.x * 4 + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;

  float in[KT][4];
  load_rows<KT>(in, a.X, a.ldx, p, valid, a.K, lane);
  for (int s = 1; s < a.nsum; ++s) {
    float t[KT][4];
    load_rows<KT>(t, a.X + s * a.sum_stride, a.ldx, p, valid, a.K, lane);
#pragma unroll
    for (int T = 0; T < KT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) in[T][r] += t[T][r];
  }

  // grid.y splits the output chunks over workgroups (more parallelism at small point counts)
  const int nchunks = a.NO / (16 * OC);
  int cnt = 0;
  if ((int)blockIdx.y < nchunks)
    stage_image(wlds, a.Wp + (long)blockIdx.y * OC * KT * WAVE, chunk_f4(KT, OC), 4, wave, lane);
  for (int c = blockIdx.y; c < nchunks; c += gridDim.y) {
    f32x4 acc[OC];
    init_bias<OC>(acc, a.bias ? a.bias + c * 16 * OC : nullptr, lane);
    const bool more = c + (int)gridDim.y < nchunks;
    mm_tiles_pipe<KT, OC>(a.Wp + (long)c * OC * KT * WAVE,
                          more ? a.Wp + (long)(c + gridDim.y) * OC * KT * WAVE : nullptr, chunk_f4(KT, OC), wlds,
                          cnt, in, acc, 4, wave, lane);
    float h[OC][4];
    acc_to_regs<OC>(acc, h);
    if (c * 16 * OC < a.nsoft) softmax_heads<OC>(h, a.dh);
    float* Y = a.Y + c * 16 * OC;
    if (a.epi == EPI_ACCUM) {
      float old[OC][4];
      load_rows<OC>(old, Y, a.ldy, p, valid, 16 * OC, lane);
#pragma unroll
      for (int T = 0; T < OC; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) h[T][r] += old[T][r];
    }
    store_rows<OC>(h, Y, a.ldy, p, valid, 16 * OC, lane);
  }
}

hipError_t launch_linear(const LinearArgs& a, int D, hipStream_t s) {
  if (a.P <= 0) return hipSuccess;
  const int oc = lds_och(D / 16, D / 16 < 8 ? D / 16 : 8);   // == the kernel's OC
  const int nchunks = a.NO / (16 * oc);
  const dim3 grid((a.P + 63) / 64, nchunks), block(256);
  switch (D) {
    case 32: hipLaunchKernelGGL(linear_kernel<32>, grid, block, 0, s, a); break;
    case 48: hipLaunchKernelGGL(linear_kernel<48>, grid, block, 0, s, a); break;
    case 64: hipLaunchKernelGGL(linear_kernel<64>, grid, block, 0, s, a); break;
    case 128: hipLaunchKernelGGL(linear_kernel<128>, grid, block, 0, s, a); break;
    case 256: hipLaunchKernelGGL(linear_kernel<256>, grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace gnot
