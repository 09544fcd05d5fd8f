// Attention projections at hidden width d = 256 on bf16x6 MFMA, output-major (x6_core.h):
//   Y[p, :NO] (=|+=) epi( sum_s X_s[p, :256] . W_s^T + bias )
// the query/key/value projections with the feature softmax of model.py:59/72/93 fused into the
// epilogue (model.py:56, 67-68, 89-90), fc_out (model.py:106), and the backward-data products
// dX = dY W of those Linears (dX = dQ Wq + dK Wk + dV Wv in one pass for the fused q|k|v).
// 8 waves x 16 points per workgroup share one weight stream (one LDS chunk = one 16-column output
// tile of an output-major x6 image); the input rows are loaded once and held as their exact bf16 split.
//   linear2_kernel     one K-segment, any NO = 16 * OT: tiles are produced one head group (dh / 16
//                      tiles) at a time and stored at once (softmax over the group when it lies in the
//                      first nsoft columns).
//   linear2_seg_kernel several K-segments (NO = 256): the 16 output tiles accumulate in registers
//                      across the segments, one segment's input split at a time.
#include <algorithm>
#include <cstdlib>

#include "gnot_kernels.h"
#include "x6_core.h"

namespace gnot {

// waves (16 points each) per workgroup: bf16x6 4 (two workgroups per CU, one's input loads and output
// stores overlap the other's MFMAs; the 384 KiB x6 image stays L2-resident), one piece 8.  Interleaved on
// one box (profiles/r04l2w_linear2_waves_ab.txt), 8 -> 4 waves: bf16x6 NO = 256 251 -> 233 us, accumulate
// 300 -> 266, three K-segments 670 -> 645, NO = 768 585 -> 552; one piece 131 -> 153 and 273 -> 351 (its
// eight waves already fit two workgroups per CU by registers)
template <int NP>
constexpr int l2_waves() { return NP == 3 ? 4 : 8; }

template <int TPH, int NP>   // output tiles per softmax head (dh / 16); operand pieces (3 = x6, 1 = bf16)
__global__ void __launch_bounds__(64 * l2_waves<NP>(), 2) linear2_kernel(LinearArgs a) {
  constexpr int DT = 16, KB = 8;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const long p = ((long)blockIdx.x * l2_waves<NP>() + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  // output tiles [ob, oe) of this workgroup: grid.y splits the NO / 16 tiles into equal chunks of whole
  // head groups (small batches: more workgroups than points / 16 / waves alone give, launch_linear2_np)
  const int OTc = a.NO / 16 / (int)gridDim.y;
  const int ob = (int)blockIdx.y * OTc, oe = ob + OTc;
  const u32x4* W = reinterpret_cast<const u32x4*>(a.Wp[0]);
  C2Stream st{c2lds, c2_tile_u4(KB, NP), 0, wave, lane, l2_waves<NP>()};
  stage_image(reinterpret_cast<float4*>(c2lds), reinterpret_cast<const float4*>(W + (size_t)ob * c2_tile_u4(KB, NP)),
              c2_tile_u4(KB, NP), l2_waves<NP>(), wave, lane);
  u32x4 bp[KB][NP];
  {
    float x[DT][4];
    load_rows<DT>(x, a.X[0], a.ldx, p, valid, a.K, lane);
    c2_split<DT, NP>(x, bp);
  }
  // bias of the next head group and the old output rows (EPI_ACCUM) are loaded one group ahead / before
  // the MFMAs: a load placed after a barrier would expose its full latency on every tile.  Heads of 128 / 256
  // features (TPH 8 / 16) load them at their use instead (three TPH-float4 arrays would not fit beside h)
  constexpr bool PF = TPH <= 4;
  constexpr int NPF = PF ? TPH : 1;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 bn[NPF];
  if constexpr (PF) {
#pragma unroll
    for (int k = 0; k < TPH; ++k) bn[k] = a.bias ? ld4(a.bias + 16 * (ob + k) + 4 * g) : zero4;
  }
  const long pc = valid ? p : 0;
  for (int o0 = ob; o0 < oe; o0 += TPH) {
    float h[TPH][4];
    float4 bc[NPF], old[NPF];
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < TPH; ++k) {
        bc[k] = bn[k];
        if (a.bias && o0 + TPH < oe) bn[k] = ld4(a.bias + 16 * (o0 + TPH + k) + 4 * g);
        if (a.epi == EPI_ACCUM && !(a.ncol > 0 && 16 * (o0 + k) + 4 * g >= a.ncol))
          old[k] = ld4(a.Y + pc * a.ldy + 16 * (o0 + k) + 4 * g);
      }
    }
#pragma unroll
    for (int k = 0; k < TPH; ++k) {
      const int o = o0 + k;
      const u32x4* cb = st.begin(W, o, oe, c2_tile_u4(KB, NP), nullptr, 0);
      const float4 b0 = PF ? bc[PF ? k : 0] : (a.bias ? ld4(a.bias + 16 * o + 4 * g) : zero4);
      // the epilogue form with no epilogue: its scheduling fences keep k-block t+1's fragment reads ahead
      // of block t's MFMAs (the plain form compiled to reads issued next to their MFMAs here)
      const f32x4 acc = c2_tile_epi<KB, NP, true>(cb, bp, f32x4{b0.x, b0.y, b0.z, b0.w}, lane, [](int) {});
#pragma unroll
      for (int r = 0; r < 4; ++r) h[k][r] = acc[r];
    }
    if (16 * o0 < a.nsoft) {
      // feature softmax over the head: TPH tiles x (4 features of each of the 4 lane groups)
      float m = -INFINITY;
#pragma unroll
      for (int k = 0; k < TPH; ++k) m = fmaxf(m, fmaxf(fmaxf(h[k][0], h[k][1]), fmaxf(h[k][2], h[k][3])));
      m = fmaxf(m, shfl_xor(m, 16));
      m = fmaxf(m, shfl_xor(m, 32));
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < TPH; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) { h[k][r] = __expf(h[k][r] - m); sum += h[k][r]; }
      sum += shfl_xor(sum, 16);
      sum += shfl_xor(sum, 32);
      const float inv = 1.0f / sum;
#pragma unroll
      for (int k = 0; k < TPH; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) h[k][r] *= inv;
    }
    if (a.dreal > 0) {
      // pad columns of a padded width (LinearArgs::dreal; whole heads of 16 / 32 / 64 features, so the
      // pad columns are whole tiles of each 256-column block)
#pragma unroll
      for (int k = 0; k < TPH; ++k)
        if ((16 * (o0 + k)) % 256 >= a.dreal) h[k][0] = h[k][1] = h[k][2] = h[k][3] = 0.f;
    }
    if (valid) {
#pragma unroll
      for (int k = 0; k < TPH; ++k) {
        const int f = 16 * (o0 + k) + 4 * g;
        if (a.ncol > 0 && f >= a.ncol) continue;     // a row pitch below NO (ncol a multiple of 4)
        float4 v = make_float4(h[k][0], h[k][1], h[k][2], h[k][3]);
        if (a.epi == EPI_ACCUM) {
          const float4 ov = PF ? old[PF ? k : 0] : ld4(a.Y + p * a.ldy + f);
          v.x += ov.x; v.y += ov.y; v.z += ov.z; v.w += ov.w;
        }
        *reinterpret_cast<float4*>(a.Y + p * a.ldy + f) = v;
      }
    }
  }
}

template <int NP>
__global__ void __launch_bounds__(64 * l2_waves<NP>(), 2) linear2_seg_kernel(LinearArgs a) {
  constexpr int DT = 16, KB = 8;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const long p = ((long)blockIdx.x * l2_waves<NP>() + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  C2Stream st{c2lds, c2_tile_u4(KB, NP), 0, wave, lane, l2_waves<NP>()};
  // output tiles [ob, oe) of this workgroup (grid.y chunks, as linear2_kernel)
  const int OTc = DT / (int)gridDim.y;
  const int ob = (int)blockIdx.y * OTc, oe = ob + OTc;
  constexpr int TU = c2_tile_u4(KB, NP);
  stage_image(reinterpret_cast<float4*>(c2lds), reinterpret_cast<const float4*>(reinterpret_cast<const u32x4*>(a.Wp[0]) + (size_t)ob * TU),
              TU, l2_waves<NP>(), wave, lane);
  f32x4 acc[DT];
#pragma unroll
  for (int o = 0; o < DT; ++o) {
    if (a.bias) {
      const float4 b = ld4(a.bias + 16 * o + 4 * g);
      acc[o] = f32x4{b.x, b.y, b.z, b.w};
    } else {
      acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  for (int s = 0; s < a.nseg; ++s) {
    u32x4 bp[KB][NP];
    {
      float x[DT][4];
      load_rows<DT>(x, a.X[s], a.ldx, p, valid, a.K, lane);
      c2_split<DT, NP>(x, bp);
    }
    const u32x4* W = reinterpret_cast<const u32x4*>(a.Wp[s]);
    const u32x4* next = s + 1 < a.nseg ? reinterpret_cast<const u32x4*>(a.Wp[s + 1]) + (size_t)ob * TU : nullptr;
#pragma unroll
    for (int o = 0; o < DT; ++o) {
      if (o < ob || o >= oe) continue;                // workgroup-uniform
      const u32x4* cb = st.begin(W, o, oe, TU, next, TU);
      acc[o] = c2_tile_epi<KB, NP, true>(cb, bp, acc[o], lane, [](int) {});   // reads one k-block ahead
    }
  }
  if (valid) {
#pragma unroll
    for (int o = 0; o < DT; ++o) {
      if (o < ob || o >= oe) continue;
      float4* y = reinterpret_cast<float4*>(a.Y + p * a.ldy + 16 * o + 4 * g);
      float4 v = make_float4(acc[o][0], acc[o][1], acc[o][2], acc[o][3]);
      if (a.epi == EPI_ACCUM) {
        const float4 old = *y;
        v.x += old.x; v.y += old.y; v.z += old.z; v.w += old.w;
      }
      *y = v;
    }
  }
}

bool linear2_supported(const LinearArgs& a, int D) {
  // K < 256: the input rows are read zero-filled past K (a padded width's scramble rows)
  return D == 256 && a.K >= 1 && a.K <= 256 && a.nsum == 1 && a.NO % 16 == 0 && (a.ldx & 3) == 0 &&
         (a.ldy & 3) == 0 && (a.ncol & 3) == 0 && (a.dreal & 15) == 0 &&
         (a.nseg == 1 ? (a.nsoft == 0 || a.dh == 16 || a.dh == 32 || a.dh == 64 || a.dh == 128 || a.dh == 256)
                      : (a.NO == 256 && a.nsoft == 0 && a.ncol == 0));
}

// output-tile chunks per launch: enough workgroups for two per CU (their register budget) on small batches
// (configs[0]: 16,384 points = 256 workgroups of 4 waves, each streaming the whole image tile by tile, one wave
// per SIMD); a divisor of the head groups, 1 from 512 point workgroups up (GNOT_LINEAR2_CHUNKS overrides)
static int l2_chunks(int nwg, int groups) {
  static const int env = [] {
    const char* e = std::getenv("GNOT_LINEAR2_CHUNKS");
    return e ? std::atoi(e) : 0;
  }();
  int want = env > 0 ? env : (512 + nwg - 1) / nwg;
  want = std::max(1, std::min(want, groups));
  while (groups % want) --want;
  return want;
}

template <int NP>
static hipError_t launch_linear2_np(const LinearArgs& a, hipStream_t s) {
  const size_t lds = 2 * (size_t)c2_tile_u4(8, NP) * 16;
  const int nwg = (a.P + 16 * l2_waves<NP>() - 1) / (16 * l2_waves<NP>());
  const int tph = a.nseg > 1 ? 1 : (a.nsoft ? a.dh / 16 : 2);
  const dim3 grid(nwg, l2_chunks(nwg, a.NO / 16 / tph)), block(64 * l2_waves<NP>());
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(linear2_kernel<1, NP>), reinterpret_cast<const void*>(linear2_kernel<2, NP>),
                          reinterpret_cast<const void*>(linear2_kernel<4, NP>), reinterpret_cast<const void*>(linear2_kernel<8, NP>),
                          reinterpret_cast<const void*>(linear2_kernel<16, NP>), reinterpret_cast<const void*>(linear2_seg_kernel<NP>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (a.nseg > 1) {
    hipLaunchKernelGGL(linear2_seg_kernel<NP>, grid, block, lds, s, a);
  } else {
    if (tph == 1) hipLaunchKernelGGL((linear2_kernel<1, NP>), grid, block, lds, s, a);
    else if (tph == 2) hipLaunchKernelGGL((linear2_kernel<2, NP>), grid, block, lds, s, a);
    else if (tph == 4) hipLaunchKernelGGL((linear2_kernel<4, NP>), grid, block, lds, s, a);
    else if (tph == 8) hipLaunchKernelGGL((linear2_kernel<8, NP>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((linear2_kernel<16, NP>), grid, block, lds, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_linear2(const LinearArgs& a, hipStream_t s) {
  if (a.P <= 0) return hipSuccess;
  if (!linear2_supported(a, 256)) return hipErrorInvalidValue;
  return a.np == 1 ? launch_linear2_np<1>(a, s) : launch_linear2_np<3>(a, s);
}

}  // namespace gnot
