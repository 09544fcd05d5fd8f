// MLP chains at hidden widths above 256 (model.py:5-18, the soft-MoE experts of model.py:128-137, the
// gating of model.py:155-156), one Linear at a time.  The fused chain kernels (chain.hip, chain2.hip)
// hold a point's whole activation row in VGPRs; at d = 320 .. 512 that row no longer fits beside the
// MFMA operands, so here every Linear is one projection launch (linear.hip, fp32 MFMA on fp32 images:
// exact fp32 products) and the activation between two Linears goes through HBM:
//   forward : h_l = W_l x_l + b_l (into the chain's save slot, or scratch without saves),
//             x_{l+1} = gelu(h_l) (scratch); the last layer's output through the mode's epilogue
//   backward: dz_{nl-1} from the mode's prologue, g = dz_l W_l (scratch), dz_{l-1} = g * gelu'(h_{l-1}),
//             dX = dz_0 W_0
// Same ChainArgs contract, save / dz layouts and results as the fused kernels (up to the fp32 summation
// order), so the engine's weight gradients, combine and input gradients are unchanged.
#include <algorithm>

#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

namespace {

// x = gelu(h) over n contiguous floats
__global__ void __launch_bounds__(256) cw_gelu_kernel(const float* __restrict__ h, float* __restrict__ x, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) x[i] = gelu(h[i]);
}

// dz = g * gelu'(h) over n contiguous floats
__global__ void __launch_bounds__(256) cw_gelu_grad_kernel(const float* __restrict__ g, const float* __restrict__ h,
                                                           float* __restrict__ dz, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dz[i] = g[i] * gelu_grad(h[i]);
}

// wave reductions over the 64 lanes
GNOT_DEV float wsum(float v) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
GNOT_DEV float wmax(float v) {
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// the last Linear's output h (row pitch D) of chain e through the mode's epilogue: one wave per point
//   CH_STORE  : Y[p, f] = h[p, f]                         (f < out_dim)
//   CH_SOFTMAX: Y[p, :] = softmax(h[p, :out_dim])          (model.py:156)
//   CH_MOE    : Y_e[p, f] = scores[p, e] * h[p, f]         (model.py:128-131: the stage term)
__global__ void __launch_bounds__(256) cw_out_kernel(ChainArgs a, int e, const float* __restrict__ h, int D) {
  const int lane = threadIdx.x & 63;
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= a.P) return;
  const float* hr = h + p * D;
  float* y = a.Y + e * a.y_chain_stride + p * a.ldy;
  if (a.mode == CH_SOFTMAX) {
    float m = -INFINITY;
    for (int f = lane; f < a.out_dim; f += 64) m = fmaxf(m, hr[f]);
    m = wmax(m);
    float s = 0.f;
    for (int f = lane; f < a.out_dim; f += 64) s += __expf(hr[f] - m);
    const float inv = 1.0f / wsum(s);
    for (int f = lane; f < a.out_dim; f += 64) y[f] = __expf(hr[f] - m) * inv;
  } else if (a.mode == CH_MOE) {
    const float sc = a.scores[p * a.ldsc + e];
    for (int f = lane; f < a.out_dim; f += 64) y[f] = sc * hr[f];
  } else {
    for (int f = lane; f < a.out_dim; f += 64) y[f] = hr[f];
  }
}

// the output gradient of chain e into dz_{nl-1} (row pitch D, columns [0, ncols); zero past out_dim):
//   CH_STORE  : dY
//   CH_SOFTMAX: s * (ds - <s, ds>)      (s = scores, ds = dscore)
//   CH_MOE    : scores[p, e] * dY, and dscore[p, e] += <dY, y_e> with y_e the saved last output
__global__ void __launch_bounds__(256) cw_dy_kernel(ChainArgs a, int e, float* __restrict__ dz, const float* __restrict__ ysave,
                                                    int D, int ncols) {
  const int lane = threadIdx.x & 63;
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= a.P) return;
  float* dr = dz + p * D;
  if (a.mode == CH_MOE) {
    const float* dq = a.dY + p * a.lddy;
    const float* yr = ysave + p * D;
    float ds = 0.f;
    for (int f = lane; f < a.out_dim; f += 64) ds += dq[f] * yr[f];
    ds = wsum(ds);
    const float sc = a.scores[p * a.ldsc + e];
    if (lane == 0) a.dscore[p * a.ldsc + e] += ds;
    for (int f = lane; f < ncols; f += 64) dr[f] = f < a.out_dim ? sc * dq[f] : 0.f;
  } else if (a.mode == CH_SOFTMAX) {
    const float* s = a.scores + p * a.ldsc;
    const float* g = a.dscore + p * a.ldsc;
    float dot = 0.f;
    for (int f = lane; f < a.out_dim; f += 64) dot += s[f] * g[f];
    dot = wsum(dot);
    for (int f = lane; f < ncols; f += 64) dr[f] = f < a.out_dim ? s[f] * (g[f] - dot) : 0.f;
  } else {
    const float* dy = a.dY + p * a.lddy;
    for (int f = lane; f < ncols; f += 64) dr[f] = f < a.out_dim ? dy[f] : 0.f;
  }
}

unsigned ew_blocks(long n) { return (unsigned)std::min<long>((n + 255) / 256, 8192); }

// one Linear: Y[p, :ncol] = X[p, :K] W^T (+ bias), W an fp32 fragment image KT tiles deep
hipError_t cw_linear(const float* X, long ldx, int K, int KT, const void* W, const float* bias, float* Y, long ldy,
                     int NO, int P, int ncol, hipStream_t s) {
  LinearArgs l{};
  l.nseg = 1; l.X[0] = X; l.Wp[0] = static_cast<const float4*>(W); l.ldx = ldx; l.nsum = 1; l.sum_stride = 0;
  l.K = K; l.bias = bias; l.Y = Y; l.ldy = ldy; l.NO = NO; l.P = P; l.epi = EPI_STORE; l.nsoft = 0; l.dh = 16;
  l.ncol = ncol;
  return launch_linear(l, 16 * KT, s);
}

}  // namespace

hipError_t launch_chainw(const ChainArgs& a, bool bwd, hipStream_t s) {
  const int D = a.D, DT = D / 16, nl = a.nlin, P = a.P;
  if (!a.layers_host || !a.scratch || nl < 2) return hipErrorInvalidValue;
  const long n = (long)P * D;
  float* s0 = a.scratch;                 // h (forward without saves) / g (backward)
  float* s1 = a.scratch + n;             // x = gelu(h)
  const dim3 rows_grid((P + 3) / 4), rows_block(256);
  for (int e = 0; e < a.nchains; ++e) {
    const ChainLayer* L = a.layers_host + (size_t)e * nl;
    const float* save = a.save ? a.save + e * a.save_chain_stride : nullptr;
    auto h_of = [&](int l) { return save ? const_cast<float*>(save) + l * a.save_layer_stride : s0; };
    if (!bwd) {
      for (int l = 0; l < nl; ++l) {
        const bool first = l == 0, last = l == nl - 1;
        float* h = h_of(l);
        hipError_t r = cw_linear(first ? a.X : s1, first ? a.ldx : D, first ? a.in_dim : D, first ? a.KT0 : DT,
                                 L[l].Wp, L[l].bias, h, D, last ? 16 * a.OTL : D, P, 0, s);
        if (r != hipSuccess) return r;
        if (!last) hipLaunchKernelGGL(cw_gelu_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, h, s1, n);
        else if (a.Y) hipLaunchKernelGGL(cw_out_kernel, rows_grid, rows_block, 0, s, a, e, h, D);
      }
    } else {
      if (!save || !a.dz) return hipErrorInvalidValue;
      float* dz = a.dz + e * a.dz_chain_stride;
      hipLaunchKernelGGL(cw_dy_kernel, rows_grid, rows_block, 0, s, a, e, dz + (nl - 1) * a.dz_layer_stride,
                         save + (nl - 1) * a.save_layer_stride, D, 16 * a.OTL);
      for (int l = nl - 1; l >= 1; --l) {
        const bool last = l == nl - 1;
        hipError_t r = cw_linear(dz + l * a.dz_layer_stride, D, last ? 16 * a.OTL : D, last ? a.OTL : DT, L[l].WpT,
                                 nullptr, s0, D, D, P, 0, s);
        if (r != hipSuccess) return r;
        hipLaunchKernelGGL(cw_gelu_grad_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, s0,
                           save + (l - 1) * a.save_layer_stride, dz + (l - 1) * a.dz_layer_stride, n);
      }
      if (a.dX) {
        hipError_t r = cw_linear(dz, D, D, DT, L[0].WpT, nullptr, a.dX + e * a.dx_chain_stride, a.lddx, 16 * a.KT0, P,
                                 a.in_dim, s);
        if (r != hipSuccess) return r;
      }
    }
  }
  return hipGetLastError();
}

}  // namespace gnot
