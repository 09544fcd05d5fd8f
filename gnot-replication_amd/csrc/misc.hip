// Small point-streaming kernels around the hot path.
//   concat_theta : x_in[p] = cat(x[p], theta[sample(p)])   (reference model.py:158-159; theta is
//                  broadcast per sample over that sample's points — packed offsets, no padding)
//   moe_combine  : q_out = q_in + sum_e stage[e]           (reference model.py:129-131, 135-137)
//                  (q_in may be null: plain sum, used for the expert-summed dX of the MoE backward)
//   segcopy      : table-driven float4 copy of contiguous runs (the point-shard scramble all-to-all's
//                  pack / unpack, engine.cpp build_exchange)
//   input grads  : d x = d x_in[:, :in] + d x_gate (x feeds the encoder through cat and the gating MLP,
//                  model.py:155, 158-161), d theta[b] = sum over sample b's points of d x_in[:, in:]
//                  (the broadcast of model.py:158), d fn = the encoder chain's input gradient
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

__global__ void __launch_bounds__(256) concat_theta_kernel(const float* __restrict__ x, long ldx, int in_dim,
                                                           const float* __restrict__ theta, int th_dim,
                                                           const long* __restrict__ off, int B,
                                                           float* __restrict__ xin, long ldxin, int P) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)P * ldxin) return;
  const long p = i / ldxin;
  const int c = (int)(i % ldxin);
  float v = 0.f;                                   // pad columns are zero
  if (c < in_dim) {
    v = x[p * ldx + c];
  } else if (c < in_dim + th_dim) {
    int lo = 0, hi = B - 1;                        // sample of point p
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= p) lo = mid; else hi = mid - 1;
    }
    v = theta[(long)lo * th_dim + (c - in_dim)];
  }
  xin[i] = v;
}

hipError_t launch_concat_theta(const float* x, long ldx, int in_dim, const float* theta, int th_dim,
                               const long* off, int B, float* xin, long ldxin, int P, hipStream_t s) {
  const long n = (long)P * ldxin;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(concat_theta_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, in_dim,
                     theta, th_dim, off, B, xin, ldxin, P);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) moe_combine_kernel(const float4* __restrict__ base,
                                                          const float4* __restrict__ stage,
                                                          long stage_stride4, int E,
                                                          float4* __restrict__ out, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 v = base ? base[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = 0; e < E; ++e) {
      const float4 s = stage[e * stage_stride4 + i];
      v.x += s.x; v.y += s.y; v.z += s.z; v.w += s.w;
    }
    out[i] = v;
  }
}

hipError_t launch_moe_combine(const float* base, const float* stage, long stage_stride, int E,
                              float* out, long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if ((n & 3) || (stage_stride & 3)) return hipErrorInvalidValue;
  const long n4 = n / 4;
  const long blocks = std::min<long>((n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(moe_combine_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(base), reinterpret_cast<const float4*>(stage),
                     stage_stride / 4, E, reinterpret_cast<float4*>(out), n4);
  return hipGetLastError();
}

// bf16 stage rows: thread = one 16-byte chunk k of a point's 512-byte pair-interleaved row (gnot_common.h
// b16_off): features f0 .. f0+3 (half 0) and f0+16 .. f0+19 (half 1), f0 = 32 (k >> 2) + 4 (k & 3).  Sums in
// expert order from base, as moe_combine does over the same (bf16-exact) values: bitwise equal to it
__global__ void __launch_bounds__(256) moe_combine_b16_kernel(const float* __restrict__ base,
                                                              const float* __restrict__ stage, long stage_stride,
                                                              int E, float* __restrict__ out, long P) {
  const long nch = P * 32;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nch; i += (long)gridDim.x * 256) {
    const long pnt = i >> 5;
    const int k = (int)(i & 31), f0 = 32 * (k >> 2) + 4 * (k & 3);
    const long fo = pnt * 256 + f0;
    float4 lo = base ? *reinterpret_cast<const float4*>(base + fo) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 hi = base ? *reinterpret_cast<const float4*>(base + fo + 16) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float* sp = stage + pnt * (kB16Row / 4) + 4 * k;
    for (int e = 0; e < E; ++e) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(sp + e * stage_stride);
      lo.x += bf16_lo(w[0]); lo.y += bf16_hi(w[0]); lo.z += bf16_lo(w[1]); lo.w += bf16_hi(w[1]);
      hi.x += bf16_lo(w[2]); hi.y += bf16_hi(w[2]); hi.z += bf16_lo(w[3]); hi.w += bf16_hi(w[3]);
    }
    *reinterpret_cast<float4*>(out + fo) = lo;
    *reinterpret_cast<float4*>(out + fo + 16) = hi;
  }
}

hipError_t launch_moe_combine_b16(const float* base, const float* stage, long stage_stride, int E, float* out,
                                  long P, hipStream_t s) {
  if (P <= 0) return hipSuccess;
  if (stage_stride & 3) return hipErrorInvalidValue;
  const long blocks = std::min<long>((P * 32 + 255) / 256, 8192);
  hipLaunchKernelGGL(moe_combine_b16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, base, stage, stage_stride, E,
                     out, P);
  return hipGetLastError();
}

// U = 4: float4 units (every run offset / length a multiple of 4 floats); U = 1: single floats (padded heads:
// runs of a head width that is not a multiple of 4)
template <int U>
__global__ void __launch_bounds__(256) segcopy_kernel(const CopySeg* __restrict__ segs, const int* __restrict__ prefix,
                                                      int nseg, int total, const float* __restrict__ src,
                                                      float* __restrict__ dst, int reverse) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (prefix[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const CopySeg sg = segs[lo];
    const long off = (long)(i - prefix[lo]) * U;
    const long so = reverse ? sg.b : sg.a, dof = reverse ? sg.a : sg.b;
    if constexpr (U == 4) *reinterpret_cast<float4*>(dst + dof + off) = *reinterpret_cast<const float4*>(src + so + off);
    else dst[dof + off] = src[so + off];
  }
}

hipError_t launch_segcopy(const CopySeg* segs, const int* prefix, int nseg, int total, const float* src, float* dst,
                          bool reverse, hipStream_t s, int unit) {
  if (nseg <= 0 || total <= 0) return hipSuccess;
  const int blocks = std::min((total + 255) / 256, 4096);
  if (unit == 4)
    hipLaunchKernelGGL(segcopy_kernel<4>, dim3(blocks), dim3(256), 0, s, segs, prefix, nseg, total, src, dst, reverse ? 1 : 0);
  else if (unit == 1)
    hipLaunchKernelGGL(segcopy_kernel<1>, dim3(blocks), dim3(256), 0, s, segs, prefix, nseg, total, src, dst, reverse ? 1 : 0);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// d x [P, in] = a[:, :in] + b[:, :in] (b may be null); a plain column copy when b is null
__global__ void __launch_bounds__(256) add_cols_kernel(const float* __restrict__ a, long lda, const float* __restrict__ b,
                                                       long ldb, int cols, float* __restrict__ out, long rows) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const long r = i / cols;
  const int c = (int)(i % cols);
  out[i] = b ? a[r * lda + c] + b[r * ldb + c] : a[r * lda + c];
}

// d theta[b][t] = sum_{p in sample b} a[p][c0 + t]: one workgroup per (b, t), strided partial sums then a
// fixed-order tree in LDS (deterministic)
__global__ void __launch_bounds__(256) seg_colsum_kernel(const float* __restrict__ a, long lda, int c0, int ncols,
                                                         const long* __restrict__ off, float* __restrict__ out) {
  __shared__ float red[256];
  const int b = blockIdx.x, t = blockIdx.y;
  float acc = 0.f;
  for (long p = off[b] + threadIdx.x; p < off[b + 1]; p += 256) acc += a[p * lda + c0 + t];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[(long)b * ncols + t] = red[0];
}

hipError_t launch_add_cols(const float* a, long lda, const float* b, long ldb, int cols, float* out, long rows,
                           hipStream_t s) {
  const long n = rows * cols;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(add_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, lda, b, ldb, cols, out,
                     rows);
  return hipGetLastError();
}

hipError_t launch_seg_colsum(const float* a, long lda, int c0, int ncols, const long* off, int B, float* out,
                             hipStream_t s) {
  if (B <= 0 || ncols <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_colsum_kernel, dim3(B, ncols), dim3(256), 0, s, a, lda, c0, ncols, off, out);
  return hipGetLastError();
}

}  // namespace gnot
