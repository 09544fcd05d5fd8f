// Normalized linear attention core (reference LinearAttention.forward, model.py:53-107).
//
// For one sample and head h (q, k already feature-softmaxed by the projection epilogue):
//   z   = sum_m k_m                      [dh]      (model.py:77 / 98)
//   S   = sum_m k_m v_m^T                [dh, dh]  (model.py:79 / 100)
//   o_n = (q_n S) / (q_n . z)                       (model.py:78,80 / 99,101)
//   res = scramble(q + mean_i o_i)                  (model.py:81-86 / 103-104)
// `scramble` is the reshape of the head-major [H, N, dh] buffer straight into [N, d] without
// un-permuting, so the apply pass WRITES head-major per sample: element (h, n, j) of sample b lands
// at flat offset off_b*d + (h*N_b + n)*dh + j, and fc_out reads that buffer as plain rows.
//
// Kernels here:
//   attn_apply_fwd / attn_apply_bwd  one 64-point segment per workgroup, one thread per (point, head)
//                in point-major order (coalesced row reads); every head's (S, z) staged in LDS.
//   attn_kv_bwd  dK, dV from (dS, dz) per (source point, head), same geometry.
// The cross-point reductions themselves (S, z forward; dS, dz backward) are point-reduction GEMMs
// on the MFMA path (wgrad.hip, state jobs), one job per sample.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

// u = x M  for a row vector x[DH] and a row-major DH x DH matrix M in LDS (float4 row reads)
template <int DH>
GNOT_DEV void rowvec_times_mat(const float (&x)[DH], const float* M, float (&u)[DH]) {
#pragma unroll
  for (int j = 0; j < DH; ++j) u[j] = 0.f;
#pragma unroll
  for (int k = 0; k < DH; ++k) {
#pragma unroll
    for (int j = 0; j < DH; j += 4) {
      const float4 m = *reinterpret_cast<const float4*>(M + k * DH + j);
      u[j] = fmaf(x[k], m.x, u[j]);
      u[j + 1] = fmaf(x[k], m.y, u[j + 1]);
      u[j + 2] = fmaf(x[k], m.z, u[j + 2]);
      u[j + 3] = fmaf(x[k], m.w, u[j + 3]);
    }
  }
}

// x . row  for a row of DH floats in LDS
template <int DH>
GNOT_DEV float dot_row(const float (&x)[DH], const float* row) {
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int j = 0; j < DH; j += 4) {
    const float4 m = *reinterpret_cast<const float4*>(row + j);
    a = fmaf(x[j], m.x, a);
    b = fmaf(x[j + 1], m.y, b);
    a = fmaf(x[j + 2], m.z, a);
    b = fmaf(x[j + 3], m.w, b);
  }
  return a + b;
}

// ---------------------------------------------------------------- apply (forward)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_fwd_kernel(AttnApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int4 ch = a.chunks[blockIdx.x];
  const int b = ch.x;
  const int H = a.H;
  constexpr int ph = DH * DH + DH;
  const int per = H * ph;
  for (int i = threadIdx.x; i < a.nsrc * per; i += 256) {
    const int sidx = i / per, e = i % per;
    smem[i] = a.state[sidx][(long)b * per + e];
  }
  __syncthreads();
  const long off_b = a.off[b];
  const long Nb = a.off[b + 1] - off_b;
  const int d = H * DH;
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  // point-major work order: consecutive lanes read consecutive heads of one point row (coalesced)
  for (int idx = threadIdx.x; idx < ch.z * H; idx += 256) {
    const long n = ch.y + idx / H;       // global point index
    const int h = idx % H;
    float q[DH], os[DH];
#pragma unroll
    for (int j = 0; j < DH; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(a.q + n * a.ldq + h * DH + j);
      q[j] = v.x; q[j + 1] = v.y; q[j + 2] = v.z; q[j + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < DH; ++j) os[j] = 0.f;
    for (int sidx = 0; sidx < a.nsrc; ++sidx) {
      const float* S = smem + sidx * per + h * ph;
      const float* z = S + DH * DH;
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k) den = fmaf(q[k], z[k], den);
      float u[DH];
      rowvec_times_mat<DH>(q, S, u);
      const float inv = 1.0f / den;
#pragma unroll
      for (int j = 0; j < DH; ++j) os[j] = fmaf(u[j], inv, os[j]);
    }
    float* dst = a.res + off_b * d + ((long)h * Nb + (n - off_b)) * DH;
#pragma unroll
    for (int j = 0; j < DH; j += 4)
      *reinterpret_cast<float4*>(dst + j) =
          make_float4(q[j] + os[j] * inv_nsrc, q[j + 1] + os[j + 1] * inv_nsrc,
                      q[j + 2] + os[j + 2] * inv_nsrc, q[j + 3] + os[j + 3] * inv_nsrc);
  }
}

// ---------------------------------------------------------------- apply (backward)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_bwd_kernel(AttnApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int4 ch = a.chunks[blockIdx.x];
  const int b = ch.x;
  const int H = a.H;
  constexpr int ph = DH * DH + DH;
  const int per = H * ph;
  for (int i = threadIdx.x; i < a.nsrc * per; i += 256) {
    const int sidx = i / per, e = i % per;
    smem[i] = a.state[sidx][(long)b * per + e];
  }
  __syncthreads();
  const long off_b = a.off[b];
  const long Nb = a.off[b + 1] - off_b;
  const int d = H * DH;
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  for (int idx = threadIdx.x; idx < ch.z * H; idx += 256) {
    const long n = ch.y + idx / H;
    const int h = idx % H;
    float q[DH], dO[DH], dq[DH];
    const float* src = a.dres + off_b * d + ((long)h * Nb + (n - off_b)) * DH;
#pragma unroll
    for (int j = 0; j < DH; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(a.q + n * a.ldq + h * DH + j);
      q[j] = v.x; q[j + 1] = v.y; q[j + 2] = v.z; q[j + 3] = v.w;
      const float4 g = *reinterpret_cast<const float4*>(src + j);
      dq[j] = g.x; dq[j + 1] = g.y; dq[j + 2] = g.z; dq[j + 3] = g.w;
    }
#pragma unroll
    for (int j = 0; j < DH; ++j) dO[j] = dq[j] * inv_nsrc;
    for (int sidx = 0; sidx < a.nsrc; ++sidx) {
      const float* S = smem + sidx * per + h * ph;
      const float* z = S + DH * DH;
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k) den = fmaf(q[k], z[k], den);
      float u[DH];
      rowvec_times_mat<DH>(q, S, u);
      const float inv = 1.0f / den;
      // o = u/den ; du = dO/den ; dden = -(dO . o)/den
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < DH; ++j) dot = fmaf(dO[j], u[j], dot);
      const float dden = -dot * inv * inv;
      float du[DH];
#pragma unroll
      for (int j = 0; j < DH; ++j) du[j] = dO[j] * inv;
      // dq += du S^T + dden z
#pragma unroll
      for (int k = 0; k < DH; ++k) dq[k] = fmaf(dden, z[k], dq[k] + dot_row<DH>(du, S + k * DH));
      float* dup = a.du[sidx] + n * a.lddu + h * DH;
#pragma unroll
      for (int j = 0; j < DH; j += 4)
        *reinterpret_cast<float4*>(dup + j) = make_float4(du[j], du[j + 1], du[j + 2], du[j + 3]);
      a.dden[sidx][n * H + h] = dden;
    }
    // softmax backward over the head's features
    float qdq = 0.f;
#pragma unroll
    for (int j = 0; j < DH; ++j) qdq = fmaf(q[j], dq[j], qdq);
    float* dst = a.dq_pre + n * a.lddq + h * DH;
#pragma unroll
    for (int j = 0; j < DH; j += 4)
      *reinterpret_cast<float4*>(dst + j) =
          make_float4(q[j] * (dq[j] - qdq), q[j + 1] * (dq[j + 1] - qdq), q[j + 2] * (dq[j + 2] - qdq),
                      q[j + 3] * (dq[j + 3] - qdq));
  }
}

// ---------------------------------------------------------------- K/V backward
template <int DH>
GNOT_DEV void attn_kv_bwd_body(const AttnKVBwdArgs& a, float* smem) {
  const int4 ch = a.chunks[blockIdx.x];
  const int b = ch.x;
  const int H = a.H;
  constexpr int ph = DH * DH + DH;
  const int per = H * ph;
  for (int i = threadIdx.x; i < per; i += 256) smem[i] = a.dstate[(long)b * per + i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < ch.z * H; idx += 256) {
    const long m = ch.y + idx / H;
    const int h = idx % H;
    const float* dS = smem + h * ph;
    const float* dz = dS + DH * DH;
    float k[DH], v[DH];
#pragma unroll
    for (int j = 0; j < DH; j += 4) {
      const float4 kv = *reinterpret_cast<const float4*>(a.k + m * a.ldkv + h * DH + j);
      k[j] = kv.x; k[j + 1] = kv.y; k[j + 2] = kv.z; k[j + 3] = kv.w;
      const float4 vv = *reinterpret_cast<const float4*>(a.v + m * a.ldkv + h * DH + j);
      v[j] = vv.x; v[j + 1] = vv.y; v[j + 2] = vv.z; v[j + 3] = vv.w;
    }
    float dk[DH], dv[DH];
#pragma unroll
    for (int i = 0; i < DH; ++i) dk[i] = dz[i] + dot_row<DH>(v, dS + i * DH);
    rowvec_times_mat<DH>(k, dS, dv);
    float kdk = 0.f;
#pragma unroll
    for (int i = 0; i < DH; ++i) kdk = fmaf(k[i], dk[i], kdk);
    float* dkp = a.dk + m * a.lddkv + h * DH;
    float* dvp = a.dv + m * a.lddkv + h * DH;
#pragma unroll
    for (int j = 0; j < DH; j += 4) {
      *reinterpret_cast<float4*>(dkp + j) =
          make_float4(k[j] * (dk[j] - kdk), k[j + 1] * (dk[j + 1] - kdk), k[j + 2] * (dk[j + 2] - kdk),
                      k[j + 3] * (dk[j + 3] - kdk));
      *reinterpret_cast<float4*>(dvp + j) = make_float4(dv[j], dv[j + 1], dv[j + 2], dv[j + 3]);
    }
  }
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_kernel(AttnKVBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  attn_kv_bwd_body<DH>(a, smem);
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_batch_kernel(const AttnKVBwdArgs* __restrict__ jobs) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const AttnKVBwdArgs a = jobs[blockIdx.y];
  if ((int)blockIdx.x >= a.nchunks) return;
  attn_kv_bwd_body<DH>(a, smem);
}

#define GNOT_DH_SWITCH(DHV, ...)        \
  switch (DHV) {                        \
    case 4: { constexpr int DH = 4; __VA_ARGS__; } break;    \
    case 8: { constexpr int DH = 8; __VA_ARGS__; } break;    \
    case 16: { constexpr int DH = 16; __VA_ARGS__; } break;  \
    case 32: { constexpr int DH = 32; __VA_ARGS__; } break;  \
    case 48: { constexpr int DH = 48; __VA_ARGS__; } break;  \
    case 64: { constexpr int DH = 64; __VA_ARGS__; } break;  \
    default: return hipErrorInvalidValue;                    \
  }

template <typename K>
static void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

hipError_t launch_attn_apply_fwd(const AttnApplyArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const size_t lds = (size_t)a.nsrc * a.H * (a.dh * a.dh + a.dh) * sizeof(float);
  GNOT_DH_SWITCH(a.dh, allow_lds(attn_apply_fwd_kernel<DH>, lds);
                 hipLaunchKernelGGL(attn_apply_fwd_kernel<DH>, dim3(a.nchunks), dim3(256), lds, s, a));
  return hipGetLastError();
}

hipError_t launch_attn_apply_bwd(const AttnApplyArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const size_t lds = (size_t)a.nsrc * a.H * (a.dh * a.dh + a.dh) * sizeof(float);
  GNOT_DH_SWITCH(a.dh, allow_lds(attn_apply_bwd_kernel<DH>, lds);
                 hipLaunchKernelGGL(attn_apply_bwd_kernel<DH>, dim3(a.nchunks), dim3(256), lds, s, a));
  return hipGetLastError();
}

hipError_t launch_attn_kv_bwd(const AttnKVBwdArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const size_t lds = (size_t)a.H * (a.dh * a.dh + a.dh) * sizeof(float);
  GNOT_DH_SWITCH(a.dh, allow_lds(attn_kv_bwd_kernel<DH>, lds);
                 hipLaunchKernelGGL(attn_kv_bwd_kernel<DH>, dim3(a.nchunks), dim3(256), lds, s, a));
  return hipGetLastError();
}

hipError_t launch_attn_kv_bwd_batch(const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks, int H, int dh,
                                    hipStream_t s) {
  if (njobs <= 0 || maxchunks <= 0) return hipSuccess;
  const size_t lds = (size_t)H * (dh * dh + dh) * sizeof(float);
  GNOT_DH_SWITCH(dh, allow_lds(attn_kv_bwd_batch_kernel<DH>, lds);
                 hipLaunchKernelGGL(attn_kv_bwd_batch_kernel<DH>, dim3(maxchunks, njobs), dim3(256), lds, s, jobs_dev));
  return hipGetLastError();
}

}  // namespace gnot
