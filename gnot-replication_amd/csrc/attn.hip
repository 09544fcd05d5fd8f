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
// Kernels:
//   attn_state   per point segment: partial S and z for every head (register-blocked 4x4 outer
//                products from an LDS-staged point tile) -> slab; attn_state_reduce sums the slabs
//                of each sample in a fixed order (deterministic; the only cross-point reduction).
//   attn_apply_fwd / attn_apply_bwd  one thread per (point, head).
//   attn_kv_bwd  dK, dV from (dS, dz) per (source point, head).
// The same state kernel also produces dS = sum_n q_n du_n^T and dz = sum_n dden_n q_n in the backward.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

constexpr int kStateSub = 16;   // points per LDS sub-tile of the state kernel
constexpr int kStateMaxB = 4;   // 4x4 blocks per thread -> d*dh <= 16384

// segment list: chunks[c] = (b, start, len, -)
__global__ void __launch_bounds__(256) attn_state_kernel(AttnStateArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int d = a.H * a.dh;
  const int dhp = a.dh;
  float* As = smem;                     // [kStateSub][d]
  float* Bs = smem + kStateSub * d;     // [kStateSub][d]
  float* Ws = Bs + kStateSub * d;       // [kStateSub][H]
  const int4 ch = a.chunks[blockIdx.x];
  const long start = ch.y;
  const int len = ch.z;
  const int t = threadIdx.x;
  const int nbh = (dhp / 4) * (dhp / 4);     // 4x4 blocks per head
  const int nblocks = a.H * nbh;

  float acc[kStateMaxB][16];
#pragma unroll
  for (int k = 0; k < kStateMaxB; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  float zacc = 0.f;

  for (int s0 = 0; s0 < len; s0 += kStateSub) {
    const int sl = min(kStateSub, len - s0);
    __syncthreads();
    for (int i = t; i < kStateSub * d; i += 256) {
      const int n = i / d, c = i % d;
      const bool ok = n < sl;
      As[i] = ok ? a.A[(start + s0 + n) * a.lda + c] : 0.f;
      Bs[i] = ok ? a.Bv[(start + s0 + n) * a.ldb + c] : 0.f;
    }
    for (int i = t; i < kStateSub * a.H; i += 256) {
      const int n = i / a.H, hh = i % a.H;
      Ws[i] = (n < sl) ? (a.w ? a.w[(start + s0 + n) * a.ldw + hh] : 1.f) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kStateMaxB; ++k) {
      const int bid = t + k * 256;
      if (bid < nblocks) {
        const int h = bid / nbh, rem = bid % nbh;
        const int ib = rem / (dhp / 4), jb = rem % (dhp / 4);
        const float* ap = As + h * dhp + 4 * ib;
        const float* bp = Bs + h * dhp + 4 * jb;
        for (int n = 0; n < sl; ++n) {
          const float4 av = *reinterpret_cast<const float4*>(ap + n * d);
          const float4 bv = *reinterpret_cast<const float4*>(bp + n * d);
          const float aa[4] = {av.x, av.y, av.z, av.w};
          const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[k][i * 4 + j] = fmaf(aa[i], bb[j], acc[k][i * 4 + j]);
        }
      }
    }
    if (t < d) {
      const int h = t / dhp;
      for (int n = 0; n < sl; ++n) zacc = fmaf(Ws[n * a.H + h], As[n * d + t], zacc);
    }
  }
  // slab layout per chunk: [H][dh*dh + dh]
  const int per_head = dhp * dhp + dhp;
  float* S = a.slab + (long)blockIdx.x * a.H * per_head;
#pragma unroll
  for (int k = 0; k < kStateMaxB; ++k) {
    const int bid = t + k * 256;
    if (bid < nblocks) {
      const int h = bid / nbh, rem = bid % nbh;
      const int ib = rem / (dhp / 4), jb = rem % (dhp / 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          S[h * per_head + (4 * ib + i) * dhp + 4 * jb + j] = acc[k][i * 4 + j];
    }
  }
  if (t < d) {
    const int h = t / dhp, i = t % dhp;
    S[h * per_head + dhp * dhp + i] = zacc;
  }
}

__global__ void __launch_bounds__(256) attn_state_reduce_kernel(AttnStateArgs a) {
  const int per = a.H * (a.dh * a.dh + a.dh);
  const int b = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= per) return;
  const int c0 = a.sample_chunk_off[b], c1 = a.sample_chunk_off[b + 1];
  float s = 0.f;
  for (int c = c0; c < c1; ++c) s += a.slab[(long)c * per + e];
  a.state[(long)b * per + e] = s;
}

hipError_t launch_attn_state(const AttnStateArgs& a, hipStream_t s) {
  const int d = a.H * a.dh;
  if (a.dh % 4 != 0 || d * a.dh > 16 * 256 * kStateMaxB || d > 256 * 4) return hipErrorInvalidValue;
  const size_t lds = (size_t)(2 * kStateSub * d + kStateSub * a.H) * sizeof(float);
  if (a.nchunks > 0)
    hipLaunchKernelGGL(attn_state_kernel, dim3(a.nchunks), dim3(256), lds, s, a);
  const int per = a.H * (a.dh * a.dh + a.dh);
  if (a.B > 0)
    hipLaunchKernelGGL(attn_state_reduce_kernel, dim3((per + 255) / 256, a.B), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------- apply (forward)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_fwd_kernel(AttnApplyArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int4 ch = a.chunks[blockIdx.x];
  const int b = ch.x;
  const int H = a.H;
  const int per = H * (DH * DH + DH);
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
    const long n = ch.y + idx / H;     // global point index
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
      const float* S = smem + sidx * per + h * (DH * DH + DH);
      const float* z = S + DH * DH;
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k) den = fmaf(q[k], z[k], den);
      float u[DH];
#pragma unroll
      for (int j = 0; j < DH; ++j) u[j] = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k)
#pragma unroll
        for (int j = 0; j < DH; ++j) u[j] = fmaf(q[k], S[k * DH + j], u[j]);
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
  const int per = H * (DH * DH + DH);
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
      const float* S = smem + sidx * per + h * (DH * DH + DH);
      const float* z = S + DH * DH;
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k) den = fmaf(q[k], z[k], den);
      float u[DH];
#pragma unroll
      for (int j = 0; j < DH; ++j) u[j] = 0.f;
#pragma unroll
      for (int k = 0; k < DH; ++k)
#pragma unroll
        for (int j = 0; j < DH; ++j) u[j] = fmaf(q[k], S[k * DH + j], u[j]);
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
      for (int k = 0; k < DH; ++k) {
        float acc = dden * z[k];
#pragma unroll
        for (int j = 0; j < DH; ++j) acc = fmaf(du[j], S[k * DH + j], acc);
        dq[k] += acc;
      }
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
__global__ void __launch_bounds__(256) attn_kv_bwd_kernel(AttnKVBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int4 ch = a.chunks[blockIdx.x];
  const int b = ch.x;
  const int H = a.H;
  const int per = H * (DH * DH + DH);
  for (int i = threadIdx.x; i < per; i += 256) smem[i] = a.dstate[(long)b * per + i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < ch.z * H; idx += 256) {
    const long m = ch.y + idx / H;
    const int h = idx % H;
    const float* dS = smem + h * (DH * DH + DH);
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
    for (int i = 0; i < DH; ++i) {
      float acc = dz[i];
#pragma unroll
      for (int j = 0; j < DH; ++j) acc = fmaf(v[j], dS[i * DH + j], acc);
      dk[i] = acc;
    }
#pragma unroll
    for (int j = 0; j < DH; ++j) dv[j] = 0.f;
#pragma unroll
    for (int i = 0; i < DH; ++i)
#pragma unroll
      for (int j = 0; j < DH; ++j) dv[j] = fmaf(k[i], dS[i * DH + j], dv[j]);
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
  GNOT_DH_SWITCH(a.dh, hipLaunchKernelGGL(attn_kv_bwd_kernel<DH>, dim3(a.nchunks), dim3(256), lds, s, a));
  return hipGetLastError();
}

}  // namespace gnot
