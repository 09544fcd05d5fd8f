// Attention apply passes on fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 sums) --
// the Q . state contractions of reference LinearAttention.forward (model.py:78-80 / 99-101) and their
// backward, for head widths dh = 16, 32, 64.  Same arguments and results as attn.hip's VALU kernels
// (which stay for other head widths and as the A/B reference, env GNOT_APPLY_VALU).
//
// Point form (gnot_common.h): a wave owns 16 points; lane l holds, for every 16-feature tile T of a
// head, features 16T + 4(l>>4) + r (r < 4) of point l & 15 -- which is both the B operand of the
// 16x16x4 MFMA contracting over those features and the layout of its result.  So per head:
//   u^T = S^T q^T     A = S^T fragments from LDS (image "ST": lane (j, g) of block (J, T) holds
//                     S[16T + 4g + r][16J + j]), B = the point's q tiles, result = u tiles
//   v^T = S dO^T      (backward) A = S fragments (image "SN": S[16K + k][16J + 4g + r])
// and den = q . z is a lane dot plus two shuffles (the 4 lanes of a point).  A workgroup (4 waves,
// one 64-point chunk per pass) walks `cpw` consecutive chunks and re-stages the images from the
// L2-resident states only when the sample changes.  HBM traffic is the rows: q and res (forward),
// q, dres, du, dq (backward).
#include <cstdlib>

#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

namespace {

constexpr int kApplyCpw = 4;   // 64-point chunks per workgroup (>= 4 waves per SIMD at 262k points)

template <int DH>
struct ApplyGeo {
  static constexpr int NT = DH / 16;                 // 16-feature tiles per head
  static constexpr int IMG = NT * NT * WAVE;         // float4 per (source, head) image
};

// LDS: [ST images: ns*H*IMG float4][SN images (backward)][z: ns*H*DH floats]
template <int DH>
size_t apply_lds_bytes(int ns, int H, bool bwd) {
  return ((size_t)(bwd ? 2 : 1) * ns * H * ApplyGeo<DH>::IMG * 4 + (size_t)ns * H * DH) * 4;
}

// stage the images of sample b (all sources, all heads) from the [B][H][DH*DH + DH] states
template <int DH, bool BWD>
GNOT_DEV void stage_states(const AttnApplyArgs& a, int b, float4* st, float4* sn, float* zl) {
  using Gm = ApplyGeo<DH>;
  constexpr int ph = DH * DH + DH;
  const int H = a.H;
  const int n4 = a.nsrc * H * Gm::IMG;
  for (int i = threadIdx.x; i < n4; i += blockDim.x) {
    const int lane = i % WAVE;
    int rest = i / WAVE;
    const int T = rest % Gm::NT; rest /= Gm::NT;
    const int J = rest % Gm::NT; rest /= Gm::NT;
    const int h = rest % H;
    const int s = rest / H;
    const float* S = a.state[s] + ((long)b * H + h) * ph;
    const int j = lane & 15, g = lane >> 4;
    // ST: S[16T + 4g + r][16J + j]  (column walk)
    const float* c0 = S + (16 * T + 4 * g) * DH + 16 * J + j;
    st[i] = make_float4(c0[0], c0[DH], c0[2 * DH], c0[3 * DH]);
    // SN: S[16J + j][16T + 4g + r]  (row segment); J plays the output tile K, T the input tile
    if (BWD) sn[i] = *reinterpret_cast<const float4*>(S + (16 * J + j) * DH + 16 * T + 4 * g);
  }
  for (int i = threadIdx.x; i < a.nsrc * H * DH; i += blockDim.x) {
    const int c = i % DH, hs = i / DH;
    zl[i] = a.state[hs / H][((long)b * H + hs % H) * ph + DH * DH + c];
  }
}

// sum over the 4 lanes of a point (lane groups g = 0..3)
GNOT_DEV float point_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

template <int NT>
GNOT_DEV void load_tiles(float (&t)[NT][4], const float* __restrict__ row, bool valid, int g) {
#pragma unroll
  for (int T = 0; T < NT; ++T) {
    const float4 v = valid ? *reinterpret_cast<const float4*>(row + 16 * T + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
    t[T][0] = v.x; t[T][1] = v.y; t[T][2] = v.z; t[T][3] = v.w;
  }
}

template <int NT>
GNOT_DEV void store_tiles(float* __restrict__ row, const float (&t)[NT][4], int g) {
#pragma unroll
  for (int T = 0; T < NT; ++T)
    *reinterpret_cast<float4*>(row + 16 * T + 4 * g) = make_float4(t[T][0], t[T][1], t[T][2], t[T][3]);
}

// out tiles (J) = image (J, T) x in tiles (T), one 16x16 output tile per J
template <int NT>
GNOT_DEV void img_mm(const float4* __restrict__ img, const float (&in)[NT][4], f32x4 (&out)[NT], int lane) {
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int T = 0; T < NT; ++T) acc = mfma_k16(img[(J * NT + T) * WAVE + lane], in[T], acc);
    out[J] = acc;
  }
}

template <int NT>
GNOT_DEV float tile_dot(const float (&x)[NT][4], const float* __restrict__ zh, int g) {
  float d = 0.f;
#pragma unroll
  for (int T = 0; T < NT; ++T) {
    const float4 z = *reinterpret_cast<const float4*>(zh + 16 * T + 4 * g);
    d = fmaf(x[T][0], z.x, fmaf(x[T][1], z.y, fmaf(x[T][2], z.z, fmaf(x[T][3], z.w, d))));
  }
  return point_sum(d);
}

}  // namespace

// ---------------------------------------------------------------- forward
// res = q + (1/nsrc) sum_s (q S_s) / (q . z_s), written head-major per sample (the scramble)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_fwd_mfma_kernel(AttnApplyArgs a, int cpw) {
  using Gm = ApplyGeo<DH>;
  constexpr int NT = Gm::NT;
  extern __shared__ __attribute__((aligned(16))) float4 alds[];
  const int H = a.H, ns = a.nsrc;
  float4* st = alds;
  float* zl = reinterpret_cast<float*>(alds + (size_t)ns * H * Gm::IMG);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const float inv_ns = 1.0f / (float)ns;
  int cur_b = -1;
  for (int i = 0; i < cpw; ++i) {
    const int c = blockIdx.x * cpw + i;
    if (c >= a.nchunks) break;
    const int4 ch = a.chunks[c];
    if (ch.x != cur_b) {
      __syncthreads();
      stage_states<DH, false>(a, ch.x, st, nullptr, zl);
      __syncthreads();
      cur_b = ch.x;
    }
    const int pl = wave * 16 + (lane & 15);
    const bool valid = pl < ch.z;
    const long n = ch.y + pl;
    const long off_b = a.off[ch.x];
    const long Nb = a.off[ch.x + 1] - off_b;
    const float* qrow = a.q + (valid ? n : 0) * a.ldq;
    float* rbase = a.res + off_b * (long)H * DH + (n - off_b) * DH;
    for (int h = 0; h < H; ++h) {
      float q[NT][4];
      load_tiles<NT>(q, qrow + h * DH, valid, g);
      float o[NT][4];
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[T][r] = 0.f;
      for (int s = 0; s < ns; ++s) {
        const int hs = s * H + h;
        const float inv = 1.0f / tile_dot<NT>(q, zl + hs * DH, g);
        f32x4 u[NT];
        img_mm<NT>(st + (size_t)hs * Gm::IMG, q, u, lane);
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[T][r] = fmaf(u[T][r], inv, o[T][r]);
      }
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[T][r] = fmaf(o[T][r], inv_ns, q[T][r]);
      if (valid) store_tiles<NT>(rbase + (long)h * Nb * DH, o, g);
    }
  }
}

// ---------------------------------------------------------------- backward
// dO = dres / nsrc; per source: u = q S, den = q . z, du = dO / den, dden = -(dO . u) / den^2,
// dq += (dO S^T) / den + dden z; dq starts at dres (the q residual); then the feature-softmax
// backward of q: dq_pre = q * (dq - q . dq)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_bwd_mfma_kernel(AttnApplyArgs a, int cpw) {
  using Gm = ApplyGeo<DH>;
  constexpr int NT = Gm::NT;
  extern __shared__ __attribute__((aligned(16))) float4 alds[];
  const int H = a.H, ns = a.nsrc;
  float4* st = alds;
  float4* sn = alds + (size_t)ns * H * Gm::IMG;
  float* zl = reinterpret_cast<float*>(alds + (size_t)2 * ns * H * Gm::IMG);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const float inv_ns = 1.0f / (float)ns;
  int cur_b = -1;
  for (int i = 0; i < cpw; ++i) {
    const int c = blockIdx.x * cpw + i;
    if (c >= a.nchunks) break;
    const int4 ch = a.chunks[c];
    if (ch.x != cur_b) {
      __syncthreads();
      stage_states<DH, true>(a, ch.x, st, sn, zl);
      __syncthreads();
      cur_b = ch.x;
    }
    const int pl = wave * 16 + (lane & 15);
    const bool valid = pl < ch.z;
    const long n = ch.y + pl;
    const long nv = valid ? n : 0;
    const long off_b = a.off[ch.x];
    const long Nb = a.off[ch.x + 1] - off_b;
    const float* qrow = a.q + nv * a.ldq;
    const float* dbase = a.dres + off_b * (long)H * DH + (n - off_b) * DH;
    for (int h = 0; h < H; ++h) {
      float q[NT][4], dq[NT][4], dO[NT][4];
      load_tiles<NT>(q, qrow + h * DH, valid, g);
      load_tiles<NT>(dq, dbase + (long)h * Nb * DH, valid, g);
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) dO[T][r] = dq[T][r] * inv_ns;
      for (int s = 0; s < ns; ++s) {
        const int hs = s * H + h;
        const float* zh = zl + hs * DH;
        const float inv = 1.0f / tile_dot<NT>(q, zh, g);
        f32x4 u[NT], v[NT];
        img_mm<NT>(st + (size_t)hs * Gm::IMG, q, u, lane);
        img_mm<NT>(sn + (size_t)hs * Gm::IMG, dO, v, lane);
        float dot = 0.f;
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
          for (int r = 0; r < 4; ++r) dot = fmaf(dO[T][r], u[T][r], dot);
        const float dden = -point_sum(dot) * inv * inv;
        float du[NT][4];
#pragma unroll
        for (int T = 0; T < NT; ++T) {
          const float4 z = *reinterpret_cast<const float4*>(zh + 16 * T + 4 * g);
          const float zr[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            du[T][r] = dO[T][r] * inv;
            dq[T][r] = fmaf(v[T][r], inv, fmaf(dden, zr[r], dq[T][r]));
          }
        }
        if (valid) {
          store_tiles<NT>(a.du[s] + n * a.lddu + h * DH, du, g);
          if (g == 0) a.dden[s][n * H + h] = dden;
        }
      }
      float qdq = 0.f;
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) qdq = fmaf(q[T][r], dq[T][r], qdq);
      qdq = point_sum(qdq);
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[T][r] = q[T][r] * (dq[T][r] - qdq);
      if (valid) store_tiles<NT>(a.dq_pre + n * a.lddq + h * DH, dq, g);
    }
  }
}

namespace {
constexpr size_t kApplyLdsMax = 160 * 1024;

template <int DH>
bool mfma_ok(const AttnApplyArgs& a, bool bwd) {
  static const bool valu = std::getenv("GNOT_APPLY_VALU") != nullptr;
  return !valu && a.nsrc >= 1 && a.nsrc <= 8 && (a.ldq & 3) == 0 && (!bwd || ((a.lddq & 3) == 0 && (a.lddu & 3) == 0)) &&
         apply_lds_bytes<DH>(a.nsrc, a.H, bwd) <= kApplyLdsMax;
}

template <int DH, bool BWD>
hipError_t launch_mfma(const AttnApplyArgs& a, hipStream_t s) {
  const size_t lds = apply_lds_bytes<DH>(a.nsrc, a.H, BWD);
  const void* f = BWD ? reinterpret_cast<const void*>(attn_apply_bwd_mfma_kernel<DH>)
                      : reinterpret_cast<const void*>(attn_apply_fwd_mfma_kernel<DH>);
  if (lds > 64 * 1024) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const dim3 grid((a.nchunks + kApplyCpw - 1) / kApplyCpw), block(256);
  if (BWD) hipLaunchKernelGGL(attn_apply_bwd_mfma_kernel<DH>, grid, block, lds, s, a, kApplyCpw);
  else hipLaunchKernelGGL(attn_apply_fwd_mfma_kernel<DH>, grid, block, lds, s, a, kApplyCpw);
  return hipGetLastError();
}
}  // namespace

// returns hipErrorNotSupported when the head width / LDS size has no MFMA variant (caller falls back)
hipError_t launch_attn_apply_mfma(const AttnApplyArgs& a, bool bwd, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  switch (a.dh) {
    case 16: if (mfma_ok<16>(a, bwd)) return bwd ? launch_mfma<16, true>(a, s) : launch_mfma<16, false>(a, s); break;
    case 32: if (mfma_ok<32>(a, bwd)) return bwd ? launch_mfma<32, true>(a, s) : launch_mfma<32, false>(a, s); break;
    case 64: if (mfma_ok<64>(a, bwd)) return bwd ? launch_mfma<64, true>(a, s) : launch_mfma<64, false>(a, s); break;
    default: break;
  }
  return hipErrorNotSupported;
}

}  // namespace gnot
