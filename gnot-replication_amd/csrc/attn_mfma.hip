// Attention apply passes on fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 sums) --
// the Q . state contractions of reference LinearAttention.forward (model.py:78-80 / 99-101) and their
// backward, for head widths dh = 16, 32, 64.  Same arguments and results as attn.hip's VALU kernels
// (which stay for other head widths and for small meshes, GNOT_APPLY_MFMA_MIN).
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
GNOT_DEV void stage_states(const float* const* state, int nsrc, int H, int b, float4* st, float4* sn, float* zl) {
  using Gm = ApplyGeo<DH>;
  constexpr int ph = DH * DH + DH;
  const int n4 = nsrc * H * Gm::IMG;
  for (int i = threadIdx.x; i < n4; i += blockDim.x) {
    const int lane = i % WAVE;
    int rest = i / WAVE;
    const int T = rest % Gm::NT; rest /= Gm::NT;
    const int J = rest % Gm::NT; rest /= Gm::NT;
    const int h = rest % H;
    const int s = rest / H;
    const float* S = state[s] + ((long)b * H + h) * ph;
    const int j = lane & 15, g = lane >> 4;
    // ST: S[16T + 4g + r][16J + j]  (column walk)
    const float* c0 = S + (16 * T + 4 * g) * DH + 16 * J + j;
    st[i] = make_float4(c0[0], c0[DH], c0[2 * DH], c0[3 * DH]);
    // SN: S[16J + j][16T + 4g + r]  (row segment); J plays the output tile K, T the input tile
    if (BWD) sn[i] = *reinterpret_cast<const float4*>(S + (16 * J + j) * DH + 16 * T + 4 * g);
  }
  for (int i = threadIdx.x; i < nsrc * H * DH; i += blockDim.x) {
    const int c = i % DH, hs = i / DH;
    zl[i] = state[hs / H][((long)b * H + hs % H) * ph + DH * DH + c];
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
      stage_states<DH, false>(a.state, a.nsrc, H, ch.x, st, nullptr, zl);
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
    float qn[NT][4];
    load_tiles<NT>(qn, qrow, valid, g);
    for (int h = 0; h < H; ++h) {
      // the next head's rows are in flight while this head computes
      float q[NT][4];
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) q[T][r] = qn[T][r];
      if (h + 1 < H) load_tiles<NT>(qn, qrow + (h + 1) * DH, valid, g);
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
      stage_states<DH, true>(a.state, a.nsrc, H, ch.x, st, sn, zl);
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
    float qn[NT][4], dn[NT][4];
    load_tiles<NT>(qn, qrow, valid, g);
    load_tiles<NT>(dn, dbase, valid, g);
    for (int h = 0; h < H; ++h) {
      float q[NT][4], dq[NT][4], dO[NT][4];
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) { q[T][r] = qn[T][r]; dq[T][r] = dn[T][r]; }
      if (h + 1 < H) {
        load_tiles<NT>(qn, qrow + (h + 1) * DH, valid, g);
        load_tiles<NT>(dn, dbase + (long)(h + 1) * Nb * DH, valid, g);
      }
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

// ---------------------------------------------------------------- K/V backward
// dv = k dS (the ST image of dS), dk = dz + v dS^T (the SN image), then the feature-softmax backward
// of k: dk_pre = k * (dk - k . dk).  One job = (k, v, dS) of one attention call; the batched form
// runs every (block, input function) job of the cross attention in one launch (job = blockIdx.z).
template <int DH>
GNOT_DEV void kv_bwd_mfma_body(const AttnKVBwdArgs& a, int cpw, int bx) {
  using Gm = ApplyGeo<DH>;
  constexpr int NT = Gm::NT;
  extern __shared__ __attribute__((aligned(16))) float4 alds[];
  const int H = a.H;
  float4* st = alds;
  float4* sn = alds + (size_t)H * Gm::IMG;
  float* zl = reinterpret_cast<float*>(alds + (size_t)2 * H * Gm::IMG);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const float* const states[1] = {a.dstate};
  int cur_b = -1;
  for (int i = 0; i < cpw; ++i) {
    const int c = bx * cpw + i;
    if (c >= a.nchunks) break;
    const int4 ch = a.chunks[c];
    if (ch.x != cur_b) {
      __syncthreads();
      stage_states<DH, true>(states, 1, H, ch.x, st, sn, zl);
      __syncthreads();
      cur_b = ch.x;
    }
    const int pl = wave * 16 + (lane & 15);
    const bool valid = pl < ch.z;
    const long n = ch.y + pl;
    const long nv = valid ? n : 0;
    float kn[NT][4], vn[NT][4];
    load_tiles<NT>(kn, a.k + nv * a.ldkv, valid, g);
    load_tiles<NT>(vn, a.v + nv * a.ldkv, valid, g);
    for (int h = 0; h < H; ++h) {
      float k[NT][4], v[NT][4];
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) { k[T][r] = kn[T][r]; v[T][r] = vn[T][r]; }
      if (h + 1 < H) {
        load_tiles<NT>(kn, a.k + nv * a.ldkv + (h + 1) * DH, valid, g);
        load_tiles<NT>(vn, a.v + nv * a.ldkv + (h + 1) * DH, valid, g);
      }
      f32x4 dv[NT], dk[NT];
      img_mm<NT>(st + (size_t)h * Gm::IMG, k, dv, lane);
      img_mm<NT>(sn + (size_t)h * Gm::IMG, v, dk, lane);
      const float* zh = zl + h * DH;
      float kdk = 0.f;
      float dko[NT][4], dvo[NT][4];
#pragma unroll
      for (int T = 0; T < NT; ++T) {
        const float4 z = *reinterpret_cast<const float4*>(zh + 16 * T + 4 * g);
        const float zr[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dko[T][r] = zr[r] + dk[T][r];
          dvo[T][r] = dv[T][r];
          kdk = fmaf(k[T][r], dko[T][r], kdk);
        }
      }
      kdk = point_sum(kdk);
#pragma unroll
      for (int T = 0; T < NT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) dko[T][r] = k[T][r] * (dko[T][r] - kdk);
      if (valid) {
        store_tiles<NT>(a.dk + n * a.lddkv + h * DH, dko, g);
        store_tiles<NT>(a.dv + n * a.lddkv + h * DH, dvo, g);
      }
    }
  }
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_mfma_kernel(AttnKVBwdArgs a, int cpw) {
  kv_bwd_mfma_body<DH>(a, cpw, blockIdx.x);
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_batch_mfma_kernel(const AttnKVBwdArgs* __restrict__ jobs, int cpw) {
  const AttnKVBwdArgs a = jobs[blockIdx.z];
  if ((int)blockIdx.x * cpw >= a.nchunks) return;
  kv_bwd_mfma_body<DH>(a, cpw, blockIdx.x);
}

namespace {
constexpr size_t kApplyLdsMax = 160 * 1024;
// below this many 64-point chunks the MFMA passes run fewer than ~128 workgroups, each staging the
// state images before its few chunks: the VALU kernels (attn.hip) are faster there (configs[1],
// 10k points: apply bwd 23 vs 70 us per call; env GNOT_APPLY_MFMA_MIN overrides)
static int mfma_min_chunks() {
  const char* e = std::getenv("GNOT_APPLY_MFMA_MIN");    // read per launch: tests force either path
  return e ? std::atoi(e) : 512;
}

template <int DH>
bool mfma_ok(const AttnApplyArgs& a, bool bwd) {
  return a.nchunks >= mfma_min_chunks() && a.nsrc >= 1 && a.nsrc <= 8 && (a.ldq & 3) == 0 &&
         (!bwd || ((a.lddq & 3) == 0 && (a.lddu & 3) == 0)) && apply_lds_bytes<DH>(a.nsrc, a.H, bwd) <= kApplyLdsMax;
}

// the dynamic-LDS cap of a kernel, raised ONCE to the largest size any launch may ask for (it is a cap
// only: occupancy follows each launch's own size), not per launch
static void allow_max_lds(const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kApplyLdsMax); }

template <int DH, bool BWD>
hipError_t launch_mfma(const AttnApplyArgs& a, hipStream_t s) {
  const size_t lds = apply_lds_bytes<DH>(a.nsrc, a.H, BWD);
  static const bool attr = [] {
    allow_max_lds(BWD ? reinterpret_cast<const void*>(attn_apply_bwd_mfma_kernel<DH>)
                      : reinterpret_cast<const void*>(attn_apply_fwd_mfma_kernel<DH>));
    return true;
  }();
  (void)attr;
  const dim3 grid((a.nchunks + kApplyCpw - 1) / kApplyCpw), block(256);
  if (BWD) hipLaunchKernelGGL(attn_apply_bwd_mfma_kernel<DH>, grid, block, lds, s, a, kApplyCpw);
  else hipLaunchKernelGGL(attn_apply_fwd_mfma_kernel<DH>, grid, block, lds, s, a, kApplyCpw);
  return hipGetLastError();
}
}  // namespace

// returns hipErrorNotSupported when the head width / LDS size has no MFMA variant (caller falls back)
hipError_t launch_attn_apply_mfma(const AttnApplyArgs& a, bool bwd, hipStream_t s) {
  if (a.dhr != 0 && a.dhr != a.dh) return hipErrorNotSupported;   // padded heads: the VALU forms
  if (a.nchunks <= 0) return hipSuccess;
  switch (a.dh) {
    case 16: if (mfma_ok<16>(a, bwd)) return bwd ? launch_mfma<16, true>(a, s) : launch_mfma<16, false>(a, s); break;
    case 32: if (mfma_ok<32>(a, bwd)) return bwd ? launch_mfma<32, true>(a, s) : launch_mfma<32, false>(a, s); break;
    case 64: if (mfma_ok<64>(a, bwd)) return bwd ? launch_mfma<64, true>(a, s) : launch_mfma<64, false>(a, s); break;
    default: break;
  }
  return hipErrorNotSupported;
}

namespace {
template <int DH>
hipError_t launch_kv(const AttnKVBwdArgs* a, const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks, int H,
                     hipStream_t s) {
  const size_t lds = apply_lds_bytes<DH>(1, H, true);
  static const bool attr = [] {
    allow_max_lds(reinterpret_cast<const void*>(attn_kv_bwd_mfma_kernel<DH>));
    allow_max_lds(reinterpret_cast<const void*>(attn_kv_bwd_batch_mfma_kernel<DH>));
    return true;
  }();
  (void)attr;
  const int nch = a ? a->nchunks : maxchunks;
  const dim3 grid((nch + kApplyCpw - 1) / kApplyCpw, 1, a ? 1 : njobs), block(256);
  if (a) hipLaunchKernelGGL(attn_kv_bwd_mfma_kernel<DH>, grid, block, lds, s, *a, kApplyCpw);
  else hipLaunchKernelGGL(attn_kv_bwd_batch_mfma_kernel<DH>, grid, block, lds, s, jobs_dev, kApplyCpw);
  return hipGetLastError();
}
}  // namespace

// K/V backward on MFMA: `a` for one job, or (jobs_dev, njobs, maxchunks) for the batched form;
// hipErrorNotSupported when the head width / LDS size has no MFMA variant
hipError_t launch_attn_kv_bwd_mfma(const AttnKVBwdArgs* a, const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks,
                                   int H, int dh, hipStream_t s) {
  if (a && ((a->ldkv & 3) || (a->lddkv & 3))) return hipErrorNotSupported;
  if ((a ? a->nchunks : maxchunks * njobs) < mfma_min_chunks()) return hipErrorNotSupported;
  switch (dh) {
    case 16: if (apply_lds_bytes<16>(1, H, true) <= kApplyLdsMax) return launch_kv<16>(a, jobs_dev, njobs, maxchunks, H, s); break;
    case 32: if (apply_lds_bytes<32>(1, H, true) <= kApplyLdsMax) return launch_kv<32>(a, jobs_dev, njobs, maxchunks, H, s); break;
    case 64: if (apply_lds_bytes<64>(1, H, true) <= kApplyLdsMax) return launch_kv<64>(a, jobs_dev, njobs, maxchunks, H, s); break;
    default: break;
  }
  return hipErrorNotSupported;
}

}  // namespace gnot
