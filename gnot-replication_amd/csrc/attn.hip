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
// Work decomposition (all three kernels): a GROUP of G lanes owns one (point, head) pair; lane q of
// the group owns C = dh/G consecutive features 4-aligned (G = a power of two, so groups never
// straddle a wave and their reductions are shfl_xor butterflies).  Consecutive groups are
// consecutive heads of one point, so a wave's row reads/writes are contiguous.  grid.x = 64-point
// segment of one sample, grid.y splits the segment's (point, head, lane) tasks into 256-thread
// workgroups -> ~8x more waves than one thread per (point, head), which is what the chip needs at
// 10k-point meshes (the per-thread dependent FMA chains were latency-bound).  The (S, z) states are
// read through the L1/L2 (every group of one head reads the same 1 KiB).  Heads wider than 64 run the
// wide forms below (16 lanes per head, 4-feature quads dealt round-robin).
//
//   attn_apply_fwd  res (head-major)
//   attn_apply_bwd  du_i, dden_i per source, d(pre-softmax q)
//   attn_kv_bwd     d(pre-softmax k), dv from (dS, dz)
// The cross-point reductions themselves (S, z forward; dS, dz backward) are state.hip's
// state_partial + state_reduce (per-head fp32 VALU blocks over LDS-staged rows, fixed-order
// reduction of per-workgroup partials), one job per sample.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

// lanes per (point, head) for head width DH
constexpr int head_lanes(int q4) {   // largest power of two <= 16 dividing q4 = DH / 4
  int g = 16;
  while (g > 1 && q4 % g != 0) g >>= 1;
  return g;
}

template <int DH>
struct HeadSplit {
  static constexpr int G = head_lanes(DH / 4);
  static constexpr int C = DH / G;          // features owned per lane (multiple of 4)
  static_assert(C % 4 == 0 && C * G == DH, "head width must split into 4-aligned lane slices");
};

template <int G>
GNOT_DEV float group_sum(float v) {
#pragma unroll
  for (int m = 1; m < G; m <<= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// compiler-only fence: keeps the k-loop's state loads from being hoisted all at once (at dh >= 32 that
// pushes a lane past 128 VGPRs); one in-flight block of kRowBlock rows is enough latency cover
constexpr int kRowBlock = 16;
GNOT_DEV void row_block_fence(int k) {
  if ((k + 1) % kRowBlock == 0) asm volatile("" ::: "memory");
}

template <int N>
GNOT_DEV void load_vec(float (&dst)[N], const float* __restrict__ src) {
#pragma unroll
  for (int j = 0; j < N; j += 4) {
    const float4 v = *reinterpret_cast<const float4*>(src + j);
    dst[j] = v.x; dst[j + 1] = v.y; dst[j + 2] = v.z; dst[j + 3] = v.w;
  }
}

template <int N>
GNOT_DEV void store_vec(float* __restrict__ dst, const float (&v)[N]) {
#pragma unroll
  for (int j = 0; j < N; j += 4) *reinterpret_cast<float4*>(dst + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
}

// task decode: returns false for tasks past the segment's end (whole groups, so shuffles stay in-group)
struct Task {
  long n;      // global (packed) point index
  int h;       // head
  int q;       // lane within the group
};

template <int G>
GNOT_DEV bool decode_task(const int4& ch, int H, Task& t) {
  const int idx = blockIdx.y * 256 + threadIdx.x;
  const int grp = idx / G;
  if (grp >= ch.z * H) return false;
  t.q = idx % G;
  t.n = ch.y + grp / H;
  t.h = grp % H;
  return true;
}

// group-transposed row sums: lane q of a G-lane group holds v[k] = sum over ITS feature slice of
// row k (k = 0 .. DH-1); returns in v[0 .. C) the group total of rows q*C .. q*C+C-1 (a butterfly
// reduce-scatter: log2(G) shfl_xor stages, each halving the rows a lane carries).  This replaces
// re-reading whole state rows per lane: a group reads each (S, z) element exactly once.
template <int G, int C>
GNOT_DEV void group_reduce_scatter(float (&v)[G * C], int q) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) {
    const bool up = (q & m) != 0;
#pragma unroll
    for (int i = 0; i < m * C; ++i) {
      const float lo = v[i], hi = v[i + m * C];
      const float send = up ? lo : hi;
      const float keep = up ? hi : lo;
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
}

// den = q . z for the group's (point, head): each lane dots its own slice, then a group sum
// (qs = the lane's own q slice, loaded separately: indexing the full q[DH] registers at the
// lane-dependent offset c0 would compile to select chains)
template <int G, int C>
GNOT_DEV float group_den(const float (&qs)[C], const float* __restrict__ z, int c0) {
  float zs[C];
  load_vec<C>(zs, z + c0);
  float d = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) d = fmaf(qs[c], zs[c], d);
  return group_sum<G>(d);
}

// ---------------------------------------------------------------- apply (forward)
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_fwd_kernel(AttnApplyArgs a) {
  constexpr int G = HeadSplit<DH>::G, C = HeadSplit<DH>::C;
  constexpr int ph = DH * DH + DH;
  const int4 ch = a.chunks[blockIdx.x];
  Task t;
  if (!decode_task<G>(ch, a.H, t)) return;
  const int b = ch.x;
  const long off_b = a.off[b];
  const long Nb = a.off[b + 1] - off_b;
  const int c0 = t.q * C;
  float qf[DH], qs[C];
  load_vec<DH>(qf, a.q + t.n * a.ldq + t.h * DH);
  load_vec<C>(qs, a.q + t.n * a.ldq + t.h * DH + c0);
  float os[C];
#pragma unroll
  for (int c = 0; c < C; ++c) os[c] = 0.f;
  for (int s = 0; s < a.nsrc; ++s) {
    const float* S = a.state[s] + (long)b * a.H * ph + t.h * ph;
    const float den = group_den<G, C>(qs, S + DH * DH, c0);
    float u[C];
#pragma unroll
    for (int c = 0; c < C; ++c) u[c] = 0.f;
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      float srow[C];
      load_vec<C>(srow, S + k * DH + c0);
#pragma unroll
      for (int c = 0; c < C; ++c) u[c] = fmaf(qf[k], srow[c], u[c]);
      row_block_fence(k);
    }
    const float inv = 1.0f / den;
#pragma unroll
    for (int c = 0; c < C; ++c) os[c] = fmaf(u[c], inv, os[c]);
  }
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  float r[C];
#pragma unroll
  for (int c = 0; c < C; ++c) r[c] = fmaf(os[c], inv_nsrc, qs[c]);
  if (a.dhr == 0) {
    store_vec<C>(a.res + off_b * (long)a.H * DH + ((long)t.h * Nb + (t.n - off_b)) * DH + c0, r);
  } else {
    // padded heads: the scramble keeps the real head width (its rows are the model's); pad features dropped
    float* dst = a.res + off_b * (long)a.H * a.dhr + ((long)t.h * Nb + (t.n - off_b)) * a.dhr;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (c0 + c < a.dhr) dst[c0 + c] = r[c];
  }
}

// ---------------------------------------------------------------- apply (backward)
// dO = dres/nsrc; per source: o = u/den, du = dO/den, dden = -(dO.u)/den^2, dq += du S^T + dden z;
// dq starts at dres (the q residual); finally the feature-softmax backward of q.  One pass over the
// lane's column slice of S gives both u (columns) and the lane's share of S dO (rows, finished by
// the group reduce-scatter).
template <int DH>
__global__ void __launch_bounds__(256) attn_apply_bwd_kernel(AttnApplyArgs a) {
  constexpr int G = HeadSplit<DH>::G, C = HeadSplit<DH>::C;
  constexpr int ph = DH * DH + DH;
  const int4 ch = a.chunks[blockIdx.x];
  Task t;
  if (!decode_task<G>(ch, a.H, t)) return;
  const int b = ch.x;
  const long off_b = a.off[b];
  const long Nb = a.off[b + 1] - off_b;
  const int c0 = t.q * C;
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  float qf[DH], qs[C], dO[C];
  load_vec<DH>(qf, a.q + t.n * a.ldq + t.h * DH);
  load_vec<C>(qs, a.q + t.n * a.ldq + t.h * DH + c0);
  if (a.dhr == 0) {
    load_vec<C>(dO, a.dres + off_b * (long)a.H * DH + ((long)t.h * Nb + (t.n - off_b)) * DH + c0);
  } else {
    const float* src = a.dres + off_b * (long)a.H * a.dhr + ((long)t.h * Nb + (t.n - off_b)) * a.dhr;
#pragma unroll
    for (int c = 0; c < C; ++c) dO[c] = c0 + c < a.dhr ? src[c0 + c] : 0.f;
  }
  float dq[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    dq[c] = dO[c];
    dO[c] *= inv_nsrc;
  }
  for (int s = 0; s < a.nsrc; ++s) {
    const float* S = a.state[s] + (long)b * a.H * ph + t.h * ph;
    const float* z = S + DH * DH;
    const float den = group_den<G, C>(qs, z, c0);
    float u[C], part[DH];
#pragma unroll
    for (int c = 0; c < C; ++c) u[c] = 0.f;
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      float srow[C];
      load_vec<C>(srow, S + k * DH + c0);
      float pk = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        u[c] = fmaf(qf[k], srow[c], u[c]);
        pk = fmaf(dO[c], srow[c], pk);
      }
      part[k] = pk;
      row_block_fence(k);
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dot = fmaf(dO[c], u[c], dot);
    dot = group_sum<G>(dot);
    const float inv = 1.0f / den;
    const float dden = -dot * inv * inv;
    float du[C];
#pragma unroll
    for (int c = 0; c < C; ++c) du[c] = dO[c] * inv;
    store_vec<C>(a.du[s] + t.n * a.lddu + t.h * DH + c0, du);
    if (t.q == 0) a.dden[s][t.n * a.H + t.h] = dden;
    // dq[k] += (sum_j dO_j S[k][j]) / den + dden z[k] for this lane's rows k = c0 .. c0+C-1
    group_reduce_scatter<G, C>(part, t.q);
    float zs[C];
    load_vec<C>(zs, z + c0);
#pragma unroll
    for (int c = 0; c < C; ++c) dq[c] = fmaf(part[c], inv, fmaf(dden, zs[c], dq[c]));
  }
  float qdq = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) qdq = fmaf(qs[c], dq[c], qdq);
  qdq = group_sum<G>(qdq);
  float dpre[C];
#pragma unroll
  for (int c = 0; c < C; ++c) dpre[c] = qs[c] * (dq[c] - qdq);
  store_vec<C>(a.dq_pre + t.n * a.lddq + t.h * DH + c0, dpre);
}

// ---------------------------------------------------------------- K/V backward
// dk = dz + v dS^T, dv = k dS (per head), then the feature-softmax backward of k.  One pass over the
// lane's column slice of dS: dv (columns) directly, dk (rows) through the group reduce-scatter.
template <int DH>
GNOT_DEV void attn_kv_bwd_body(const AttnKVBwdArgs& a, const int4& ch) {
  constexpr int G = HeadSplit<DH>::G, C = HeadSplit<DH>::C;
  constexpr int ph = DH * DH + DH;
  Task t;
  if (!decode_task<G>(ch, a.H, t)) return;
  const int b = ch.x;
  const int c0 = t.q * C;
  const float* dS = a.dstate + (long)b * a.H * ph + t.h * ph;
  const float* dz = dS + DH * DH;
  float kf[DH], ks[C], vs[C];
  load_vec<DH>(kf, a.k + t.n * a.ldkv + t.h * DH);
  load_vec<C>(ks, a.k + t.n * a.ldkv + t.h * DH + c0);
  load_vec<C>(vs, a.v + t.n * a.ldkv + t.h * DH + c0);
  float dv[C], part[DH];
#pragma unroll
  for (int c = 0; c < C; ++c) dv[c] = 0.f;
#pragma unroll
  for (int i = 0; i < DH; ++i) {
    float srow[C];
    load_vec<C>(srow, dS + i * DH + c0);
    float pk = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      dv[c] = fmaf(kf[i], srow[c], dv[c]);
      pk = fmaf(vs[c], srow[c], pk);
    }
    part[i] = pk;
    row_block_fence(i);
  }
  group_reduce_scatter<G, C>(part, t.q);
  float dzs[C], dk[C];
  load_vec<C>(dzs, dz + c0);
#pragma unroll
  for (int c = 0; c < C; ++c) dk[c] = dzs[c] + part[c];
  float kdk = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) kdk = fmaf(ks[c], dk[c], kdk);
  kdk = group_sum<G>(kdk);
#pragma unroll
  for (int c = 0; c < C; ++c) dk[c] = ks[c] * (dk[c] - kdk);
  store_vec<C>(a.dk + t.n * a.lddkv + t.h * DH + c0, dk);
  store_vec<C>(a.dv + t.n * a.lddkv + t.h * DH + c0, dv);
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_kernel(AttnKVBwdArgs a) {
  attn_kv_bwd_body<DH>(a, a.chunks[blockIdx.x]);
}

template <int DH>
__global__ void __launch_bounds__(256) attn_kv_bwd_batch_kernel(const AttnKVBwdArgs* __restrict__ jobs) {
  const AttnKVBwdArgs& a = jobs[blockIdx.z];
  if ((int)blockIdx.x >= a.nchunks) return;
  attn_kv_bwd_body<DH>(a, a.chunks[blockIdx.x]);
}

// ---------------------------------------------------------------- wide heads (64 < dh <= 256)
// A 16-lane group per (point, head); lane q owns the 4-feature quads q, q + 16, q + 32, ... of the head
// (features 64 b + 4 q .. +3 for b < NB = ceil(dh / 64); a quad at or past dh is not owned), so every 64-row
// block of a state reduces with one 16-lane reduce-scatter (group_reduce_scatter<16, 4>) that lands row
// 64 b + 4 q + j in the lane that owns feature 64 b + 4 q + j.  The q / k row is read 4 features at a time
// through the L1 (the group shares it) instead of being held whole in registers as above: 2 dh floats per
// lane do not fit beside the rest at dh = 256.  dh is a runtime multiple of 4; the per-column k order of
// the sums is the narrow kernels'.
constexpr int kWideG = 16;

template <int NB>
struct WideSlice {
  int q, dh;
  GNOT_DEV bool own(int b) const { return 64 * b + 4 * q < dh; }
  GNOT_DEV int f(int b) const { return 64 * b + 4 * q; }
};

template <int NB>
GNOT_DEV void wide_load(float (&v)[NB][4], const float* __restrict__ row, const WideSlice<NB>& w) {
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float4 x = w.own(b) ? *reinterpret_cast<const float4*>(row + w.f(b)) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[b][0] = x.x; v[b][1] = x.y; v[b][2] = x.z; v[b][3] = x.w;
  }
}

template <int NB>
GNOT_DEV void wide_store(float* __restrict__ row, const float (&v)[NB][4], const WideSlice<NB>& w) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
    if (w.own(b)) *reinterpret_cast<float4*>(row + w.f(b)) = make_float4(v[b][0], v[b][1], v[b][2], v[b][3]);
}

template <int NB>
GNOT_DEV float wide_dot(const float (&x)[NB][4], const float (&y)[NB][4]) {
  float d = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) d = fmaf(x[b][c], y[b][c], d);
  return d;
}

template <int NB>
GNOT_DEV void wide_zero(float (&v)[NB][4]) {
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) v[b][c] = 0.f;
}

// one pass over rows [64 kb, 64 kb + 64) of a state M (pitch dh): acc[b][c] += x[k] M[k][f(b) + c] (the lane's
// columns) and rows[j] = sum over the whole group of y . M[64 kb + 4 q + j][:] (the lane's rows)
template <int NB>
GNOT_DEV void wide_rows(const float* __restrict__ M, const float* __restrict__ xrow, const float (&y)[NB][4], int kb,
                        const WideSlice<NB>& w, float (&acc)[NB][4], float (&rows)[4]) {
  float part[64];
#pragma unroll
  for (int i4 = 0; i4 < 16; ++i4) {
    const int k0 = 64 * kb + 4 * i4;
    if (k0 < w.dh) {
      const float4 x4 = *reinterpret_cast<const float4*>(xrow + k0);
      const float xk[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sr[NB][4];
        wide_load(sr, M + (long)(k0 + r) * w.dh, w);
        float pk = 0.f;
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            acc[b][c] = fmaf(xk[r], sr[b][c], acc[b][c]);
            pk = fmaf(y[b][c], sr[b][c], pk);
          }
        part[4 * i4 + r] = pk;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) part[4 * i4 + r] = 0.f;
    }
  }
  group_reduce_scatter<kWideG, 4>(part, w.q);
#pragma unroll
  for (int j = 0; j < 4; ++j) rows[j] = part[j];
}

template <int NB>
__global__ void __launch_bounds__(256) attn_apply_fwd_wide_kernel(AttnApplyArgs a) {
  const int4 ch = a.chunks[blockIdx.x];
  Task t;
  if (!decode_task<kWideG>(ch, a.H, t)) return;
  const int dh = a.dh;
  const long ph = (long)dh * dh + dh;
  const WideSlice<NB> w{t.q, dh};
  const int sb = ch.x;
  const long off_b = a.off[sb];
  const long Nb = a.off[sb + 1] - off_b;
  const float* qrow = a.q + t.n * a.ldq + (long)t.h * dh;
  float qs[NB][4], os[NB][4];
  wide_load(qs, qrow, w);
  wide_zero(os);
  for (int s = 0; s < a.nsrc; ++s) {
    const float* S = a.state[s] + (long)sb * a.H * ph + t.h * ph;
    float zs[NB][4], u[NB][4];
    wide_load(zs, S + (long)dh * dh, w);
    const float den = group_sum<kWideG>(wide_dot(qs, zs));
    wide_zero(u);
    for (int k0 = 0; k0 < dh; k0 += 4) {
      const float4 q4 = *reinterpret_cast<const float4*>(qrow + k0);
      const float qk[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sr[NB][4];
        wide_load(sr, S + (long)(k0 + r) * dh, w);
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int c = 0; c < 4; ++c) u[b][c] = fmaf(qk[r], sr[b][c], u[b][c]);
      }
    }
    const float inv = 1.0f / den;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) os[b][c] = fmaf(u[b][c], inv, os[b][c]);
  }
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  float r[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) r[b][c] = fmaf(os[b][c], inv_nsrc, qs[b][c]);
  if (a.dhr == 0) {
    wide_store(a.res + off_b * (long)a.H * dh + ((long)t.h * Nb + (t.n - off_b)) * dh, r, w);
  } else {
    float* dst = a.res + off_b * (long)a.H * a.dhr + ((long)t.h * Nb + (t.n - off_b)) * a.dhr;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (w.f(b) + c < a.dhr) dst[w.f(b) + c] = r[b][c];
  }
}

template <int NB>
__global__ void __launch_bounds__(256) attn_apply_bwd_wide_kernel(AttnApplyArgs a) {
  const int4 ch = a.chunks[blockIdx.x];
  Task t;
  if (!decode_task<kWideG>(ch, a.H, t)) return;
  const int dh = a.dh;
  const long ph = (long)dh * dh + dh;
  const WideSlice<NB> w{t.q, dh};
  const int sb = ch.x;
  const long off_b = a.off[sb];
  const long Nb = a.off[sb + 1] - off_b;
  const float inv_nsrc = 1.0f / (float)a.nsrc;
  const float* qrow = a.q + t.n * a.ldq + (long)t.h * dh;
  float qs[NB][4], dO[NB][4], dq[NB][4];
  wide_load(qs, qrow, w);
  if (a.dhr == 0) {
    wide_load(dO, a.dres + off_b * (long)a.H * dh + ((long)t.h * Nb + (t.n - off_b)) * dh, w);
  } else {
    const float* src = a.dres + off_b * (long)a.H * a.dhr + ((long)t.h * Nb + (t.n - off_b)) * a.dhr;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) dO[b][c] = w.f(b) + c < a.dhr ? src[w.f(b) + c] : 0.f;
  }
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      dq[b][c] = dO[b][c];
      dO[b][c] *= inv_nsrc;
    }
  for (int s = 0; s < a.nsrc; ++s) {
    const float* S = a.state[s] + (long)sb * a.H * ph + t.h * ph;
    float zs[NB][4], u[NB][4], pr[NB][4];
    wide_load(zs, S + (long)dh * dh, w);
    const float den = group_sum<kWideG>(wide_dot(qs, zs));
    wide_zero(u);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) wide_rows(S, qrow, dO, kb, w, u, pr[kb]);
    const float dot = group_sum<kWideG>(wide_dot(dO, u));
    const float inv = 1.0f / den;
    const float dden = -dot * inv * inv;
    float du[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) du[b][c] = dO[b][c] * inv;
    wide_store(a.du[s] + t.n * a.lddu + (long)t.h * dh, du, w);
    if (t.q == 0) a.dden[s][t.n * a.H + t.h] = dden;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) dq[b][c] = fmaf(pr[b][c], inv, fmaf(dden, zs[b][c], dq[b][c]));
  }
  const float qdq = group_sum<kWideG>(wide_dot(qs, dq));
  float dpre[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) dpre[b][c] = qs[b][c] * (dq[b][c] - qdq);
  wide_store(a.dq_pre + t.n * a.lddq + (long)t.h * dh, dpre, w);
}

template <int NB>
GNOT_DEV void attn_kv_bwd_wide_body(const AttnKVBwdArgs& a, const int4& ch) {
  Task t;
  if (!decode_task<kWideG>(ch, a.H, t)) return;
  const int dh = a.dh;
  const long ph = (long)dh * dh + dh;
  const WideSlice<NB> w{t.q, dh};
  const float* dS = a.dstate + (long)ch.x * a.H * ph + t.h * ph;
  const float* krow = a.k + t.n * a.ldkv + (long)t.h * dh;
  float ks[NB][4], vs[NB][4], dv[NB][4], pr[NB][4], dk[NB][4];
  wide_load(ks, krow, w);
  wide_load(vs, a.v + t.n * a.ldkv + (long)t.h * dh, w);
  wide_zero(dv);
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) wide_rows(dS, krow, vs, kb, w, dv, pr[kb]);
  wide_load(dk, dS + (long)dh * dh, w);
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) dk[b][c] += pr[b][c];
  const float kdk = group_sum<kWideG>(wide_dot(ks, dk));
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < 4; ++c) dk[b][c] = ks[b][c] * (dk[b][c] - kdk);
  wide_store(a.dk + t.n * a.lddkv + (long)t.h * dh, dk, w);
  wide_store(a.dv + t.n * a.lddkv + (long)t.h * dh, dv, w);
}

template <int NB>
__global__ void __launch_bounds__(256) attn_kv_bwd_wide_kernel(AttnKVBwdArgs a) {
  attn_kv_bwd_wide_body<NB>(a, a.chunks[blockIdx.x]);
}

template <int NB>
__global__ void __launch_bounds__(256) attn_kv_bwd_wide_batch_kernel(const AttnKVBwdArgs* __restrict__ jobs) {
  const AttnKVBwdArgs& a = jobs[blockIdx.z];
  if ((int)blockIdx.x >= a.nchunks) return;
  attn_kv_bwd_wide_body<NB>(a, a.chunks[blockIdx.x]);
}

// workgroups per 64-point segment of the wide forms: 64 H groups of 16 lanes
static unsigned wide_split(int H) { return (unsigned)((64 * H * kWideG + 255) / 256); }

#define GNOT_WIDE_SWITCH(DHV, ...)                                            \
  switch ((DHV + 63) / 64) {                                                  \
    case 2: { constexpr int NB = 2; __VA_ARGS__; } break;                     \
    case 3: { constexpr int NB = 3; __VA_ARGS__; } break;                     \
    case 4: { constexpr int NB = 4; __VA_ARGS__; } break;                     \
    default: return hipErrorInvalidValue;                                     \
  }

#define GNOT_DH_SWITCH(DHV, ...)        \
  switch (DHV) {                        \
    case 4: { constexpr int DH = 4; __VA_ARGS__; } break;    \
    case 8: { constexpr int DH = 8; __VA_ARGS__; } break;    \
    case 12: { constexpr int DH = 12; __VA_ARGS__; } break;  \
    case 16: { constexpr int DH = 16; __VA_ARGS__; } break;  \
    case 20: { constexpr int DH = 20; __VA_ARGS__; } break;  \
    case 24: { constexpr int DH = 24; __VA_ARGS__; } break;  \
    case 28: { constexpr int DH = 28; __VA_ARGS__; } break;  \
    case 32: { constexpr int DH = 32; __VA_ARGS__; } break;  \
    case 36: { constexpr int DH = 36; __VA_ARGS__; } break;  \
    case 40: { constexpr int DH = 40; __VA_ARGS__; } break;  \
    case 44: { constexpr int DH = 44; __VA_ARGS__; } break;  \
    case 48: { constexpr int DH = 48; __VA_ARGS__; } break;  \
    case 52: { constexpr int DH = 52; __VA_ARGS__; } break;  \
    case 56: { constexpr int DH = 56; __VA_ARGS__; } break;  \
    case 60: { constexpr int DH = 60; __VA_ARGS__; } break;  \
    case 64: { constexpr int DH = 64; __VA_ARGS__; } break;  \
    default: return hipErrorInvalidValue;                    \
  }

// workgroups per 64-point segment: ceil(64 * H * G / 256)
template <int DH>
static unsigned seg_split(int H) {
  return (unsigned)((64 * H * HeadSplit<DH>::G + 255) / 256);
}

hipError_t launch_attn_apply_fwd(const AttnApplyArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const hipError_t m = launch_attn_apply_mfma(a, false, s);   // attn_mfma.hip where it applies
  if (m != hipErrorNotSupported) return m;
  if (a.dh > 64) {
    if (a.dh % 4 != 0) return hipErrorInvalidValue;
    GNOT_WIDE_SWITCH(a.dh, hipLaunchKernelGGL(attn_apply_fwd_wide_kernel<NB>, dim3(a.nchunks, wide_split(a.H)),
                                              dim3(256), 0, s, a));
    return hipGetLastError();
  }
  GNOT_DH_SWITCH(a.dh, hipLaunchKernelGGL(attn_apply_fwd_kernel<DH>, dim3(a.nchunks, seg_split<DH>(a.H)), dim3(256),
                                          0, s, a));
  return hipGetLastError();
}

hipError_t launch_attn_apply_bwd(const AttnApplyArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const hipError_t m = launch_attn_apply_mfma(a, true, s);
  if (m != hipErrorNotSupported) return m;
  if (a.dh > 64) {
    if (a.dh % 4 != 0) return hipErrorInvalidValue;
    GNOT_WIDE_SWITCH(a.dh, hipLaunchKernelGGL(attn_apply_bwd_wide_kernel<NB>, dim3(a.nchunks, wide_split(a.H)),
                                              dim3(256), 0, s, a));
    return hipGetLastError();
  }
  GNOT_DH_SWITCH(a.dh, hipLaunchKernelGGL(attn_apply_bwd_kernel<DH>, dim3(a.nchunks, seg_split<DH>(a.H)), dim3(256),
                                          0, s, a));
  return hipGetLastError();
}

hipError_t launch_attn_kv_bwd(const AttnKVBwdArgs& a, hipStream_t s) {
  if (a.nchunks <= 0) return hipSuccess;
  const hipError_t m = launch_attn_kv_bwd_mfma(&a, nullptr, 1, a.nchunks, a.H, a.dh, s);
  if (m != hipErrorNotSupported) return m;
  if (a.dh > 64) {
    if (a.dh % 4 != 0) return hipErrorInvalidValue;
    GNOT_WIDE_SWITCH(a.dh, hipLaunchKernelGGL(attn_kv_bwd_wide_kernel<NB>, dim3(a.nchunks, wide_split(a.H)),
                                              dim3(256), 0, s, a));
    return hipGetLastError();
  }
  GNOT_DH_SWITCH(a.dh, hipLaunchKernelGGL(attn_kv_bwd_kernel<DH>, dim3(a.nchunks, seg_split<DH>(a.H)), dim3(256), 0,
                                          s, a));
  return hipGetLastError();
}

hipError_t launch_attn_kv_bwd_batch(const AttnKVBwdArgs* jobs_dev, int njobs, int maxchunks, int H, int dh,
                                    hipStream_t s) {
  if (njobs <= 0 || maxchunks <= 0) return hipSuccess;
  // the batched jobs' pitches are 4-aligned by construction (rows of d floats)
  const hipError_t m = launch_attn_kv_bwd_mfma(nullptr, jobs_dev, njobs, maxchunks, H, dh, s);
  if (m != hipErrorNotSupported) return m;
  if (dh > 64) {
    if (dh % 4 != 0) return hipErrorInvalidValue;
    GNOT_WIDE_SWITCH(dh, hipLaunchKernelGGL(attn_kv_bwd_wide_batch_kernel<NB>, dim3(maxchunks, wide_split(H), njobs),
                                            dim3(256), 0, s, jobs_dev));
    return hipGetLastError();
  }
  GNOT_DH_SWITCH(dh, hipLaunchKernelGGL(attn_kv_bwd_batch_kernel<DH>, dim3(maxchunks, seg_split<DH>(H), njobs),
                                        dim3(256), 0, s, jobs_dev));
  return hipGetLastError();
}

}  // namespace gnot
