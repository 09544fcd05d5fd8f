// Point-reduction GEMM:  C = sum_p A[p]^T B[p]  (+ column sums of A)  over a point range.
//
// Two users, one kernel:
//  * weight gradients of every Linear: dW = sum_p dZ[p]^T X[p], db = sum_p dZ[p] (the autograd of
//    nn.Linear, reference model.py:9-14 / 43-51 behind main.py:102).  X may be a saved
//    PRE-activation, GELU'd on load (the input of hidden Linear l is gelu(h_{l-1}), model.py:10-13).
//  * the linear-attention state of one sample: S = sum_m k_m^T v_m, z = sum_m k_m (model.py:77,79)
//    and in the backward dS = sum_n q_n^T du_n, dz = sum_n dden_n q_n.  The GEMM computes the full
//    128x128 tile and the reduce pass keeps only the per-head dh x dh diagonal blocks.
//
// Layout: one workgroup (4 waves) owns a 128x128 output tile of one job and one chunk of points.
// Per stage kStage = 32 points of A and B rows (2 x 16 KiB, coalesced 16-B loads, GELU applied while
// staging) go to LDS; the NEXT stage's rows are already in flight in registers while the current one
// is consumed.  Each wave computes a 64x64 quadrant with v_mfma_f32_32x32x2_f32 (2 points per MFMA
// k-step, 4 MFMAs per pair of A/B fragment loads).  Partial tiles go to a slab; the reduce pass sums
// the splits in a fixed order (deterministic, no atomics).
#include <cstdlib>
#include <type_traits>

#include "gnot_common.h"
#include "gnot_kernels.h"
#include "x6_core.h"

namespace gnot {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;       // output tile edge
constexpr int kStage = 32;       // points per LDS stage
constexpr int kLdsRow = kTile;   // floats per staged row

GNOT_DEV int find_job(const int* __restrict__ prefix, int njobs, int idx) {
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Staging geometry: thread t owns column group c4 = t & 31 (columns 4*c4 .. 4*c4+3 of the tile) and
// rows r0 + 8k (r0 = t >> 5, k < kStage / 8) of each stage, for both A and B (64 points measured no faster).
struct StageRegs {
  float4 a[kStage / 8], b[kStage / 8];
};

GNOT_DEV float4 load4(const float* __restrict__ base, long p, long ld, int c, int ncols, bool pv) {
  if (!pv) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (c + 3 < ncols && (ld & 3) == 0) return *reinterpret_cast<const float4*>(base + p * ld + c);
  float t[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) t[r] = (c + r < ncols) ? base[p * ld + c + r] : 0.f;
  return make_float4(t[0], t[1], t[2], t[3]);
}

GNOT_DEV void stage_load(StageRegs& R, const WgradJob& J, long pbase, long pend, int co, int ci, int r0) {
#pragma unroll
  for (int k = 0; k < kStage / 8; ++k) {
    const long p = pbase + r0 + 8 * k;
    const bool pv = p < pend;
    R.a[k] = load4(J.dz, p, J.lddz, co, J.out, pv);
    R.b[k] = load4(J.x, p, J.ldx, ci, J.in, pv);
  }
}

__global__ void __launch_bounds__(256) pgemm_kernel(const WgradJob* __restrict__ jobs, const int* __restrict__ prefix,
                                                    int njobs, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float smem[2 * kStage * kLdsRow];
  float* As = smem;
  float* Bs = smem + kStage * kLdsRow;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = find_job(prefix, njobs, blockIdx.x);
  const WgradJob J = jobs[j];
  int t = blockIdx.x - prefix[j];
  const int split = t % J.splits;
  t /= J.splits;
  int to, ti;
  if (J.diag_only) { to = t; ti = t; } else { ti = t % J.tiles_i; to = t / J.tiles_i; }
  const int chunk = ((J.P + J.splits - 1) / J.splits + kStage - 1) / kStage * kStage;
  const long pb = (long)split * chunk;
  const long pe = min((long)J.P, pb + chunk);
  const int c0o = to * kTile, c0i = ti * kTile;
  const int wo = wave >> 1, wi = wave & 1;      // 64x64 quadrant of this wave
  const int r32 = lane & 31, h = lane >> 5;
  const int c4 = tid & 31, r0 = tid >> 5;       // staging role
  const int co = c0o + 4 * c4, ci = c0i + 4 * c4;
  const bool want_db = (J.db != nullptr) && (J.diag_only || ti == 0);
  const bool use_w = J.w != nullptr;
  const bool gel = J.x_gelu != 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float4 dbacc = make_float4(0.f, 0.f, 0.f, 0.f);   // column sums of this thread's A columns

  StageRegs R;
  if (pb < pe) stage_load(R, J, pb, pe, co, ci, r0);
  for (long p0 = pb; p0 < pe; p0 += kStage) {
    __syncthreads();                          // previous stage fully consumed
#pragma unroll
    for (int k = 0; k < kStage / 8; ++k) {
      const int row = r0 + 8 * k;
      float4 vb = R.b[k];
      if (gel) { vb.x = gelu(vb.x); vb.y = gelu(vb.y); vb.z = gelu(vb.z); vb.w = gelu(vb.w); }
      reinterpret_cast<float4*>(As)[row * 32 + c4] = R.a[k];
      reinterpret_cast<float4*>(Bs)[row * 32 + c4] = vb;
      if (want_db) {
        const long p = p0 + row;
        const float wgt = (use_w && p < pe && co < J.out) ? J.w[p * J.ldw + co / J.wdh] : 1.f;
        dbacc.x = fmaf(wgt, R.a[k].x, dbacc.x);
        dbacc.y = fmaf(wgt, R.a[k].y, dbacc.y);
        dbacc.z = fmaf(wgt, R.a[k].z, dbacc.z);
        dbacc.w = fmaf(wgt, R.a[k].w, dbacc.w);
      }
    }
    __syncthreads();
    if (p0 + kStage < pe) stage_load(R, J, p0 + kStage, pe, co, ci, r0);   // in flight during MFMAs
    // 16 k-steps (2 points each) in four batches of 4: fragment reads first, then 16 MFMAs
#pragma unroll
    for (int half = 0; half < kStage / 8; ++half) {
      float a0[4], a1[4], b0[4], b1[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = 2 * (4 * half + s) + h;
        const float* ar = As + row * kLdsRow + wo * 64 + r32;
        const float* br = Bs + row * kLdsRow + wi * 64 + r32;
        a0[s] = ar[0]; a1[s] = ar[32];
        b0[s] = br[0]; b1[s] = br[32];
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the 8 LDS reads batched ahead of the 16 MFMAs
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc[1][1], 0, 0, 0);
      }
    }
  }

  // partial tile -> slab [split][tile 128 x (128 + 1)]
  const int ntile = J.diag_only ? J.tiles_o : J.tiles_o * J.tiles_i;
  const int tile = J.diag_only ? to : to * J.tiles_i + ti;
  float* S = slab + J.slab_off + ((long)split * ntile + tile) * (kTile * (kTile + 1));
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wo * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wi * 64 + b * 32 + r32;
        S[row * (kTile + 1) + col] = acc[a][b][r];
      }
  if (want_db) {
    // sum the 8 row-owners of every column group through LDS (reuses the A stage buffer)
    __syncthreads();
    reinterpret_cast<float4*>(As)[r0 * 32 + c4] = dbacc;
    __syncthreads();
    if (r0 == 0) {
      float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float4 v = reinterpret_cast<const float4*>(As)[k * 32 + c4];
        tot.x += v.x; tot.y += v.y; tot.z += v.z; tot.w += v.w;
      }
      S[(4 * c4 + 0) * (kTile + 1) + kTile] = tot.x;
      S[(4 * c4 + 1) * (kTile + 1) + kTile] = tot.y;
      S[(4 * c4 + 2) * (kTile + 1) + kTile] = tot.z;
      S[(4 * c4 + 3) * (kTile + 1) + kTile] = tot.w;
    }
  }
}

// ---------------------------------------------------------------- bf16x6 variant (plain weight-gradient jobs)
// Same tiling, split-K and slab as pgemm_kernel, on v_mfma_f32_32x32x16_bf16: every staged fp32 value
// is split exactly into three bf16 pieces (split8_x6) and each 32x32x16 block product is the six
// order <= 2 piece products, accumulated in fp32 (the dropped terms are ~2^-24 relative: fp32-level,
// like the forward chains; one accumulator per block keeps two workgroups per CU within the register
// file): 6 x 32 = 192 matrix-pipe cycles per 32x32x16 block
// instead of 8 x 64 = 512 on v_mfma_f32_32x32x2_f32.
// Staging: thread (pair fp = t & 63, octet o = t >> 6 = its wave) loads features 2fp, 2fp+1 of the
// stage's points 8o .. 8o+7 (one float2 per point: a wave reads whole 512-byte rows), so 8 consecutive
// points of one feature are register-local and go to LDS as one 16-byte vector per piece.  The LDS
// image is [operand][piece][feature][point] with an 80-byte feature row (32 points + pad): the MFMA
// fragment read (lane = feature, 8 consecutive points) is a conflict-free ds_read_b128.
constexpr int kX6Stage = 32;                 // points per stage = two 16-point MFMA k-steps
constexpr int kX6Row = 40;                   // bf16 per staged feature row (80 B)
constexpr int kX6Piece = kTile * kX6Row;     // bf16 per (operand, piece) image

// global-address-space view of a job pointer (the pointers come from a job table, so the compiler
// cannot infer it and would emit flat loads, which also count against lgkmcnt)
#if defined(__HIP_DEVICE_COMPILE__)
#define GNOT_GLOBAL __attribute__((address_space(1)))
#else
#define GNOT_GLOBAL
#endif
typedef const float GNOT_GLOBAL* gfloat_ptr;
typedef const float2 GNOT_GLOBAL* gfloat2_ptr;

// 8 points x 2 features of one operand: v[j][k] = rows[p_k][f0 + j]; rows past `pe` and features
// past `ncols` read as 0.  Edge path: clamped (always valid) addresses plus selects, no branches
// per load; the row clamp is wave-uniform (prow is per wave).
GNOT_DEV void x6_load8x2(float (&v)[2][8], const float* base, long ld, long prow, long pe, int f0, int ncols,
                         bool full, bool vec) {
  gfloat_ptr g = (gfloat_ptr)base;
  if (full && vec) {
    gfloat_ptr r = g + prow * ld + f0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float2 x = *(gfloat2_ptr)(r + k * ld);
      v[0][k] = x.x;
      v[1][k] = x.y;
    }
    return;
  }
  const int c0 = min(f0, ncols - 1), c1 = min(f0 + 1, ncols - 1);
  const bool ok0 = f0 < ncols, ok1 = f0 + 1 < ncols;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const long p = min(prow + k, pe - 1);
    const bool pv = prow + k < pe;
    gfloat_ptr r = g + p * ld;
    const float x0 = r[c0], x1 = r[c1];
    v[0][k] = (pv && ok0) ? x0 : 0.f;
    v[1][k] = (pv && ok1) ? x1 : 0.f;
  }
}

GNOT_DEV void x6_mfma6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16& c) {
#define GNOT_MFMA32(X, Y) \
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, X), __builtin_bit_cast(bf16x8, Y), c, 0, 0, 0)
  GNOT_MFMA32(a[2], b[0]);
  GNOT_MFMA32(a[1], b[1]);
  GNOT_MFMA32(a[0], b[2]);
  GNOT_MFMA32(a[1], b[0]);
  GNOT_MFMA32(a[0], b[1]);
  GNOT_MFMA32(a[0], b[0]);
#undef GNOT_MFMA32
}
template <int NP>
GNOT_DEV void mfma_np(const u32x4 (&a)[NP], const u32x4 (&b)[NP], f32x16& c) {
  if constexpr (NP == 3) x6_mfma6(a, b, c);
  else c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[0]), __builtin_bit_cast(bf16x8, b[0]), c, 0, 0, 0);
}

// NP = 1 (bf16 mode): one RNE bf16 piece per operand and one MFMA per 32x32x16 block
template <int NP>
__global__ void __launch_bounds__(256) pgemm_x6_kernel(const WgradJob* __restrict__ jobs,
                                                       const int* __restrict__ prefix, int njobs,
                                                       float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * NP * kX6Piece];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = find_job(prefix, njobs, blockIdx.x);
  const WgradJob J = jobs[j];
  int t = blockIdx.x - prefix[j];
  const int split = t % J.splits;
  t /= J.splits;
  const int ti = t % J.tiles_i, to = t / J.tiles_i;
  const int chunk = ((J.P + J.splits - 1) / J.splits + kX6Stage - 1) / kX6Stage * kX6Stage;
  const long pb = (long)split * chunk;
  const long pe = min((long)J.P, pb + chunk);
  const int wo = wave >> 1, wi = wave & 1;      // 64x64 quadrant of this wave
  const int r32 = lane & 31, h = lane >> 5;
  const int fp = lane, o = wave;                // staging role
  const int fo = to * kTile + 2 * fp, fi = ti * kTile + 2 * fp;
  // float2 fast path: the whole tile inside the operand's columns and 8-byte aligned rows
  const bool tile_a = to * kTile + kTile <= J.out && (J.lddz & 1) == 0 && (reinterpret_cast<size_t>(J.dz) & 7) == 0;
  const bool tile_b = ti * kTile + kTile <= J.in && (J.ldx & 1) == 0 && (reinterpret_cast<size_t>(J.x) & 7) == 0;
  const bool want_db = (J.db != nullptr) && ti == 0;
  const bool gel = J.x_gelu != 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float dbacc[2] = {0.f, 0.f};

  float ra[2][8], rb[2][8];
  auto load_stage = [&](long pbase) {
    const long prow = pbase + 8 * o;
    const bool full = prow + 7 < pe;
    x6_load8x2(ra, J.dz, J.lddz, prow, pe, fo, J.out, full, tile_a);
    x6_load8x2(rb, J.x, J.ldx, prow, pe, fi, J.in, full, tile_b);
  };

  if (pb < pe) load_stage(pb);
  for (long p0 = pb; p0 < pe; p0 += kX6Stage) {
    __syncthreads();                          // previous stage fully consumed
#pragma unroll
    for (int jf = 0; jf < 2; ++jf) {
      float vb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        vb[k] = gel ? gelu(rb[jf][k]) : rb[jf][k];
        dbacc[jf] += ra[jf][k];
      }
      u32x4 pa[NP], pbv[NP];
      split8_np<NP>(ra[jf], pa);
      split8_np<NP>(vb, pbv);
      const int f = 2 * fp + jf;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        *reinterpret_cast<u32x4*>(lds + q * kX6Piece + f * kX6Row + 8 * o) = pa[q];
        *reinterpret_cast<u32x4*>(lds + (NP + q) * kX6Piece + f * kX6Row + 8 * o) = pbv[q];
      }
      asm volatile("" ::: "memory");          // one feature at a time: bounds the staging registers
    }
    __syncthreads();
    if (p0 + kX6Stage < pe) load_stage(p0 + kX6Stage);   // in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int koff = 16 * ks + 8 * h;
      u32x4 af[2][NP], bf[2][NP];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          af[a][q] = *reinterpret_cast<const u32x4*>(lds + q * kX6Piece + (wo * 64 + a * 32 + r32) * kX6Row + koff);
          bf[a][q] = *reinterpret_cast<const u32x4*>(lds + (NP + q) * kX6Piece + (wi * 64 + a * 32 + r32) * kX6Row + koff);
        }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) mfma_np<NP>(af[a], bf[b], acc[a][b]);   // smallest terms first
      asm volatile("" ::: "memory");          // k-step 1's fragments are not hoisted over k-step 0
    }
  }

  // partial tile -> slab [split][tile 128 x (128 + 1)] (same layout as pgemm_kernel)
  const int ntile = J.tiles_o * J.tiles_i;
  const int tile = to * J.tiles_i + ti;
  float* S = slab + J.slab_off + ((long)split * ntile + tile) * (kTile * (kTile + 1));
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wo * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wi * 64 + b * 32 + r32;
        S[row * (kTile + 1) + col] = acc[a][b][r];
      }
  if (want_db) {
    // column sums of A: the four point octets of every feature through LDS, in a fixed order
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
    red[o * kTile + 2 * fp] = dbacc[0];
    red[o * kTile + 2 * fp + 1] = dbacc[1];
    __syncthreads();
    if (tid < kTile) S[tid * (kTile + 1) + kTile] = (red[tid] + red[kTile + tid]) + (red[2 * kTile + tid] + red[3 * kTile + tid]);
  }
}

// ---------------------------------------------------------------- wide bf16x6 variant (d = 256 weight gradients)
// One workgroup owns a job's WHOLE 256 x 256 output (out, in <= 256) for one split-K point range, so
// every staged dZ / X value is loaded, GELU'd and split exactly once (the 128 x 128 kernel above
// stages each value twice and splits it on the same wave that issues the MFMAs).  8 waves, two per
// SIMD (<= 256 registers each: the accumulators are 8 32x32 blocks = 128 AGPRs), so one wave's
// staging VALU runs beside its partner's MFMAs.
//   rows:    the raw fp32 rows of a 16-point stage land by LDS-DMA in a ring PRIVATE to each wave: wave w
//            stages features 64 (w & 3) .. +63 of points 8 (w >> 2) .. +7 and brings exactly those 8 x 64
//            values of each operand (2 wave-instructions of 1 KiB per operand), so no barrier hands them
//            over and its slot is refilled as soon as its own reads of it have returned.  Two slots: stage
//            s + 3 is requested while stage s is multiplied and read at the top of iteration s + 2 (the
//            HBM latency of the row loads, the kernel's first limiter, DESIGN.md section 5.2, gets two
//            iterations instead of one, and the raw rows in flight hold no registers).
//   staging: thread t owns feature f = t & 255 and point half h = t >> 8 of a stage, for both operands:
//            mask, column sum, GELU, then 3 bf16 pieces of 8 consecutive points = three 16-byte LDS stores.
//   LDS:     per (buffer, operand, piece) a fragment-order image of 8 row blocks x 64 lanes x 16 B:
//            lane (r, h) of block rb holds rows 32 rb + r, points 8h .. 8h+7 -- the A/B operand layout of
//            v_mfma_f32_32x32x16_bf16, so fragment reads are contiguous 1 KiB ds_read_b128.
//   MFMA:    wave (wr, wc) computes rows [128 wr, +128) x cols [64 wc, +64): 4 x 2 blocks, six order <= 2
//            piece products each (smallest first), one accumulator per block.
// Double-buffered fragment images: stage s+1 is split into the other buffer while stage s is multiplied.
// Partials go to the same slab layout as pgemm_kernel (128-tiles).
// TW = 128 (round 5): the same kernel at d <= 128 (configs[1]) with a 128 x 128 output per workgroup and 4
// waves (one 64 x 64 quadrant each, 2 x 2 blocks), in place of the 128-tile kernel above, whose staging and
// MFMAs run as separate phases on one wave per SIMD.
constexpr int kWStage = 16;
constexpr int kWThreads = 512;                   // TW = 256; TW = 128: 256
constexpr int w_threads(int tw) { return tw * 2; }
constexpr int w_piece(int tw) { return tw / 32 * 64; }   // u32x4 per (operand, piece) image
// one stage buffer: A pieces 0..NP-1 | B pieces 0..NP-1 (NP = 3: bf16x6, 1: bf16 mode)
constexpr int w_buf(int np, int tw = 256) { return 2 * np * w_piece(tw); }
constexpr int kWRawSlot = 2 * 2 * 64;            // u32x4 per wave-private raw slot: 2 operands x 2 KiB
constexpr int kWRawSlots = 2;
// LDS: two fragment buffers | waves x 2 raw slots (96 + 64 = 160 KiB at NP = 3, TW = 256; 48 + 32 at 128)
constexpr size_t w_lds_bytes(int np, int tw = 256) {
  return (2 * (size_t)w_buf(np, tw) + (size_t)(tw / 32) * kWRawSlots * kWRawSlot) * 16;
}

// one dword of a wave-private raw slot (inline asm: the compiler does not order it against the LDS-DMA
// still in flight to the OTHER slot; the caller's counted vmcnt already retired this slot's DMA, and a
// later `s_waitcnt lgkmcnt(0)` that names the register makes the value valid)
template <int OFF>
GNOT_DEV float lds_read_b32_off(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

// segs / seg_start (balanced groups, engine.cpp finish_group): workgroup w runs the point ranges
// segs[seg_start[w] .. seg_start[w + 1]) = {job, slab slot, first point, end point} one after the other (a
// range of the groups' concatenated points, cut at job boundaries), so every workgroup gets the same share
// of the group's points whatever the job count; without them, one split of one job (prefix)
template <int NP = 3, int TW = 256>
__global__ void __launch_bounds__(w_threads(TW)) pgemm_x6w_kernel(const WgradJob* __restrict__ jobs,
                                                                 const int* __restrict__ prefix, int njobs,
                                                                 float* __restrict__ slab,
                                                                 const int4* __restrict__ segs,
                                                                 const int* __restrict__ seg_start) {
  constexpr int NW = TW / 32;            // waves
  constexpr int FG = TW / 64;            // 64-feature groups of the raw-row DMA
  constexpr int WC = NW / 2;             // waves along the columns
  constexpr int RB = TW / 64;            // 32-row blocks per wave (columns: 2 blocks per wave)
  constexpr int kWPiece = w_piece(TW);
  extern __shared__ __attribute__((aligned(16))) u32x4 wl[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int k0 = 0, k1 = 1;
  if (segs != nullptr) { k0 = seg_start[blockIdx.x]; k1 = seg_start[blockIdx.x + 1]; }
  for (int kseg = k0; kseg < k1; ++kseg) {
  int j, split;
  long pb, pe;
  if (segs != nullptr) {
    const int4 sg = segs[kseg];
    j = sg.x; split = sg.y; pb = sg.z; pe = sg.w;
    if (kseg > k0) __syncthreads();      // the previous range's LDS readers are done (its DMAs have landed)
  } else {
    j = find_job(prefix, njobs, blockIdx.x);
    split = blockIdx.x - prefix[j];
    const int chunk = ((jobs[j].P + jobs[j].splits - 1) / jobs[j].splits + kWStage - 1) / kWStage * kWStage;
    pb = (long)split * chunk;
    pe = min((long)jobs[j].P, pb + chunk);
  }
  const WgradJob J = jobs[j];
  const int nst = pe > pb ? (int)((pe - pb + kWStage - 1) / kWStage) : 0;
  // staging role (the point half hh is wave-uniform: waves 0 .. NW/2-1 / NW/2 ..)
  const int f = tid & (TW - 1), hh = tid / TW;
  const bool fa = f < J.out, fb = f < J.in;
  const int sdst = (f >> 5) * 64 + (f & 31) + 32 * hh;
  // MFMA role
  const int wr = wave / WC, wc = wave % WC;
  const int nrb = max(0, min(RB, (J.out - 32 * RB * wr + 31) / 32));
  const int ncb = max(0, min(2, (J.in - 64 * wc + 31) / 32));
  const bool full = nrb == RB && ncb == 2;
  const bool gel = J.x_gelu != 0;

  f32x16 acc[RB][2];
#pragma unroll
  for (int a = 0; a < RB; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float dbacc = 0.f;
  float ra_raw[8], rb_raw[8];                      // this thread's 8 points of the stage being staged
  // buffer resources based at the split's first row (64-bit base, so the 32-bit offsets span one split:
  // finish_group bounds a split's rows x pitch below 2^31 bytes): rows past the split read 0 (only the
  // last split ends inside a stage; the DMAs of stages past a split's end bring zeros nobody reads);
  // columns past out / in (inside the row pitch, which is a multiple of 4) are masked at staging
  const long nsp = pe > pb ? pe - pb : 0;
  const rsrc_t rA = make_rsrc(J.dz + pb * J.lddz, (unsigned)(nsp * J.lddz * 4));
  const rsrc_t rB = make_rsrc(J.x + pb * J.ldx, (unsigned)(nsp * J.ldx * 4));
  // DMA lane role: instruction i of operand o brings points 4 i + (lane >> 4) of the wave's half, features
  // 64 (wave % FG) + 4 (lane & 15) .. +3; in the slot, point k of the half is the 256-byte row k (64 floats)
  const int fcol = 64 * (wave % FG) + 4 * (lane & 15);
  const int dvA = ((lane >> 4) * (int)J.lddz + fcol) * 4, dvB = ((lane >> 4) * (int)J.ldx + fcol) * 4;
  u32x4* const raw = wl + 2 * w_buf(NP, TW) + wave * kWRawSlots * kWRawSlot;
  auto raw_dma = [&](int st) __attribute__((always_inline)) {
    u32x4* dst = raw + (st & 1) * kWRawSlot;
    const unsigned p0 = (unsigned)(st * kWStage + 8 * (wave / FG));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      dma16(rA, dst + i * 64, dvA, (int)((p0 + 4 * i) * (unsigned)J.lddz * 4u));
      dma16(rB, dst + 128 + i * 64, dvB, (int)((p0 + 4 * i) * (unsigned)J.ldx * 4u));
    }
  };
  const unsigned raw_addr = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)raw + 4u * lane;
  // this thread's 8 points of stage st (its slot's DMAs retired by the caller's counted wait)
  auto raw_read = [&](int st) __attribute__((always_inline)) {
    const unsigned a = raw_addr + (unsigned)((st & 1) * kWRawSlot * 16);
    ra_raw[0] = lds_read_b32_off<0>(a);    rb_raw[0] = lds_read_b32_off<2048>(a);
    ra_raw[1] = lds_read_b32_off<256>(a);  rb_raw[1] = lds_read_b32_off<2304>(a);
    ra_raw[2] = lds_read_b32_off<512>(a);  rb_raw[2] = lds_read_b32_off<2560>(a);
    ra_raw[3] = lds_read_b32_off<768>(a);  rb_raw[3] = lds_read_b32_off<2816>(a);
    ra_raw[4] = lds_read_b32_off<1024>(a); rb_raw[4] = lds_read_b32_off<3072>(a);
    ra_raw[5] = lds_read_b32_off<1280>(a); rb_raw[5] = lds_read_b32_off<3328>(a);
    ra_raw[6] = lds_read_b32_off<1536>(a); rb_raw[6] = lds_read_b32_off<3584>(a);
    ra_raw[7] = lds_read_b32_off<1792>(a); rb_raw[7] = lds_read_b32_off<3840>(a);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(ra_raw[0]), "+v"(ra_raw[1]), "+v"(ra_raw[2]), "+v"(ra_raw[3]), "+v"(ra_raw[4]),
                   "+v"(ra_raw[5]), "+v"(ra_raw[6]), "+v"(ra_raw[7]), "+v"(rb_raw[0]), "+v"(rb_raw[1]),
                   "+v"(rb_raw[2]), "+v"(rb_raw[3]), "+v"(rb_raw[4]), "+v"(rb_raw[5]), "+v"(rb_raw[6]),
                   "+v"(rb_raw[7])::"memory");
  };
  // split + LDS store of the staged rows; gel is uniform per workgroup: one branch around the whole
  // stage (not per element), so each variant is one straight-line block the scheduler can interleave
  auto stage_v = [&](int buf, auto GEL) {
    float ra[8], vb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ra[k] = fa ? ra_raw[k] : 0.f;               // columns past out / in
      const float b = fb ? rb_raw[k] : 0.f;
      dbacc += ra[k];
      vb[k] = decltype(GEL)::value ? gelu(b) : b;
    }
    u32x4 pa[NP], pq[NP];
    split8_np<NP>(ra, pa);
    split8_np<NP>(vb, pq);
    u32x4* base = wl + buf * w_buf(NP, TW);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      base[q * kWPiece + sdst] = pa[q];
      base[(NP + q) * kWPiece + sdst] = pq[q];
    }
  };
  auto stage = [&](int buf) {
    if (gel) stage_v(buf, std::true_type{});
    else stage_v(buf, std::false_type{});
  };
  auto compute = [&](int buf) {
    const u32x4* A = wl + buf * w_buf(NP, TW);
    const u32x4* Bm = A + NP * kWPiece;
    u32x4 bf[2][NP];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < NP; ++q) bf[jb][q] = Bm[q * kWPiece + (wc * 2 + jb) * 64 + lane];
#pragma unroll
    for (int ib = 0; ib < RB; ++ib) {
      if (ib >= nrb) break;
      u32x4 af[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) af[q] = A[q * kWPiece + (wr * RB + ib) * 64 + lane];
      if (ncb > 0) mfma_np<NP>(af, bf[0], acc[ib][0]);
      if (ncb > 1) mfma_np<NP>(af, bf[1], acc[ib][1]);
    }
  };
  // the LDS hand-off of the fragment images: their stores retired, then the workgroup barrier (no vmcnt:
  // the raw DMAs stay in flight across it)
  auto lds_barrier = []() __attribute__((always_inline)) { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  // The staging of stage s+1 (GELU, split, LDS stores) is interleaved instruction by instruction with the
  // MFMAs of stage s on the SAME wave, so the VALU issues in the MFMA shadows instead of in a separate
  // phase that both waves of a SIMD reach together after every barrier (full 256 x 256 tiles; edge tiles
  // take the plain double-buffered loop)
  if (nst > 0) {
    // prologue: stages 0 and 1 requested; stage 0 read (its slot then refilled with stage 2) and staged
    raw_dma(0);
    raw_dma(1);
    c2_wait_vm<4>();
    raw_read(0);
    raw_dma(2);
    stage(0);
    lds_barrier();
    int buf = 0;
    // MASK: columns past out / in exist (the fa / fb selects); jobs with out = in = 256 skip them
    auto fused = [&](int b, auto GEL, auto MASK) {
      const u32x4* A = wl + b * w_buf(NP, TW);
      const u32x4* Bm = A + NP * kWPiece;
      u32x4 bf[2][NP], af[2][NP], pa[NP], pq[NP];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < NP; ++q) bf[jb][q] = Bm[q * kWPiece + (wc * 2 + jb) * 64 + lane];
#pragma unroll
      for (int q = 0; q < NP; ++q) af[0][q] = A[q * kWPiece + (wr * RB) * 64 + lane];
      float ra[8], vb[8];
      // after each six-MFMA group (one 32 x 32 block) one point's staging (mask, column sum, GELU; every
      // second point the split of the pair just finished); sched_barrier pins the order, so each wave
      // alternates MFMA groups and VALU chunks and the two waves of a SIMD fill each other's gaps
      auto chunk = [&](int k) {
        ra[k] = (!decltype(MASK)::value || fa) ? ra_raw[k] : 0.f;
        dbacc += ra[k];
        const float bv = (!decltype(MASK)::value || fb) ? rb_raw[k] : 0.f;
        vb[k] = decltype(GEL)::value ? gelu(bv) : bv;
        // pin the chunk's results here: IR-level sinking would otherwise move the whole staging
        // next to its LDS stores after the last MFMA group (sched_barrier only binds the scheduler)
        asm volatile("" : "+v"(ra[k]), "+v"(vb[k]), "+v"(dbacc));
        if (k & 1) {
          split2_np<NP>(ra[k - 1], ra[k], pa, k >> 1);
          split2_np<NP>(vb[k - 1], vb[k], pq, k >> 1);
#pragma unroll
          for (int q = 0; q < NP; ++q) asm volatile("" : "+v"(pa[q][k >> 1]), "+v"(pq[q][k >> 1]));
        }
      };
      // 2 RB MFMA groups per stage and 8 points to stage: 8 / (2 RB) points after each group
      constexpr int CPG = 8 / (2 * RB);
#pragma unroll
      for (int ib = 0; ib < RB; ++ib) {
        if (ib + 1 < RB) {
#pragma unroll
          for (int q = 0; q < NP; ++q) af[(ib + 1) & 1][q] = A[q * kWPiece + (wr * RB + ib + 1) * 64 + lane];
        }
        mfma_np<NP>(af[ib & 1], bf[0], acc[ib][0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < CPG; ++k) chunk(CPG * 2 * ib + k);
        __builtin_amdgcn_sched_barrier(0);
        mfma_np<NP>(af[ib & 1], bf[1], acc[ib][1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < CPG; ++k) chunk(CPG * (2 * ib + 1) + k);
        __builtin_amdgcn_sched_barrier(0);
      }
      u32x4* base = wl + (b ^ 1) * w_buf(NP, TW);
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        base[q * kWPiece + sdst] = pa[q];
        base[(NP + q) * kWPiece + sdst] = pq[q];
      }
    };
    // iteration s: stage s + 1's rows (the wait leaves stage s + 2's four DMAs in flight) are read, their
    // slot refilled with stage s + 3, and staged while stage s is multiplied
    auto run = [&](auto GEL, auto MASK) {
      for (int s = 0; s + 1 < nst; ++s) {
        c2_wait_vm<4>();
        raw_read(s + 1);
        raw_dma(s + 3);
        fused(buf, GEL, MASK);
        lds_barrier();
        buf ^= 1;
      }
    };
    if (full) {
      if (J.out >= TW && J.in >= TW) {
        if (gel) run(std::true_type{}, std::false_type{});
        else run(std::false_type{}, std::false_type{});
      } else {
        if (gel) run(std::true_type{}, std::true_type{});
        else run(std::false_type{}, std::true_type{});
      }
    } else {
      for (int s = 0; s + 1 < nst; ++s) {
        c2_wait_vm<4>();
        raw_read(s + 1);
        raw_dma(s + 3);
        compute(buf);
        stage(buf ^ 1);
        lds_barrier();
        buf ^= 1;
      }
    }
    compute(buf);   // the last stage
    // the DMAs of the two stages past the end (zeros) land before the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // partials -> slab [split][128-tile][128 x (128 + 1)] (the pgemm_kernel layout)
  const int ntile = J.tiles_o * J.tiles_i;
  float* S0 = slab + J.slab_off + (long)split * ntile * (kTile * (kTile + 1));
#pragma unroll
  for (int ib = 0; ib < RB; ++ib)
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wr * 32 * RB + ib * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wc * 64 + jb * 32 + (lane & 31);
        if (row < J.out && col < J.in)
          S0[((row >> 7) * J.tiles_i + (col >> 7)) * (kTile * (kTile + 1)) + (row & 127) * (kTile + 1) + (col & 127)] =
              acc[ib][jb][r];
      }
  if (J.db != nullptr) {
    // column sums of A: the two point halves of every feature through LDS, in a fixed order
    // (red overlays stage buffer 0, which other waves may still be reading in the last compute(): the
    // interleaved loop ends without a barrier)
    float* red = reinterpret_cast<float*>(wl);
    __syncthreads();
    red[hh * TW + f] = dbacc;
    __syncthreads();
    if (tid < TW && f < J.out)
      S0[((f >> 7) * J.tiles_i) * (kTile * (kTile + 1)) + (f & 127) * (kTile + 1) + kTile] = red[f] + red[TW + f];
  }
  }
}

// ---------------------------------------------------------------- bf16-storage variant (bf16 mode)
// In bf16 mode the soft-MoE chains store dZ and every Linear's input (gelu already applied, RNE bf16: the
// operand bits the forward's MFMAs used) as pair-interleaved rows (gnot_common.h), so this kernel stages
// nothing by hand:
//   DMA:  32-point stages of both operands (2 x 16 KiB) land by LDS-DMA in a 4-slot ring with three
//         stages in flight per workgroup (96 KiB: about one CU's share of HBM bandwidth x latency).  One
//         wave-instruction brings two 512-byte rows; the lane at chunk position c of row r fetches chunk
//         c ^ 4 (r & 3), so the 4 rows one 16-lane transposed read touches sit on disjoint banks;
//   MFMA: ds_read_b64_tr_b16 turns the point-major rows into v_mfma_f32_32x32x16_bf16 fragments (lane i
//         of a 16-lane group receives 4 points of feature i); wave (wr, wc) owns rows [128 wr, +128) x
//         cols [64 wc, +64) as in the wide kernel; db (column sums of dZ) comes from the fragment of row
//         block wc that each wave reads anyway.
// Cost per point and job: 1 KiB of HBM against 2 x 256 x 256 flops (128 flop/B): HBM-bound.
constexpr int kBStage = 32;
constexpr int kBSlots = 4;
constexpr int kBOpnd = kBStage * kB16Row;                  // bytes per operand per stage (16 KiB)
constexpr int kBSlotBytes = 2 * kBOpnd;
constexpr size_t kBLds = (size_t)kBSlots * kBSlotBytes;    // 128 KiB

GNOT_DEV u32x2 lds_tr_b64(unsigned addr) {
  u32x2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// segs / seg_start: the balanced point ranges of pgemm_x6w_kernel
__global__ void __launch_bounds__(kWThreads) pgemm_b16_kernel(const WgradJob* __restrict__ jobs,
                                                             const int* __restrict__ prefix, int njobs,
                                                             float* __restrict__ slab, const int4* __restrict__ segs,
                                                             const int* __restrict__ seg_start) {
  extern __shared__ __attribute__((aligned(16))) u32x4 bl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int k0 = 0, k1 = 1;
  if (segs != nullptr) { k0 = seg_start[blockIdx.x]; k1 = seg_start[blockIdx.x + 1]; }
  for (int kseg = k0; kseg < k1; ++kseg) {
  int j, split;
  long pb, pe;
  if (segs != nullptr) {
    const int4 sg = segs[kseg];
    j = sg.x; split = sg.y; pb = sg.z; pe = sg.w;
    if (kseg > k0) __syncthreads();      // every wave is done with the previous range's stage slots
  } else {
    j = find_job(prefix, njobs, blockIdx.x);
    split = blockIdx.x - prefix[j];
    const int chunk = ((jobs[j].P + jobs[j].splits - 1) / jobs[j].splits + kBStage - 1) / kBStage * kBStage;
    pb = (long)split * chunk;
    pe = min((long)jobs[j].P, pb + chunk);
  }
  const WgradJob J = jobs[j];
  const int nst = pe > pb ? (int)((pe - pb + kBStage - 1) / kBStage) : 0;
  const int wr = wave >> 2, wc = wave & 3;
  // resources based at the split's first row: rows past the split read 0 (only the last split's last
  // stage reaches past it)
  const unsigned bytes = (unsigned)((pe > pb ? pe - pb : 0) * kB16Row);
  const long rb = pb * (kB16Row / 4);                        // the split's first row, in 4-byte units
  const rsrc_t rA = make_rsrc(J.dz + rb, bytes), rB = make_rsrc(J.x + rb, bytes);
  // DMA role: wave w brings rows 2w, 2w+1 (instruction 0) and 2w+16, 2w+17 (instruction 1) of both
  // operands; (r & 3) is the same for both instructions
  const int hi = lane >> 5;
  const int dvoff = hi * kB16Row + (((lane & 31) ^ (((2 * wave + hi) & 3) << 2)) * 16);
  auto dma_stage = [&](int s) __attribute__((always_inline)) {
    const unsigned p0 = (unsigned)(s * kBStage);           // relative to the split's first row
    u32x4* slot = bl + (s % kBSlots) * (kBSlotBytes / 16);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 2 * wave + 16 * i;
      const int soff = (int)((p0 + (unsigned)row) * (unsigned)kB16Row);
      dma16(rA, slot + row * (kB16Row / 16), dvoff, soff);
      dma16(rB, slot + (kBOpnd + row * kB16Row) / 16, dvoff, soff);
    }
  };
  // transposed-read address of feature block m (32 features = PI chunk column m), K-step ks (16 points),
  // half h (4 points): lane 4q + pq of group G reads row 16 ks + 8 (G >> 1) + 4 h + q, features
  // 32 m + 16 (G & 1) + 4 pq .. + 3 = chunk m * 4 + pq (position (m ^ q) * 4 + pq), half G & 1
  const int G = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)bl;
  auto frag = [&](unsigned base, int m, int ks) {
    const unsigned a = base + (unsigned)((16 * ks + 8 * (G >> 1) + q) * kB16Row + (((m ^ q) * 4 + pq) * 16) + (G & 1) * 8);
    const u32x2 x0 = lds_tr_b64(a), x1 = lds_tr_b64(a + 4 * kB16Row);
    return u32x4{x0[0], x0[1], x1[0], x1[1]};
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float dbacc = 0.f;
  for (int s = 0; s < 3 && s < nst; ++s) dma_stage(s);
  for (int s = 0; s < nst; ++s) {
    // stage s has landed (this wave's DMAs of stages s+1, s+2 stay in flight: 4 each) and every wave is
    // done with stage s-1, whose slot stage s+3 refills
    c2_sync_n(4 * min(2, nst - 1 - s));
    if (s + 3 < nst) dma_stage(s + 3);
    const unsigned base = lds0 + (unsigned)((s % kBSlots) * kBSlotBytes);
    u32x4 af[2][4], bf[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) af[ks][ib] = frag(base, 4 * wr + ib, ks);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) bf[ks][jb] = frag(base + kBOpnd, 2 * wc + jb, ks);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // the reads are inline asm: the compiler does not know they are pending, so wait for them by name
      // (K-step 1's reads stay in flight under K-step 0's MFMAs)
      __builtin_amdgcn_sched_barrier(0);
      if (ks == 0)
        asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(af[0][0]), "+v"(af[0][1]), "+v"(af[0][2]), "+v"(af[0][3]),
                     "+v"(bf[0][0]), "+v"(bf[0][1])::"memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[1][0]), "+v"(af[1][1]), "+v"(af[1][2]), "+v"(af[1][3]),
                     "+v"(bf[1][0]), "+v"(bf[1][1])::"memory");
#pragma unroll
      for (int ib = 0; ib < 4; ++ib)
        if (ib == wc) {
          const u32x4 w = af[ks][ib];
#pragma unroll
          for (int d = 0; d < 4; ++d) dbacc += bf16_lo(w[d]) + bf16_hi(w[d]);
        }
#pragma unroll
      for (int ib = 0; ib < 4; ++ib)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
          acc[ib][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[ks][ib]),
                                                                __builtin_bit_cast(bf16x8, bf[ks][jb]), acc[ib][jb], 0,
                                                                0, 0);
    }
  }

  // partials -> slab [split][128-tile][128 x (128 + 1)] (the pgemm_kernel layout)
  const int ntile = J.tiles_o * J.tiles_i;
  float* S0 = slab + J.slab_off + (long)split * ntile * (kTile * (kTile + 1));
#pragma unroll
  for (int ib = 0; ib < 4; ++ib)
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wr * 128 + ib * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wc * 64 + jb * 32 + (lane & 31);
        S0[((row >> 7) * J.tiles_i + (col >> 7)) * (kTile * (kTile + 1)) + (row & 127) * (kTile + 1) + (col & 127)] =
            acc[ib][jb][r];
      }
  // db: lane l summed points of half l >> 5 of feature 128 wr + 32 wc + (l & 31)
  dbacc += shfl_xor(dbacc, 32);
  if (J.db != nullptr && lane < 32) {
    const int f = wr * 128 + wc * 32 + lane;
    S0[((f >> 7) * J.tiles_i) * (kTile * (kTile + 1)) + (f & 127) * (kTile + 1) + kTile] = dbacc;
  }
  }
}

// sum the split partials; normal jobs write dW[out, in] (+ db[out]); state jobs (state_dh > 0) write
// the per-head diagonal blocks into [H][dh*dh + dh] (S row-major, then z)
__global__ void __launch_bounds__(256) pgemm_reduce_kernel(const WgradJob* __restrict__ jobs,
                                                           const int* __restrict__ prefix, int njobs, int total,
                                                           const float* __restrict__ slab) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int j = find_job(prefix, njobs, idx);
  const WgradJob& J = jobs[j];
  int e = idx - prefix[j];
  const int ntile = J.diag_only ? J.tiles_o : J.tiles_o * J.tiles_i;
  const int tile = e / (kTile * (kTile + 1));
  e -= tile * (kTile * (kTile + 1));
  const int rl = e / (kTile + 1), cl = e % (kTile + 1);
  const int to = J.diag_only ? tile : tile / J.tiles_i;
  const int ti = J.diag_only ? tile : tile % J.tiles_i;
  const int row = to * kTile + rl;
  const bool isdb = cl == kTile;
  const int col = ti * kTile + cl;
  if (row >= J.out) return;
  if (isdb) {
    if (J.db == nullptr || (!J.diag_only && ti != 0)) return;
  } else if (col >= J.in) {
    return;
  }
  if (J.state_dh > 0 && !isdb && (row / J.state_dh) != (col / J.state_dh)) return;
  const float* S = slab + J.slab_off + (long)tile * (kTile * (kTile + 1)) + rl * (kTile + 1) + cl;
  const long sstride = (long)ntile * (kTile * (kTile + 1));
  // 8 independent partial sums keep 8 slab loads in flight (the loop is latency-bound otherwise);
  // the combination order is fixed, so the result is still deterministic
  float part[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= J.splits; k += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) part[u] += S[(long)(k + u) * sstride];
  for (; k < J.splits; ++k) part[0] += S[(long)k * sstride];
  const float s = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
  float* dst;
  if (J.state_dh > 0) {
    const int dh = J.state_dh, hh = row / dh, i = row % dh;
    float* base = J.dW + (long)hh * (dh * dh + dh);
    dst = isdb ? base + dh * dh + i : base + i * dh + (col % dh);
  } else {
    dst = isdb ? (J.db + row) : (J.dW + (long)row * J.in + col);
  }
  *dst = J.accumulate ? (*dst + s) : s;
}

hipError_t launch_wgrad_b16(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                            const int* red_prefix_dev, int total_red, float* slab, hipStream_t s, const int4* segs,
                            const int* seg_start) {
  if (njobs <= 0) return hipSuccess;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pgemm_b16_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kBLds);
    attr = true;
  }
  hipLaunchKernelGGL(pgemm_b16_kernel, dim3(total_wgs), dim3(kWThreads), kBLds, s, jobs_dev, wg_prefix_dev, njobs, slab,
                     segs, seg_start);
  hipLaunchKernelGGL(pgemm_reduce_kernel, dim3((total_red + 255) / 256), dim3(256), 0, s, jobs_dev, red_prefix_dev,
                     njobs, total_red, (const float*)slab);
  return hipGetLastError();
}

hipError_t launch_wgrad(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                        const int* red_prefix_dev, int total_red, float* slab, hipStream_t s, bool x6, bool wide,
                        int np, int tw, const int4* segs, const int* seg_start) {
  if (njobs <= 0) return hipSuccess;
  if (wide) {
    const size_t lds = w_lds_bytes(np, tw);
#define GNOT_X6W(NP_, TW_)                                                                                     \
  if (np == NP_ && tw == TW_) {                                                                                \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pgemm_x6w_kernel<NP_, TW_>),                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                         \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL((pgemm_x6w_kernel<NP_, TW_>), dim3(total_wgs), dim3(w_threads(TW_)), lds, s, jobs_dev,  \
                       wg_prefix_dev, njobs, slab, segs, seg_start);                                           \
  }
    GNOT_X6W(3, 256) GNOT_X6W(1, 256) GNOT_X6W(3, 128) GNOT_X6W(1, 128)
#undef GNOT_X6W
  } else if (x6) {
    if (np == 1) hipLaunchKernelGGL(pgemm_x6_kernel<1>, dim3(total_wgs), dim3(256), 0, s, jobs_dev, wg_prefix_dev, njobs, slab);
    else hipLaunchKernelGGL(pgemm_x6_kernel<3>, dim3(total_wgs), dim3(256), 0, s, jobs_dev, wg_prefix_dev, njobs, slab);
  }
  else
    hipLaunchKernelGGL(pgemm_kernel, dim3(total_wgs), dim3(256), 0, s, jobs_dev, wg_prefix_dev, njobs, slab);
  hipLaunchKernelGGL(pgemm_reduce_kernel, dim3((total_red + 255) / 256), dim3(256), 0, s, jobs_dev,
                     red_prefix_dev, njobs, total_red, (const float*)slab);
  return hipGetLastError();
}

}  // namespace gnot
