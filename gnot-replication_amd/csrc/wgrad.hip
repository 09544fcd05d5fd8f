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
// Per stage 32 points of A and B rows (2 x 16 KiB, coalesced 16-B loads, GELU applied while
// staging) go to LDS; the NEXT stage's rows are already in flight in registers while the current one
// is consumed.  Each wave computes a 64x64 quadrant with v_mfma_f32_32x32x2_f32 (2 points per MFMA
// k-step, 4 MFMAs per pair of A/B fragment loads).  Partial tiles go to a slab; the reduce pass sums
// the splits in a fixed order (deterministic, no atomics).
#include "gnot_common.h"
#include "gnot_kernels.h"

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

// stage registers: thread t loads 4 float4 of A rows and 4 of B rows (32 rows x 32 float4 each)
struct StageRegs {
  float4 a[4], b[4];
  float wa[4];   // per-row weight for the A column sums (z / db), per float4
};

GNOT_DEV void stage_load(StageRegs& R, const WgradJob& J, long pbase, long pend, int c0o, int c0i, int tid) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + k * 256;          // 0..1023
    const int row = idx >> 5, c4 = idx & 31;
    const long p = pbase + row;
    const bool pv = p < pend;
    const int co = c0o + 4 * c4, ci = c0i + 4 * c4;
    float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
    if (pv) {
      if (co + 3 < J.out && (J.lddz & 3) == 0) {
        va = *reinterpret_cast<const float4*>(J.dz + p * J.lddz + co);
      } else {
        float t[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (co + r < J.out) ? J.dz[p * J.lddz + co + r] : 0.f;
        va = make_float4(t[0], t[1], t[2], t[3]);
      }
      if (ci + 3 < J.in && (J.ldx & 3) == 0) {
        vb = *reinterpret_cast<const float4*>(J.x + p * J.ldx + ci);
      } else {
        float t[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (ci + r < J.in) ? J.x[p * J.ldx + ci + r] : 0.f;
        vb = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
    R.a[k] = va;
    R.b[k] = vb;
    R.wa[k] = 1.f;
    if (J.w && pv && co < J.out) R.wa[k] = J.w[p * J.ldw + co / J.wdh];
  }
}

GNOT_DEV void stage_store(const StageRegs& R, const WgradJob& J, float* __restrict__ As, float* __restrict__ Bs,
                          float* __restrict__ colw, int tid) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + k * 256;
    float4 vb = R.b[k];
    if (J.x_gelu) { vb.x = gelu(vb.x); vb.y = gelu(vb.y); vb.z = gelu(vb.z); vb.w = gelu(vb.w); }
    reinterpret_cast<float4*>(As)[idx] = R.a[k];
    reinterpret_cast<float4*>(Bs)[idx] = vb;
    if (J.w) colw[idx] = R.wa[k];     // weight of row (idx>>5) for A columns 4*(idx&31) .. +3
  }
}

__global__ void __launch_bounds__(256) pgemm_kernel(const WgradJob* __restrict__ jobs, const int* __restrict__ prefix,
                                                    int njobs, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float smem[2 * kStage * kLdsRow + kStage * 32];
  float* As = smem;
  float* Bs = smem + kStage * kLdsRow;
  float* colw = Bs + kStage * kLdsRow;     // [32 rows][32 float4 groups]
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
  const bool want_db = (J.db != nullptr) && (wi == 0) && (J.diag_only || ti == 0);

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float dbacc[2] = {0.f, 0.f};

  StageRegs R;
  if (pb < pe) stage_load(R, J, pb, pe, c0o, c0i, tid);
  for (long p0 = pb; p0 < pe; p0 += kStage) {
    __syncthreads();                          // previous stage fully consumed
    stage_store(R, J, As, Bs, colw, tid);
    __syncthreads();
    if (p0 + kStage < pe) stage_load(R, J, p0 + kStage, pe, c0o, c0i, tid);   // in flight during MFMAs
#pragma unroll 4
    for (int s = 0; s < kStage / 2; ++s) {
      const int row = 2 * s + h;
      const float* ar = As + row * kLdsRow + wo * 64 + r32;
      const float* br = Bs + row * kLdsRow + wi * 64 + r32;
      const float a0 = ar[0], a1 = ar[32];
      const float b0 = br[0], b1 = br[32];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      if (want_db) {
        if (J.w) {
          const float* wr = colw + row * 32;
          dbacc[0] = fmaf(wr[(wo * 64 + r32) >> 2], a0, dbacc[0]);
          dbacc[1] = fmaf(wr[(wo * 64 + 32 + r32) >> 2], a1, dbacc[1]);
        } else {
          dbacc[0] += a0;
          dbacc[1] += a1;
        }
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
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float v = dbacc[a] + __shfl_xor(dbacc[a], 32, 64);
      if (h == 0) S[(wo * 64 + a * 32 + r32) * (kTile + 1) + kTile] = v;
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

hipError_t launch_wgrad(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                        const int* red_prefix_dev, int total_red, float* slab, hipStream_t s) {
  if (njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(pgemm_kernel, dim3(total_wgs), dim3(256), 0, s, jobs_dev, wg_prefix_dev, njobs, slab);
  hipLaunchKernelGGL(pgemm_reduce_kernel, dim3((total_red + 255) / 256), dim3(256), 0, s, jobs_dev,
                     red_prefix_dev, njobs, total_red, (const float*)slab);
  return hipGetLastError();
}

}  // namespace gnot
