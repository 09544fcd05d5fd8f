// Weight gradients of every Linear: dW = sum_p dZ[p]^T X[p], db = sum_p dZ[p]   (the "autograd of
// nn.Linear" of reference model.py:9-14, 43-51 behind main.py:102's loss.backward()).
//
// A batched, split-K GEMM over points: one launch covers a whole list of (dZ, X) jobs (all
// experts x all layers of a MoE, or the q/k/v/fc_out projections of an attention).  One wave
// computes one 32x32 tile of dW over one point chunk with v_mfma_f32_32x32x2_f32 (the two k rows
// of an MFMA step are two points; each operand fetch is a 128 B contiguous row segment), writes a
// partial slab, and a second pass sums the slabs in a fixed order — deterministic, no atomics.
// X may be the layer's saved PRE-activation, in which case GELU is applied on load (the input of
// hidden Linear l is gelu(h_{l-1}), model.py:10-13).
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

typedef float f32x16 __attribute__((ext_vector_type(16)));

GNOT_DEV int find_job(const int* __restrict__ prefix, int njobs, int idx) {
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) wgrad_kernel(const WgradJob* __restrict__ jobs,
                                                    const int* __restrict__ prefix, int njobs,
                                                    int total_waves, float* __restrict__ slab) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= total_waves) return;
  const int lane = threadIdx.x & 63;
  const int j = find_job(prefix, njobs, wid);
  const WgradJob& J = jobs[j];
  int t = wid - prefix[j];
  const int split = t % J.splits;
  t /= J.splits;
  const int ti = t % J.tiles_i;
  const int to = t / J.tiles_i;

  const int chunk = (((J.P + J.splits - 1) / J.splits) + 1) & ~1;
  const long pb = (long)split * chunk;
  const long pe = min((long)J.P, pb + chunk);

  const int r32 = lane & 31, h = lane >> 5;
  const int oi = to * 32 + r32;   // dW row handled by this lane's A operand
  const int ii = ti * 32 + r32;   // dW column handled by this lane's B operand
  const bool ao = oi < J.out, bi = ii < J.in;
  const bool want_db = (ti == 0) && J.db;

  f32x16 acc = {};
  float dbacc = 0.f;
  // uniform trip count over point PAIRS (the MFMA needs all 64 lanes); lane half h takes point
  // pb + 2*step + h, zero operands past the chunk end
  const int nsteps = (int)((pe - pb + 1) >> 1);
#pragma unroll 4
  for (int st = 0; st < nsteps; ++st) {
    const long p = pb + 2 * st + h;
    const bool pv = p < pe;
    const float av = (ao && pv) ? J.dz[p * J.lddz + oi] : 0.f;
    float bv = (bi && pv) ? J.x[p * J.ldx + ii] : 0.f;
    if (J.x_gelu) bv = gelu(bv);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    dbacc += av;
  }

  const int out_p = J.tiles_o * 32, in_p = J.tiles_i * 32;
  float* S = slab + J.slab_off + (long)split * out_p * (in_p + 1);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = to * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const int col = ti * 32 + r32;
    S[(long)row * (in_p + 1) + col] = acc[r];
  }
  if (want_db) {
    dbacc += __shfl_xor(dbacc, 32, 64);
    if (h == 0) S[(long)oi * (in_p + 1) + in_p] = dbacc;
  }
}

__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const WgradJob* __restrict__ jobs,
                                                           const int* __restrict__ prefix, int njobs,
                                                           int total, const float* __restrict__ slab) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int j = find_job(prefix, njobs, idx);
  const WgradJob& J = jobs[j];
  const int e = idx - prefix[j];
  const int in_p = J.tiles_i * 32, out_p = J.tiles_o * 32;
  const int row = e / (in_p + 1), col = e % (in_p + 1);
  if (row >= J.out) return;
  const bool isdb = col == in_p;
  if (isdb ? (J.db == nullptr) : (col >= J.in)) return;
  const float* S = slab + J.slab_off + (long)row * (in_p + 1) + col;
  const long sstride = (long)out_p * (in_p + 1);
  float s = 0.f;
  for (int k = 0; k < J.splits; ++k) s += S[k * sstride];
  float* dst = isdb ? (J.db + row) : (J.dW + (long)row * J.in + col);
  *dst = J.accumulate ? (*dst + s) : s;
}

hipError_t launch_wgrad(const WgradJob* jobs_dev, const int* wave_prefix_dev, int njobs, int total_waves,
                        const int* red_prefix_dev, int total_red, float* slab, hipStream_t s) {
  if (njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(wgrad_kernel, dim3((total_waves + 3) / 4), dim3(256), 0, s, jobs_dev,
                     wave_prefix_dev, njobs, total_waves, slab);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total_red + 255) / 256), dim3(256), 0, s, jobs_dev,
                     red_prefix_dev, njobs, total_red, (const float*)slab);
  return hipGetLastError();
}

}  // namespace gnot
