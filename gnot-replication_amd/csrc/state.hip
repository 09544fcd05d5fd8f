// Linear-attention states: the only cross-point reductions of the reference attention.
//
//   forward   S[h] = sum_m k_m^T v_m  (dh x dh),  z[h] = sum_m k_m          (model.py:77, 79 / 98, 100)
//   backward  dS[h] = sum_n q_n^T du_n,           dz[h] = sum_n dden_n q_n  (autograd of model.py:78-80)
// One job = one sample (or one (block, input function, sample) of the batched cross states).  The
// sum over a job's points is split over workgroups of state_pts(d) points; each writes its partial
// [H][dh*dh + dh] state to a slab and state_reduce sums the partials in a fixed order, so results
// are bitwise reproducible (no atomics).
//
// VALU form (any head width): each thread owns a 4x4 block of one head's S (and the 4 matching z entries, kept by every
// block; only j-block 0 stores them).  Arithmetic is plain fp32 FMA on the VALU: H*dh^2 MACs per
// point (2 Ki at d=128, H=8) against 2*d*4 bytes of rows, so the pass is bound by row traffic and
// latency, not math.  It replaces a 128x128 MFMA tile of which only the H diagonal dh x dh blocks
// were kept.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

constexpr int kStateThreads = 256;

GNOT_DEV int find_job_s(const int* __restrict__ prefix, int njobs, int idx) {
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= idx) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// floats of one row-stage region: pts * d rounded up to whole 64-lane x 16-byte DMA instructions
// (d > 128 takes pts = 8192 / d, e.g. 56 points x 144 = 8,064 floats: 31.5 instructions)
__host__ __device__ constexpr int state_stage_floats(int pts, int d) { return (pts * d + 255) / 256 * 256; }

// One workgroup = state_pts(d) points of one job.  The workgroup first pulls all of its A and B
// rows into LDS with LDS-DMA (global_load_lds, 16 B per lane, every load in flight at once: one
// round of memory latency instead of one per row batch) plus the per-(point, head) weights w, then
// thread t owns output block t % nblk (head h, i-block, j-block) for the points p = r, r + R, ...
// (r = t / nblk, R = 256 / nblk point lanes).  The R partial blocks are combined through LDS (the
// A region, reused) and the workgroup's partial state goes to the slab.
__global__ void __launch_bounds__(kStateThreads) state_partial_kernel(const WgradJob* __restrict__ jobs,
                                                                     const int* __restrict__ prefix, int njobs,
                                                                     float* __restrict__ slab, int pts) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int j = find_job_s(prefix, njobs, blockIdx.x);
  const WgradJob& J = jobs[j];
  const int split = blockIdx.x - prefix[j];
  const int dh = J.state_dh, d = J.out, H = d / dh, nb = dh / 4;
  const int nblk = H * nb * nb;
  const int per = H * (dh * dh + dh);
  const long p0 = (long)split * pts;
  const int np = (int)min((long)pts, (long)J.P - p0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool use_w = J.w != nullptr;
  // each stage region is whole 1 KiB LDS-DMA wave-instructions (state_stage_floats): the last
  // instruction of a stage writes all 64 lanes, so an unrounded region would spill into the next one
  const int stage_f = state_stage_floats(pts, d);
  float* As = lds;
  float* Bs = lds + stage_f;
  float* Ws = lds + 2 * stage_f;
  float* S = slab + J.slab_off + (long)split * per;
  if (np > 0) {
    // ---- rows -> LDS (flat float4 index f of the [np, d] stage; lanes past the end re-read the last float4)
    const int d4 = d / 4, n4 = np * d4;
    for (int base = wave * 64; base < n4; base += kStateThreads) {
      const int f = min(base + lane, n4 - 1);
      const int row = f / d4, c = (f % d4) * 4;
      __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(J.dz + (p0 + row) * J.lddz + c), (lds_void_ptr)(As + base * 4),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(J.x + (p0 + row) * J.ldx + c), (lds_void_ptr)(Bs + base * 4),
                                       16, 0, 0);
    }
    if (use_w)
      for (int f = tid; f < np * H; f += kStateThreads) Ws[f] = J.w[(p0 + f / H) * J.ldw + f % H];
  }
  lds_dma_wait();
  __syncthreads();
  const int R = nblk >= kStateThreads ? 1 : kStateThreads / nblk;
  const int r = tid / (nblk < kStateThreads ? nblk : kStateThreads);
  float keep[20];
  // 4x4 output blocks per thread: ceil(H (dh/4)^2 / 256) of them (d dh / 4096; round 5 capped this at 4, i.e.
  // d dh <= 16384, which refused d = 512 with heads of 64)
  const int nk = nblk >= kStateThreads ? (nblk + kStateThreads - 1) / kStateThreads : 1;
  for (int k = 0; k < nk; ++k) {
    const int blk = (nblk >= kStateThreads ? tid + k * kStateThreads : tid % nblk);
    const bool active = (nblk >= kStateThreads) ? blk < nblk : (k == 0 && r < R);
    f32x4 acc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                    f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 zacc = f32x4{0.f, 0.f, 0.f, 0.f};
    const int h = blk / (nb * nb), ib = (blk / nb) % nb, jb = blk % nb;
    if (active) {
      const float* Ap = As + h * dh + 4 * ib;
      const float* Bp = Bs + h * dh + 4 * jb;
      for (int pp = r; pp < np; pp += R) {
        const float4 a4 = *reinterpret_cast<const float4*>(Ap + pp * d);
        const float4 b4 = *reinterpret_cast<const float4*>(Bp + pp * d);
        const float wt = use_w ? Ws[pp * H + h] : 1.f;
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          acc[rr][0] = fmaf(av[rr], b4.x, acc[rr][0]);
          acc[rr][1] = fmaf(av[rr], b4.y, acc[rr][1]);
          acc[rr][2] = fmaf(av[rr], b4.z, acc[rr][2]);
          acc[rr][3] = fmaf(av[rr], b4.w, acc[rr][3]);
          zacc[rr] = fmaf(wt, av[rr], zacc[rr]);
        }
      }
    }
    if (R == 1) {
      if (active) {
        float* Sh = S + h * (dh * dh + dh);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          *reinterpret_cast<float4*>(Sh + (4 * ib + rr) * dh + 4 * jb) =
              make_float4(acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]);
        if (jb == 0) *reinterpret_cast<float4*>(Sh + dh * dh + 4 * ib) = make_float4(zacc[0], zacc[1], zacc[2], zacc[3]);
      }
    } else if (k == 0) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int c = 0; c < 4; ++c) keep[rr * 4 + c] = acc[rr][c];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) keep[16 + rr] = zacc[rr];
    }
  }
  if (R > 1) {
    // combine the R point lanes of every block (fixed order) through LDS (the A/B region is free now)
    __syncthreads();
    float* mine = lds + tid * 20;
#pragma unroll
    for (int e = 0; e < 20; ++e) mine[e] = keep[e];
    __syncthreads();
    if (r == 0) {
      const int blk = tid;
      const int h = blk / (nb * nb), ib = (blk / nb) % nb, jb = blk % nb;
      float tot[20];
#pragma unroll
      for (int e = 0; e < 20; ++e) tot[e] = mine[e];
      for (int o = 1; o < R; ++o) {
        const float* other = lds + (tid + o * nblk) * 20;
#pragma unroll
        for (int e = 0; e < 20; ++e) tot[e] += other[e];
      }
      float* Sh = S + h * (dh * dh + dh);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        *reinterpret_cast<float4*>(Sh + (4 * ib + rr) * dh + 4 * jb) =
            make_float4(tot[rr * 4], tot[rr * 4 + 1], tot[rr * 4 + 2], tot[rr * 4 + 3]);
      if (jb == 0) *reinterpret_cast<float4*>(Sh + dh * dh + 4 * ib) = make_float4(tot[16], tot[17], tot[18], tot[19]);
    }
  }
}

// ---- fp32 MFMA form (dh = 16/32/64, H % 4 == 0): wave w owns heads w*HPW .. w*HPW+HPW-1 of the
// workgroup's `pts` points; per 4-point k-step one v_mfma_f32_16x16x4_f32 per 16x16 tile of S:
//   A[i][k] = A_row[p0 + k][h*dh + 16I + i]   (lane (i, g=k) loads one float)
//   B[k][j] = B_row[p0 + k][h*dh + 16J + j]
// so every row element is loaded once, straight from HBM into the operand registers (no LDS), and
// z = sum_p w A_row is a lane-local FMA finished by two shuffles.  Exact fp32 products, fp32 sums,
// fixed order: deterministic.
template <int DH, int HPW>
__global__ void __launch_bounds__(256) state_mfma_kernel(const WgradJob* __restrict__ jobs,
                                                         const int* __restrict__ prefix, int njobs,
                                                         float* __restrict__ slab, int pts) {
  constexpr int NT = DH / 16, U = 8;   // U 4-point steps per batch of loads in flight
  const int j = find_job_s(prefix, njobs, blockIdx.x);
  const WgradJob& J = jobs[j];
  const int split = blockIdx.x - prefix[j];
  const int H = J.out / DH;
  const long p0 = (long)split * pts;
  const long pend = min(p0 + (long)pts, (long)J.P);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, g = lane >> 4;
  const bool use_w = J.w != nullptr;
  const float* __restrict__ Ar = J.dz;
  const float* __restrict__ Br = J.x;
  f32x4 acc[HPW][NT][NT];
  float zp[HPW][NT];
#pragma unroll
  for (int kh = 0; kh < HPW; ++kh)
#pragma unroll
    for (int I = 0; I < NT; ++I) {
      zp[kh][I] = 0.f;
#pragma unroll
      for (int Jt = 0; Jt < NT; ++Jt) acc[kh][I][Jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  const int col0 = wave * HPW * DH + i16;
  for (long pb = p0; pb < pend; pb += 4 * U) {
    float a[U][HPW][NT], b[U][HPW][NT], w[U][HPW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long pp = pb + 4 * u + g;
      const bool valid = pp < pend;
      const long pr = valid ? pp : p0;
#pragma unroll
      for (int kh = 0; kh < HPW; ++kh) {
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          const float av = Ar[pr * J.lddz + col0 + kh * DH + 16 * I];
          const float bv = Br[pr * J.ldx + col0 + kh * DH + 16 * I];
          a[u][kh][I] = valid ? av : 0.f;
          b[u][kh][I] = valid ? bv : 0.f;
        }
        w[u][kh] = use_w ? J.w[pr * J.ldw + wave * HPW + kh] : 1.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int kh = 0; kh < HPW; ++kh)
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          zp[kh][I] = fmaf(w[u][kh], a[u][kh][I], zp[kh][I]);
#pragma unroll
          for (int Jt = 0; Jt < NT; ++Jt) acc[kh][I][Jt] = mfma4(a[u][kh][I], b[u][kh][Jt], acc[kh][I][Jt]);
        }
  }
  float* S = slab + J.slab_off + (long)split * H * (DH * DH + DH);
#pragma unroll
  for (int kh = 0; kh < HPW; ++kh) {
    float* Sh = S + (wave * HPW + kh) * (DH * DH + DH);
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int Jt = 0; Jt < NT; ++Jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) Sh[(16 * I + 4 * g + r) * DH + 16 * Jt + i16] = acc[kh][I][Jt][r];
      float z = zp[kh][I];
      z += __shfl_xor(z, 16, 64);
      z += __shfl_xor(z, 32, 64);
      if (g == 0) Sh[DH * DH + 16 * I + i16] = z;
    }
  }
}

// out[e] = sum over splits of the partials: 8 lanes per state element, each summing every 8th
// split with 4 loads in flight, then a fixed butterfly -> deterministic.
__global__ void __launch_bounds__(256) state_reduce_kernel(const WgradJob* __restrict__ jobs,
                                                           const int* __restrict__ red_prefix, int njobs, int total,
                                                           const float* __restrict__ slab) {
  const int gidx = blockIdx.x * 256 + threadIdx.x;
  const int idx = gidx >> 3, lane8 = gidx & 7;
  const bool valid = idx < total;
  float s = 0.f;
  int j = 0, e = 0;
  if (valid) {
    j = find_job_s(red_prefix, njobs, idx);
    e = idx - red_prefix[j];
    const WgradJob& J = jobs[j];
    const int per = J.out / J.state_dh * (J.state_dh * J.state_dh + J.state_dh);
    const float* S = slab + J.slab_off + e;
    float part[4] = {0.f, 0.f, 0.f, 0.f};
    int k = lane8;
    for (; k + 24 < J.splits; k += 32)
#pragma unroll
      for (int u = 0; u < 4; ++u) part[u] += S[(long)(k + 8 * u) * per];
    for (; k < J.splits; k += 8) part[0] += S[(long)k * per];
    s = (part[0] + part[1]) + (part[2] + part[3]);
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (valid && lane8 == 0) jobs[j].dW[e] = s;
}

hipError_t launch_state(const WgradJob* jobs_dev, const int* wg_prefix_dev, int njobs, int total_wgs,
                        const int* red_prefix_dev, int total_red, float* slab, int d, int dh, int pts, int nw,
                        bool mfma, hipStream_t s) {
  if (njobs <= 0 || total_wgs <= 0) return hipSuccess;
  if (mfma) {
    if (!state_mfma_ok(d, dh)) return hipErrorInvalidValue;
    const int hpw = d / dh / 4;
    const dim3 grid(total_wgs), block(256);
#define GNOT_STATE_MFMA(DHV, HPWV)                                                                             \
    if (dh == DHV && hpw == HPWV) {                                                                            \
      hipLaunchKernelGGL((state_mfma_kernel<DHV, HPWV>), grid, block, 0, s, jobs_dev, wg_prefix_dev, njobs, slab, pts); \
    } else
    GNOT_STATE_MFMA(16, 1) GNOT_STATE_MFMA(16, 2) GNOT_STATE_MFMA(16, 4) GNOT_STATE_MFMA(32, 1) GNOT_STATE_MFMA(32, 2)
    GNOT_STATE_MFMA(32, 4) GNOT_STATE_MFMA(64, 1) GNOT_STATE_MFMA(64, 2) return hipErrorInvalidValue;
#undef GNOT_STATE_MFMA
    hipLaunchKernelGGL(state_reduce_kernel, dim3((total_red * 8 + 255) / 256), dim3(256), 0, s, jobs_dev, red_prefix_dev,
                       njobs, total_red, (const float*)slab);
    return hipGetLastError();
  }
  // dynamic LDS, what the workgroup stages: A and B rows (pts * d floats each, rounded up to whole
  // DMA instructions) + the per-(point, head) weights; the partial-state combine reuses the A/B region
  // (256 x 20 floats)
  const size_t lds = std::max<size_t>((size_t)(2 * state_stage_floats(pts, d) + pts * nw), 256 * 20) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(state_partial_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)((2 * 8192 + 64 * 64) * sizeof(float)));
    attr = true;
  }
  hipLaunchKernelGGL(state_partial_kernel, dim3(total_wgs), dim3(kStateThreads), lds, s, jobs_dev, wg_prefix_dev,
                     njobs, slab, pts);
  hipLaunchKernelGGL(state_reduce_kernel, dim3((total_red * 8 + 255) / 256), dim3(256), 0, s, jobs_dev, red_prefix_dev,
                     njobs, total_red, (const float*)slab);
  return hipGetLastError();
}

}  // namespace gnot
