// Prototype (microbenchmark only, not in the library): the d = 256 chain forward with 32 points per
// wave on v_mfma_f32_32x32x16_bf16 (bf16x6), one wave per SIMD, to measure whether the 32x32 shape
// (24 of 32 issue cycles free per MFMA instead of 8 of 16) lifts the chain off its issue bound.
//   lane (r = lane & 31, h = lane >> 5) carries point r of the wave; a 32-feature output tile o is
//   acc[reg] = feature 32o + (reg & 3) + 8 (reg >> 2) + 4h, so registers 8s..8s+7 of tile o are, after
//   GELU and the three-piece split, the next layer's B fragment of k-block 2o + s with no lane movement.
//   Weight images: image[((o * 16 + kb) * 3 + q) * 64 + lane] = 8 bf16 of piece q of row 32o + r,
//   k = 16 kb + 8 (j >> 2) + 4h + (j & 3), j = 0..7.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gnot_common.h"
#include "x6_core.h"

namespace gnot {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int C3W = 4;                         // waves per workgroup (one per SIMD)
constexpr int C3Tile = 16 * 3 * 64;            // u32x4 per output-tile image (48 KiB)

GNOT_DEV f32x16 mfma32(const u32x4& a, const u32x4& b, f32x16 c) {
#ifdef C3_NO_MFMA
  asm volatile("" : "+v"(c) : "v"(a), "v"(b));
  return c;
#endif
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

#ifndef C3_SCHED
#define C3_SCHED 0
#endif
#ifndef C3_NV
#define C3_NV 3
#endif
// per k-block scheduling: 0 = the block's 3 LDS reads, its 6 MFMAs, then the epilogue share (fenced);
// 1 = the reads, then 6 x (one MFMA, C3_NV VALU), epilogue unfenced so its VALU fills the MFMA gaps
GNOT_DEV void c3_sched(int kb) {
  if (kb + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#if C3_SCHED == 1
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, C3_NV, 0);
  }
#else
  __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  __builtin_amdgcn_sched_barrier(0);
#endif
}
GNOT_DEV void c3_fence() {
#if C3_SCHED == 0
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// DMA instruction i (0 .. 11) of this wave's share of a 48 KiB tile image
GNOT_DEV void c3_dma_piece(u32x4* nb, rsrc_t r, int w, int lane, int i) {
#ifndef C3_NO_DMA
  const int base = (w + i * C3W) * 64;
  dma16(r, nb + base, lane * 16, base * 16);
#endif
}

template <int N>
GNOT_DEV void c3_wait_bar() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// one layer: 8 output tiles of the layer input f (fp32, 16 k-blocks x 8 values of this lane), which tile
// 0 splits into three bf16 pieces k-block by k-block as it consumes them; the tiles' GELU outputs are
// written back into f (the epilogue of tile o - 1 runs inside tile o's MFMA stream, the last one after)
GNOT_DEV void c3_layer(u32x4* lds, int& cnt, const u32x4* W, const u32x4* nextW, const float* bias_lds,
                       rsrc_t rs, int rowoff, float (&f)[16][8], int wave, int lane, bool first) {
  const int h = lane >> 5;
  u32x4 in[16][3];
  f32x16 prev;
  auto store_h = [&](int o, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      buf_store_f32x4(make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]), rs,
                      rowoff + (32 * o + 8 * q + 4 * h) * 4);
  };
  auto gelu2 = [&](int o, const f32x16& acc, int i) {   // registers 2i, 2i + 1 of tile o
    f[2 * o + (i >> 2)][(2 * i) & 7] = gelu(acc[2 * i]);
    f[2 * o + (i >> 2)][(2 * i + 1) & 7] = gelu(acc[2 * i + 1]);
    asm volatile("" : "+v"(f[2 * o + (i >> 2)][(2 * i) & 7]), "+v"(f[2 * o + (i >> 2)][(2 * i + 1) & 7]));
  };
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    // this tile's chunk (DMA'd one tile ahead) must have landed; stores since then: 4 (epilogue o-2's,
    // issued during tile o-1), or, at o == 0, the last layer's tile-7 epilogue too
    c3_wait_bar<0>();
    const u32x4* cb = lds + (cnt & 1) * C3Tile;
    u32x4* nb = lds + ((cnt + 1) & 1) * C3Tile;
    ++cnt;
    const u32x4* src = o + 1 < 8 ? W + (size_t)(o + 1) * C3Tile : nextW;
    const rsrc_t rw = make_rsrc(src, src ? (unsigned)C3Tile * 16u : 0u);
    const int w = __builtin_amdgcn_readfirstlane(wave);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = bias_lds[32 * o + (r & 3) + 8 * (r >> 2) + 4 * h];
    if (o == 0) split8_x6(f[0], in[0]);
    u32x4 ab[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) ab[0][q] = cb[q * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
      if (kb + 1 < 16) {
#pragma unroll
        for (int q = 0; q < 3; ++q) ab[(kb + 1) & 1][q] = cb[((kb + 1) * 3 + q) * 64 + lane];
      }
#if C3_SCHED == 2
      const u32x4(&a)[3] = ab[kb & 1];
      // per-MFMA gap work, fenced: the epilogue of tile o - 1 (GELU of register kb of prev in six steps, the
      // save store of quad kb at kb < 4) or, in tile 0, the split of k-block kb + 1 in six steps
      float gx = prev[kb], gt = 0.f, gP = 0.f, ge = 0.f, gq = 0.f, gr = 0.f;
      unsigned w0[8], w1[8], w2[8];
      auto gap = [&](int m) __attribute__((always_inline)) {
        if (m == 0) {
          if (kb < 12) c3_dma_piece(nb, rw, w, lane, kb);
        }
        if (o > 0) {
          if (m == 0) gt = __builtin_amdgcn_rcpf(fmaf(fabsf(gx), 0.3275911f * kSqrt1_2, 1.0f));
          if (m == 1) { gP = fmaf(gt, 0.5f * 1.061405429f, 0.5f * -1.453152027f); gP = fmaf(gt, gP, 0.5f * 1.421413741f); }
          if (m == 2) { gP = fmaf(gt, gP, 0.5f * -0.284496736f); gP = fmaf(gt, gP, 0.5f * 0.254829592f); }
          if (m == 3) ge = __builtin_amdgcn_exp2f(gx * (gx * -0.72134752044448170368f));
          if (m == 4) { gq = (gP * gt) * ge; asm("v_max_f32 %0, 0, %1" : "=v"(gr) : "v"(gx)); }
          if (m == 5) {
            f[2 * (o - 1) + (kb >> 3)][kb & 7] = fmaf(-fabsf(gx), gq, gr);
            if (kb < 4)
              buf_store_f32x4(make_float4(prev[4 * kb], prev[4 * kb + 1], prev[4 * kb + 2], prev[4 * kb + 3]), rs,
                              rowoff + (32 * (o - 1) + 8 * kb + 4 * h) * 4);
          }
        } else if (kb + 1 < 16) {
          if (m < 4) {
#pragma unroll
            for (int j = 2 * m; j < 2 * m + 2; ++j) {
              const float v = f[kb + 1][j];
              const unsigned b = f2u(v);
              const float r1 = v - u2f(b & 0xFFFF0000u);
              const unsigned b1 = f2u(r1);
              w0[j] = b; w1[j] = b1; w2[j] = f2u(r1 - u2f(b1 & 0xFFFF0000u));
            }
          } else if (m == 4) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              in[kb + 1][0][d] = pack_hi16(w0[2 * d + 1], w0[2 * d]);
              in[kb + 1][1][d] = pack_hi16(w1[2 * d + 1], w1[2 * d]);
            }
          } else {
#pragma unroll
            for (int d = 0; d < 4; ++d) in[kb + 1][2][d] = pack_hi16(w2[2 * d + 1], w2[2 * d]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      acc = mfma32(a[2], in[kb][0], acc);
      gap(0);
      acc = mfma32(a[1], in[kb][1], acc);
      gap(1);
      acc = mfma32(a[0], in[kb][2], acc);
      gap(2);
      acc = mfma32(a[1], in[kb][0], acc);
      gap(3);
      acc = mfma32(a[0], in[kb][1], acc);
      gap(4);
      acc = mfma32(a[0], in[kb][0], acc);
      gap(5);
    }
#else
      const u32x4(&a)[3] = ab[kb & 1];
      acc = mfma32(a[2], in[kb][0], acc);
      acc = mfma32(a[1], in[kb][1], acc);
      acc = mfma32(a[0], in[kb][2], acc);
      acc = mfma32(a[1], in[kb][0], acc);
      acc = mfma32(a[0], in[kb][1], acc);
      acc = mfma32(a[0], in[kb][0], acc);
      c3_sched(kb);
      if (o > 0 && kb == 0) store_h(o - 1, prev);
      if (kb < 12) c3_dma_piece(nb, rw, w, lane, kb);   // no next image: a 0-byte resource, nothing is read
      if (o == 0) {
        if (kb + 1 < 16) split8_x6(f[kb + 1], in[kb + 1]);
      } else {
        if (kb >= 1 && kb <= 8) gelu2(o - 1, prev, kb - 1);
      }
      c3_fence();
    }
#endif
    prev = acc;
  }
  store_h(7, prev);
#pragma unroll
  for (int i = 0; i < 8; ++i) gelu2(7, prev, i);
}

__global__ void __launch_bounds__(64 * C3W) c3f_kernel(const float* __restrict__ X, const u32x4* __restrict__ W,
                                                       const float* __restrict__ bias, float* __restrict__ save,
                                                       int P, int NL) {
  extern __shared__ u32x4 lds[];
  float* bias_lds = reinterpret_cast<float*>(lds + 2 * C3Tile);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < NL * 256; i += 64 * C3W) bias_lds[i] = bias[i];
  const int h = lane >> 5;
  const long p = ((long)blockIdx.x * C3W + wave) * 32 + (lane & 31);
  const bool valid = p < P;
  float f[16][8];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb)
#pragma unroll
    for (int j = 0; j < 8; ++j) f[kb][j] = valid ? X[p * 256 + 16 * kb + 8 * (j >> 2) + 4 * h + (j & 3)] : 0.f;
  int cnt = 0;
  dma_image_n<C3Tile, C3W>(lds, W, wave, lane);
  const int rowoff = (int)(p * 1024);
  const size_t L = (size_t)8 * C3Tile;
  for (int l = 0; l < NL; ++l) {
    const rsrc_t r = make_rsrc(save + (size_t)l * P * 256, (unsigned)P * 1024u);
    c3_layer(lds, cnt, W + l * L, l + 1 < NL ? W + (l + 1) * L : nullptr, bias_lds + l * 256, r, rowoff, f, wave,
             lane, l == 0);
  }
}

// ---- backward: g = W_l^T dz_l (A = the transposed image), dz_{l-1} = g * gelu'(h_{l-1}) stored and carried
// as the next layer's input; HAS_H false: the chain's first Linear (g = dX, stored).  h_{l-1} of tile o is
// loaded into registers at tile o's start (4 x 16 B per lane) and consumed by tile o's epilogue, which
// runs inside tile o + 1.  Vector-memory order per tile o: [wait] DMA(o+1) hload(o) ... stores(o-1).
template <int N>
GNOT_DEV void c3_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
GNOT_DEV void c3_vmwait_n(int n) {
  switch (n) {
    case 4: c3_vmwait<4>(); break;
    case 8: c3_vmwait<8>(); break;
    case 12: c3_vmwait<12>(); break;
    case 16: c3_vmwait<16>(); break;
    case 20: c3_vmwait<20>(); break;
    default: c3_vmwait<0>(); break;
  }
}
template <int N>
GNOT_DEV void c3_wait_bar_n(int n) {
  switch (n) {
    case 4: c3_wait_bar<4>(); break;
    case 8: c3_wait_bar<8>(); break;
    case 12: c3_wait_bar<12>(); break;
    default: c3_wait_bar<0>(); break;
  }
}
GNOT_DEV void c3b_layer(u32x4* lds, int& cnt, const u32x4* W, const u32x4* nextW, rsrc_t rh, rsrc_t rs,
                        int rowoff, float (&f)[16][8], int wave, int lane, int first_wait, bool HAS_H) {
  const int h = lane >> 5;
  const int HL = HAS_H ? 4 : 0;
  u32x4 in[16][3];
  f32x16 prev;
  float4 hv[2][4];
  auto epi = [&](int o, const f32x16& acc, int q) {   // quad q: registers 4q .. 4q + 3
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r] = HAS_H ? acc[4 * q + r] * gelu_grad(hv[o & 1][q][r]) : acc[4 * q + r];
    }
    buf_store_f32x4(make_float4(d[0], d[1], d[2], d[3]), rs, rowoff + (32 * o + 8 * q + 4 * h) * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f[2 * o + (q >> 1)][4 * (q & 1) + r] = d[r];
      asm volatile("" : "+v"(f[2 * o + (q >> 1)][4 * (q & 1) + r]));
    }
  };
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    c3_wait_bar<0>();
    const u32x4* cb = lds + (cnt & 1) * C3Tile;
    u32x4* nb = lds + ((cnt + 1) & 1) * C3Tile;
    ++cnt;
    const u32x4* src = o + 1 < 8 ? W + (size_t)(o + 1) * C3Tile : nextW;
    const rsrc_t rw = make_rsrc(src, src ? (unsigned)C3Tile * 16u : 0u);
    const int w = __builtin_amdgcn_readfirstlane(wave);
    if (HAS_H) {
#pragma unroll
      for (int q = 0; q < 4; ++q) hv[o & 1][q] = buf_load_f32x4(rh, rowoff + (32 * o + 8 * q + 4 * h) * 4, 0);
    }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if (o == 0) split8_x6(f[0], in[0]);
    u32x4 ab[2][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) ab[0][q] = cb[q * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
      if (kb + 1 < 16) {
#pragma unroll
        for (int q = 0; q < 3; ++q) ab[(kb + 1) & 1][q] = cb[((kb + 1) * 3 + q) * 64 + lane];
      }
      const u32x4(&a)[3] = ab[kb & 1];
      acc = mfma32(a[2], in[kb][0], acc);
      acc = mfma32(a[1], in[kb][1], acc);
      acc = mfma32(a[0], in[kb][2], acc);
      acc = mfma32(a[1], in[kb][0], acc);
      acc = mfma32(a[0], in[kb][1], acc);
      acc = mfma32(a[0], in[kb][0], acc);
      c3_sched(kb);
      if (kb < 12) c3_dma_piece(nb, rw, w, lane, kb);   // no next image: a 0-byte resource, nothing is read
      if (o == 0) {
        if (kb + 1 < 16) split8_x6(f[kb + 1], in[kb + 1]);
      } else if (kb >= 1 && kb <= 4) {
        epi(o - 1, prev, kb - 1);   // hload(o - 1) landed before this tile's barrier (vmcnt(0))
      }
      c3_fence();
    }
    prev = acc;
  }
  if (HAS_H) c3_vmwait<0>();
#pragma unroll
  for (int q = 0; q < 4; ++q) epi(7, prev, q);
}

// dY [P][256] -> dz_{l-1} for l = NL-1 .. 1 into dz[l-1], dX into dX; h [NL-1][P][256] (saves of the forward)
__global__ void __launch_bounds__(64 * C3W) c3b_kernel(const float* __restrict__ dY, const u32x4* __restrict__ WT,
                                                       const float* __restrict__ hsave, float* __restrict__ dz,
                                                       float* __restrict__ dX, int P, int NL) {
  extern __shared__ u32x4 lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const long p = ((long)blockIdx.x * C3W + wave) * 32 + (lane & 31);
  const bool valid = p < P;
  float f[16][8];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb)
#pragma unroll
    for (int j = 0; j < 8; ++j) f[kb][j] = valid ? dY[p * 256 + 16 * kb + 8 * (j >> 2) + 4 * h + (j & 3)] : 0.f;
  int cnt = 0;
  const size_t L = (size_t)8 * C3Tile;
  dma_image_n<C3Tile, C3W>(lds, WT + (NL - 1) * L, wave, lane);
  const int rowoff = (int)(p * 1024);
  const unsigned lay = (unsigned)P * 1024u;
  int fw = 0;
  for (int l = NL - 1; l >= 0; --l) {
    const bool hh = l > 0;
    c3b_layer(lds, cnt, WT + l * L, hh ? WT + (l - 1) * L : nullptr,
              make_rsrc(hh ? hsave + (size_t)(l - 1) * P * 256 : nullptr, hh ? lay : 0u),
              make_rsrc(hh ? dz + (size_t)(l - 1) * P * 256 : dX, lay), rowoff, f, wave, lane, fw, hh);
    fw = 12;   // after a layer with h: hload(7), stores(6), stores(7) are younger than the next tile-0 DMA
  }
}

}  // namespace gnot

using namespace gnot;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

static unsigned short bf_trunc(float x) {
  unsigned u;
  std::memcpy(&u, &x, 4);
  return (unsigned short)(u >> 16);
}
static float bf_f(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 262144;
  const int NL = argc > 2 ? std::atoi(argv[2]) : 5;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
  std::vector<float> hX((size_t)P * 256), hW((size_t)NL * 256 * 256), hb((size_t)NL * 256);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : hX) v = rnd();
  for (auto& v : hW) v = rnd() * 0.0625f;
  for (auto& v : hb) v = rnd() * 0.1f;
  // images: [l][o][kb][q][lane] 8 bf16: row 32o + r, k = 16kb + 8(j>>2) + 4h + (j&3)
  std::vector<unsigned short> img((size_t)NL * 8 * C3Tile * 8);
  for (int l = 0; l < NL; ++l)
    for (int o = 0; o < 8; ++o)
      for (int kb = 0; kb < 16; ++kb)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int r = lane & 31, h = lane >> 5;
            const int row = 32 * o + r, k = 16 * kb + 8 * (j >> 2) + 4 * h + (j & 3);
            float w = hW[((size_t)l * 256 + row) * 256 + k];
            for (int q = 0; q < 3; ++q) {
              const unsigned short b = bf_trunc(w);
              img[((((size_t)(l * 8 + o) * 16 + kb) * 3 + q) * 64 + lane) * 8 + j] = b;
              w -= bf_f(b);
            }
          }
  float *dX, *db, *dsave;
  u32x4* dW;
  CK(hipMalloc(&dX, hX.size() * 4));
  CK(hipMalloc(&db, hb.size() * 4));
  CK(hipMalloc(&dsave, (size_t)NL * P * 256 * 4));
  CK(hipMalloc(&dW, img.size() * 2));
  CK(hipMemcpy(dX, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, img.data(), img.size() * 2, hipMemcpyHostToDevice));
  const int lds = 2 * C3Tile * 16 + NL * 256 * 4;
  CK(hipFuncSetAttribute((const void*)c3f_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int grid = (P + 32 * C3W - 1) / (32 * C3W);
  hipLaunchKernelGGL(c3f_kernel, dim3(grid), dim3(64 * C3W), lds, nullptr, dX, dW, db, dsave, P, NL);
  CK(hipDeviceSynchronize());
  // check a few points against a CPU double reference
  std::vector<float> hs((size_t)NL * P * 256);
  CK(hipMemcpy(hs.data(), dsave, hs.size() * 4, hipMemcpyDeviceToHost));
  double maxrel = 0;
  for (int pi = 0; pi < 64; ++pi) {
    const long p = (long)((pi * 104729L) % P);
    std::vector<double> a(256), hh(256);
    for (int k = 0; k < 256; ++k) a[k] = hX[p * 256 + k];
    for (int l = 0; l < NL; ++l) {
      for (int n = 0; n < 256; ++n) {
        double s = hb[l * 256 + n];
        for (int k = 0; k < 256; ++k) s += (double)hW[((size_t)l * 256 + n) * 256 + k] * a[k];
        hh[n] = s;
        const double g = hs[((size_t)l * P + p) * 256 + n];
        maxrel = std::max(maxrel, std::fabs(g - s) / (std::fabs(s) + 1e-3));
      }
      for (int n = 0; n < 256; ++n) a[n] = 0.5 * hh[n] * (1.0 + std::erf(hh[n] / std::sqrt(2.0)));
    }
  }
  std::printf("check: max rel err %.3e over 64 points x %d layers\n", maxrel, NL);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL(c3f_kernel, dim3(grid), dim3(64 * C3W), lds, nullptr, dX, dW, db, dsave, P, NL);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL(c3f_kernel, dim3(grid), dim3(64 * C3W), lds, nullptr, dX, dW, db, dsave, P, NL);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double fl = 2.0 * P * NL * 256.0 * 256.0;
  std::printf("c3f P=%d NL=%d: %.3f ms  %.1f TFLOP/s fp32-eq  (%.3f of the bf16x6 pipe 416.7)\n", P, NL, ms,
              fl / ms / 1e9, fl / ms / 1e9 / 416.67);
  // ---- backward: transposed images, dY random; h = the forward's saves (layers 0 .. NL-2)
  std::vector<unsigned short> imgT(img.size());
  for (int l = 0; l < NL; ++l)
    for (int o = 0; o < 8; ++o)
      for (int kb = 0; kb < 16; ++kb)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int r = lane & 31, h = lane >> 5;
            const int row = 32 * o + r, k = 16 * kb + 8 * (j >> 2) + 4 * h + (j & 3);
            float w = hW[((size_t)l * 256 + k) * 256 + row];     // W^T[row][k] = W[k][row]
            for (int q = 0; q < 3; ++q) {
              const unsigned short b = bf_trunc(w);
              imgT[((((size_t)(l * 8 + o) * 16 + kb) * 3 + q) * 64 + lane) * 8 + j] = b;
              w -= bf_f(b);
            }
          }
  std::vector<float> hdY((size_t)P * 256);
  for (auto& v : hdY) v = rnd();
  float *ddY, *ddz, *ddX;
  u32x4* dWT;
  CK(hipMalloc(&ddY, hdY.size() * 4));
  CK(hipMalloc(&ddz, (size_t)NL * P * 256 * 4));
  CK(hipMalloc(&ddX, (size_t)P * 256 * 4));
  CK(hipMalloc(&dWT, imgT.size() * 2));
  CK(hipMemcpy(ddY, hdY.data(), hdY.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dWT, imgT.data(), imgT.size() * 2, hipMemcpyHostToDevice));
  const int ldsb = 2 * C3Tile * 16;
  CK(hipFuncSetAttribute((const void*)c3b_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ldsb));
  hipLaunchKernelGGL(c3b_kernel, dim3(grid), dim3(64 * C3W), ldsb, nullptr, ddY, dWT, dsave, ddz, ddX, P, NL);
  CK(hipDeviceSynchronize());
  std::vector<float> hdz((size_t)NL * P * 256), hdX((size_t)P * 256);
  CK(hipMemcpy(hdz.data(), ddz, hdz.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hdX.data(), ddX, hdX.size() * 4, hipMemcpyDeviceToHost));
  double maxb = 0;
  for (int pi = 0; pi < 64; ++pi) {
    const long p = (long)((pi * 7919L + 13) % P);
    std::vector<double> d(256), g(256);
    for (int k = 0; k < 256; ++k) d[k] = hdY[p * 256 + k];
    for (int l = NL - 1; l >= 0; --l) {
      for (int n = 0; n < 256; ++n) {
        double s = 0;
        for (int k = 0; k < 256; ++k) s += (double)hW[((size_t)l * 256 + k) * 256 + n] * d[k];
        g[n] = s;
      }
      for (int n = 0; n < 256; ++n) {
        double v = g[n];
        if (l > 0) {
          const double x = hs[((size_t)(l - 1) * P + p) * 256 + n];
          const double Phi = 0.5 * (1.0 + std::erf(x / std::sqrt(2.0)));
          v *= Phi + x * std::exp(-0.5 * x * x) / std::sqrt(2.0 * M_PI);
        }
        const double gpu = l > 0 ? hdz[((size_t)(l - 1) * P + p) * 256 + n] : hdX[p * 256 + n];
        maxb = std::max(maxb, std::fabs(gpu - v) / (std::fabs(v) + 1e-3));
        d[n] = v;
      }
    }
  }
  std::printf("check bwd: max rel err %.3e over 64 points x %d layers\n", maxb, NL);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL(c3b_kernel, dim3(grid), dim3(64 * C3W), ldsb, nullptr, ddY, dWT, dsave, ddz, ddX, P, NL);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL(c3b_kernel, dim3(grid), dim3(64 * C3W), ldsb, nullptr, ddY, dWT, dsave, ddz, ddX, P, NL);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  std::printf("c3b P=%d NL=%d: %.3f ms  %.1f TFLOP/s fp32-eq  (%.3f of the bf16x6 pipe 416.7)\n", P, NL, ms,
              fl / ms / 1e9, fl / ms / 1e9 / 416.67);
  return 0;
}
