// Output-major bf16x6 point-form core shared by chain2.hip (MLP chains) and linear2.hip (projections)
// at hidden width d = 256: 8 waves x 16 points per workgroup, one weight chunk = one 16-feature output
// tile of an output-major x6 image (pack.hip x6 = 2), double-buffered through LDS by LDS-DMA.
#pragma once
#include <type_traits>

#include "gnot_common.h"

namespace gnot {

constexpr int kC2Waves = 8;

// u32x4 per output tile of an x6 image with KB k-blocks
constexpr int c2_tile_u4(int KB) { return KB * 3 * WAVE; }

// acc += sum_t W[o][t] . in[t] for one output tile: the weight pieces of k-block t+1 are read from
// LDS while the six MFMAs of block t run (smallest terms first, one accumulator)
template <int KB, bool AHEAD = true>
GNOT_DEV f32x4 c2_tile(const u32x4* __restrict__ cb, const u32x4 (&bp)[KB][3], f32x4 acc, int lane) {
  u32x4 a[AHEAD ? 2 : 1][3];
#pragma unroll
  for (int q = 0; q < 3; ++q) a[0][q] = cb[q * WAVE + lane];
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    if (!AHEAD && t > 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) a[0][q] = cb[(t * 3 + q) * WAVE + lane];
    }
    if (AHEAD && t + 1 < KB) {
#pragma unroll
      for (int q = 0; q < 3; ++q) a[(t + 1) & 1][q] = cb[((t + 1) * 3 + q) * WAVE + lane];
    }
    const u32x4(&w)[3] = a[AHEAD ? (t & 1) : 0];
    acc = mfma_bf16(w[2], bp[t][0], acc);
    acc = mfma_bf16(w[1], bp[t][1], acc);
    acc = mfma_bf16(w[0], bp[t][2], acc);
    acc = mfma_bf16(w[1], bp[t][0], acc);
    acc = mfma_bf16(w[0], bp[t][1], acc);
    acc = mfma_bf16(w[0], bp[t][0], acc);
  }
  return acc;
}

// The weight stream of one workgroup: chunk = one output tile.  `begin` waits for the chunk in flight,
// barriers, and starts the DMA of the following chunk (tile o+1 of this image, or `next` = the first
// tile of the next image, or nothing).
struct C2Stream {
  u32x4* lds;       // 2 buffers of `buf_u4`
  int buf_u4;
  int cnt = 0;
  int wave, lane;
  GNOT_DEV const u32x4* begin(const u32x4* img, int o, int OT, int tile_u4, const u32x4* next, int next_u4) {
    lds_dma_wait();
    __syncthreads();
    u32x4* nb = lds + ((cnt + 1) & 1) * buf_u4;
    const float4* src = nullptr;
    int n = 0;
    if (o + 1 < OT) { src = reinterpret_cast<const float4*>(img + (size_t)(o + 1) * tile_u4); n = tile_u4; }
    else if (next) { src = reinterpret_cast<const float4*>(next); n = next_u4; }
    if (src) stage_image(reinterpret_cast<float4*>(nb), src, n, kC2Waves, wave, lane);
    const u32x4* cb = lds + (cnt & 1) * buf_u4;
    ++cnt;
    return cb;
  }
};

template <int KT>
GNOT_DEV void c2_split(const float (&v)[KT][4], u32x4 (&bp)[(KT + 1) / 2][3]) {
#pragma unroll
  for (int t = 0; t < (KT + 1) / 2; ++t) split_block_x6<KT>(v, t, bp[t]);
}

GNOT_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// keeps a tile's epilogue results from being sunk to their far-away use (the next layer's split):
// deferred GELUs would keep every raw accumulator of the layer alive
GNOT_DEV void pin4(float (&v)[4]) { asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])); }

}  // namespace gnot
