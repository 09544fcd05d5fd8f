// Output-major bf16x6 point-form core shared by chain2.hip (MLP chains) and linear2.hip (projections)
// at hidden width d = 256: 8 waves x 16 points per workgroup, one weight chunk = one 16-feature output
// tile of an output-major x6 image (pack.hip x6 = 2), double-buffered through LDS by LDS-DMA.
#pragma once
#include <type_traits>

#include "gnot_common.h"

namespace gnot {

constexpr int kC2Waves = 8;
static_assert(kC2Rows == 16 * kC2Waves, "chain workgroup rows (gnot_kernels.h) != 16 points per wave");

// Piece count NP: 3 = the exact bf16x6 form (fp32 arithmetic), 1 = plain bf16 (RNE operands, fp32
// accumulation: the bf16 arithmetic mode, gnot_plan_set_precision).
// u32x4 per output tile of an image with KB k-blocks
constexpr int c2_tile_u4(int KB, int NP = 3) { return KB * NP * WAVE; }

// acc += sum_t W[o][t] . in[t] for one output tile: the weight pieces of k-block t+1 are read from
// LDS while the MFMAs of block t run (x6: the six order <= 2 products, smallest terms first, one
// accumulator; bf16: one product)
// fragment sets in flight: bf16x6 one k-block ahead (its six MFMAs cover the next block's LDS latency);
// one piece three ahead (a single 16-cycle MFMA per block would leave each read's latency exposed)
template <int NP, bool AHEAD>
constexpr int c2_frag_depth() { return AHEAD ? (NP == 1 ? 4 : 2) : 1; }
template <int KB, bool AHEAD = true, int NP = 3>
GNOT_DEV f32x4 c2_tile(const u32x4* __restrict__ cb, const u32x4 (&bp)[KB][NP], f32x4 acc, int lane) {
  constexpr int DP = c2_frag_depth<NP, AHEAD>();
  u32x4 a[DP][NP];
#pragma unroll
  for (int d = 0; d + 1 < DP || d == 0; ++d)
    if (d < KB) {
#pragma unroll
      for (int q = 0; q < NP; ++q) a[d][q] = cb[(d * NP + q) * WAVE + lane];
    }
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    if (!AHEAD && t > 0) {
#pragma unroll
      for (int q = 0; q < NP; ++q) a[0][q] = cb[(t * NP + q) * WAVE + lane];
    }
    if (AHEAD && t + DP - 1 < KB) {
#pragma unroll
      for (int q = 0; q < NP; ++q) a[(t + DP - 1) % DP][q] = cb[((t + DP - 1) * NP + q) * WAVE + lane];
    }
    const u32x4(&w)[NP] = a[AHEAD ? (t % DP) : 0];
    if constexpr (NP == 3) {
      acc = mfma_bf16(w[2], bp[t][0], acc);
      acc = mfma_bf16(w[1], bp[t][1], acc);
      acc = mfma_bf16(w[0], bp[t][2], acc);
      acc = mfma_bf16(w[1], bp[t][0], acc);
      acc = mfma_bf16(w[0], bp[t][1], acc);
    }
    acc = mfma_bf16(w[0], bp[t][0], acc);
    if (AHEAD) {
      if (t + DP - 1 < KB) __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NP == 3 ? 6 : 1, 0);
    }
  }
  return acc;
}

// c2_tile with the previous tile's epilogue split into 4 parts, part i placed after the MFMAs of k-block
// 2i+1 (the rest after the last block when KB < 8).  sched_barrier pins the order for the scheduler and
// the epilogue pins its results with empty asm (IR sinking would otherwise move them to their uses), so
// the VALU issues in this wave's own MFMA shadows instead of as one burst after the tile that both
// waves of a SIMD reach together.
// `pre` runs right after k-block 0's fragment reads are issued (the tile's DMA issue goes there, so its
// issue time overlaps their LDS latency instead of delaying them behind the barrier).
struct C2NoPre {
  GNOT_DEV void operator()() const {}
};
template <int KB, int NP, bool AHEAD, typename Epi, typename Pre = C2NoPre>
GNOT_DEV f32x4 c2_tile_epi(const u32x4* __restrict__ cb, const u32x4 (&bp)[KB][NP], f32x4 acc, int lane, Epi&& epi,
                           Pre&& pre = Pre()) {
  constexpr int DP = c2_frag_depth<NP, AHEAD>();
  u32x4 ab[DP][NP];
  if (AHEAD) {
#pragma unroll
    for (int d = 0; d + 1 < DP; ++d)
      if (d < KB) {
#pragma unroll
        for (int q = 0; q < NP; ++q) ab[d][q] = cb[(d * NP + q) * WAVE + lane];
      }
  }
  __builtin_amdgcn_sched_barrier(0);
  pre();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    if (AHEAD) {
      if (t + DP - 1 < KB) {
#pragma unroll
        for (int q = 0; q < NP; ++q) ab[(t + DP - 1) % DP][q] = cb[((t + DP - 1) * NP + q) * WAVE + lane];
      }
    } else {
#pragma unroll
      for (int q = 0; q < NP; ++q) ab[0][q] = cb[(t * NP + q) * WAVE + lane];
    }
    const u32x4(&a)[NP] = ab[AHEAD ? (t % DP) : 0];
    if constexpr (NP == 3) {
      acc = mfma_bf16(a[2], bp[t][0], acc);
      acc = mfma_bf16(a[1], bp[t][1], acc);
      acc = mfma_bf16(a[0], bp[t][2], acc);
      acc = mfma_bf16(a[1], bp[t][0], acc);
      acc = mfma_bf16(a[0], bp[t][1], acc);
    }
    acc = mfma_bf16(a[0], bp[t][0], acc);
    if (AHEAD) {
      // keep the fragment reads DP-1 blocks ahead of block t's MFMAs (the scheduler otherwise sinks them
      // next to their use to save registers, exposing the LDS latency every block)
      if (t + DP - 1 < KB) __builtin_amdgcn_sched_group_barrier(0x100, NP, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NP == 3 ? 6 : 1, 0);
    }
    if ((t & 1) && (t >> 1) < 4) {
      __builtin_amdgcn_sched_barrier(0);
      epi(t >> 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = KB / 2; i < 4; ++i) epi(i);
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
  int nwaves = kC2Waves;   // waves of the workgroup sharing the stream
  GNOT_DEV const u32x4* begin(const u32x4* img, int o, int OT, int tile_u4, const u32x4* next, int next_u4) {
    lds_dma_wait();
    __syncthreads();
    u32x4* nb = lds + ((cnt + 1) & 1) * buf_u4;
    const float4* src = nullptr;
    int n = 0;
    if (o + 1 < OT) { src = reinterpret_cast<const float4*>(img + (size_t)(o + 1) * tile_u4); n = tile_u4; }
    else if (next) { src = reinterpret_cast<const float4*>(next); n = next_u4; }
    if (src) stage_image(reinterpret_cast<float4*>(nb), src, n, nwaves, wave, lane);
    const u32x4* cb = lds + (cnt & 1) * buf_u4;
    ++cnt;
    return cb;
  }
};

// ---- counted LDS-DMA pipeline (chain2.hip) ------------------------------------------------------
// hipcc drains every outstanding vector-memory op (vmcnt(0)) at a __syncthreads() or at the use of an
// ordinary load while an LDS-DMA is in flight, which also waits for the epilogue stores issued just
// before.  The chains therefore use ONLY LDS-DMA loads inside the tile loop (weights, bias, saved
// pre-activations) and a raw barrier preceded by a COUNTED wait: vmcnt(N) with N = the vector-memory
// ops this wave issued after the DMA that must have landed (in-order completion), so the last tile's
// stores stay in flight across the barrier.
template <int N>
GNOT_DEV void c2_sync() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
// counted wait without a barrier (the wave's own LDS-DMA)
template <int N>
GNOT_DEV void c2_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
GNOT_DEV void c2_sync_n(int n) {   // n is wave-uniform and small
  switch (n) {
    case 1: c2_sync<1>(); break;
    case 2: c2_sync<2>(); break;
    case 3: c2_sync<3>(); break;
    case 4: c2_sync<4>(); break;
    case 5: c2_sync<5>(); break;
    case 6: c2_sync<6>(); break;
    case 7: c2_sync<7>(); break;
    case 8: c2_sync<8>(); break;
    case 9: c2_sync<9>(); break;
    case 10: c2_sync<10>(); break;
    case 11: c2_sync<11>(); break;
    case 12: c2_sync<12>(); break;
    case 13: c2_sync<13>(); break;
    case 14: c2_sync<14>(); break;
    case 15: c2_sync<15>(); break;
    case 16: c2_sync<16>(); break;
    default: c2_sync<0>(); break;
  }
}
// the weight-chunk stream of a chain kernel (chain2.hip): a ring of kC2Ring chunk buffers.  The
// forward keeps one chunk in flight (cur / nxt by the chunk count cnt); the backward keeps
// c2b_lead<NP>() in flight at static ring positions and waits for a chunk with a counted vmcnt: `issued`
// counts this wave's vector-memory ops as they are issued, mark[b] is that count right after the DMA of
// the chunk in buffer b, so issued - mark[b] ops are younger than it
constexpr int kC2Ring = 4;
#ifdef GNOT_DIAG_STAMP
// DIAGNOSTIC builds only (lib/microbench_st): in-kernel clock stamps around the chain kernels' per-chunk
// wait + barrier (cdna_hip_programming.md section 7, In-kernel stamps); sums leave through ChainArgs::dbg
GNOT_DEV unsigned long long c2_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif
struct C2Pipe {
  u32x4* lds;
  int WB;
  int cnt;          // weight chunks consumed (ring position)
  int wave, lane;
  int issued = 0;
  int mark[kC2Ring] = {};
#ifdef GNOT_DIAG_STAMP
  unsigned long long ts_body = 0, ts_sync = 0, ts_n = 0, ts_last = 0;
  GNOT_DEV unsigned long long stamp_in() {
    const unsigned long long t = c2_stamp();
    if (ts_last) ts_body += t - ts_last;
    return t;
  }
  GNOT_DEV void stamp_out(unsigned long long t0) {
    ts_last = c2_stamp();
    ts_sync += ts_last - t0;
    ++ts_n;
  }
#endif
  GNOT_DEV const u32x4* cur() const { return lds + (cnt % kC2Ring) * WB; }
  GNOT_DEV u32x4* nxt() const { return lds + ((cnt + 1) % kC2Ring) * WB; }
};
// this wave's instruction count of dma_image(lds, src, n16, nwaves, wave, lane)
GNOT_DEV int dma_image_count(int n16, int nwaves, int wave) {
  const int w = __builtin_amdgcn_readfirstlane(wave);
  return w * 64 < n16 ? (n16 - w * 64 + nwaves * 64 - 1) / (nwaves * 64) : 0;
}

// LDS read of a slot this wave filled by LDS-DMA and already waited for with a counted vmcnt: inline
// asm, so hipcc does not insert its own vmcnt(0) for the DMA still in flight to OTHER buffers (it cannot
// tell the addresses apart and would drain the whole pipeline)
GNOT_DEV float4 lds_read16_sync(const u32x4* p) {
  float4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// the same read WITHOUT the wait: the result registers are valid only after a later
// `s_waitcnt lgkmcnt(0)` asm that names them as in/out operands (so the compiler does not touch them
// in between); an LDS op older than the compiler's own only makes its counted waits stricter
GNOT_DEV f32x4 lds_read16_issue(const u32x4* p) {
  f32x4 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// 8-byte form of lds_read16_issue (bf16 saved tiles): `byte` is added to the slot address
GNOT_DEV u32x2 lds_read8_issue(const u32x4* p, int byte) {
  u32x2 v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) u32x4*)p + (unsigned)byte;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// this wave's own LDS-DMA (lane l: 16 B at lds + l) from a buffer resource at byte offset voff + soff
GNOT_DEV void dma16(rsrc_t r, u32x4* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)lds, 16, voff, soff, 0, 0);
}
// n16 16-byte units (a multiple of 64) of an image, split over the workgroup's waves
GNOT_DEV void dma_image(u32x4* lds, const void* src, int n16, int nwaves, int wave, int lane) {
  const rsrc_t r = make_rsrc(src, (unsigned)n16 * 16u);
  // the LDS base (M0) and soffset must be SGPRs: a wave index the compiler cannot prove uniform turns
  // every DMA into a waterfall loop
  const int w = __builtin_amdgcn_readfirstlane(wave);
  for (int base = w * WAVE; base < n16; base += nwaves * WAVE) dma16(r, lds + base, lane * 16, base * 16);
}

// the same with the size known at compile time: unrolled (no loop counter and branch per DMA)
template <int N16, int NW>
GNOT_DEV void dma_image_n(u32x4* lds, const void* src, int wave, int lane) {
  const rsrc_t r = make_rsrc(src, (unsigned)N16 * 16u);
  const int w = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
  for (int i = 0; i < (N16 + NW * WAVE - 1) / (NW * WAVE); ++i) {
    const int base = (w + i * NW) * WAVE;
    if ((i + 1) * NW * WAVE <= N16 || base < N16) dma16(r, lds + base, lane * 16, base * 16);
  }
}

template <int KT, int NP = 3>
GNOT_DEV void c2_split(const float (&v)[KT][4], u32x4 (&bp)[(KT + 1) / 2][NP]) {
#pragma unroll
  for (int t = 0; t < (KT + 1) / 2; ++t) split_block_x6<KT, NP>(v, t, bp[t]);
}

GNOT_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// keeps a tile's epilogue results from being sunk to their far-away use (the next layer's split):
// deferred GELUs would keep every raw accumulator of the layer alive
GNOT_DEV void pin4(float (&v)[4]) { asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])); }

}  // namespace gnot
