// Shared device helpers for the GNOT MI355X (gfx950) kernels.
//
// Register "point form" used by every point-streaming kernel in this library
// ---------------------------------------------------------------------------
// A wave owns 16 consecutive points (rows of a [P, F] row-major activation).  Lane l holds
// point  p0 + (l & 15)  and, for every 16-feature tile T, the four features
//            16*T + 4*(l >> 4) + r ,  r = 0..3      ->  act[T][r]
// This is exactly the C/D layout of v_mfma_f32_16x16x4_f32 when the MFMA computes
// OUT^T = W * ACT^T (output features on MFMA rows, points on MFMA columns), and it is also the
// B-operand layout that the next 16x16x4 MFMA needs when it contracts over those features:
// B[k = l>>4][j = l&15] at k-step r is feature 16T + 4(l>>4) + r of point j.  A whole MLP chain
// therefore runs with activations resident in VGPRs, no LDS transpose between layers; only the
// weights (A operand) are streamed, from a pre-packed "fragment order" image (pack.hip) in which
// one wave-instruction reads 1 KiB contiguous (16 B per lane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GNOT_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace gnot {

constexpr int WAVE = 64;

// one k=4 step of the f32-input MFMA: acc(16x16) += A(16x4) * B(4x16)
GNOT_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc += W-fragment (float4 = 4 k-steps) x act tile (4 regs)
GNOT_DEV f32x4 mfma_k16(const float4 w, const float (&x)[4], f32x4 c) {
  c = mfma4(w.x, x[0], c);
  c = mfma4(w.y, x[1], c);
  c = mfma4(w.z, x[2], c);
  c = mfma4(w.w, x[3], c);
  return c;
}

constexpr float kSqrt1_2 = 0.70710678118654752440f;
constexpr float kInvSqrt2Pi = 0.39894228040143267794f;

// nn.GELU() (exact-erf form, reference model.py:10,13): gelu(x) = x * Phi(x), Phi(x) = (1 + erf(x/sqrt2))/2.
// erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, below fp32 rounding of the result for |x| > 1):
// one v_rcp, one v_exp and 4 FMAs instead of ocml erff's two-branch ~40-instruction sequence.  Written
// around the tail q = Phi(-|x|) = (1 - erf(|x|/sqrt2))/2 = t P(t) e^{-x^2/2} (the 1/2 folded into
// P's coefficients, 1/sqrt2 into t's, log2(e)/2 into the exponent's), so that
//   gelu(x)  = max(x, 0) - |x| q                      (no sign select: x Phi(x) = relu(x) - |x| Phi(-|x|))
//   gelu'(x) = Phi(x) + x phi(x),  Phi(x) = 1/2 + sign(x) (1/2 - q),  phi(x) = e^{-x^2/2} / sqrt(2 pi)
// 13 VALU for gelu (the chain epilogues run beside MFMAs, where VALU issue is the scarce resource).
GNOT_DEV float gelu_tail(float x, float& e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), 0.3275911f * kSqrt1_2, 1.0f));
  float P = fmaf(t, 0.5f * 1.061405429f, 0.5f * -1.453152027f);
  P = fmaf(t, P, 0.5f * 1.421413741f);
  P = fmaf(t, P, 0.5f * -0.284496736f);
  P = fmaf(t, P, 0.5f * 0.254829592f);
  e = __builtin_amdgcn_exp2f(x * (x * -0.72134752044448170368f));   // 2^(-x^2 log2(e) / 2) = e^{-x^2/2}
  return (P * t) * e;
}
GNOT_DEV float gelu(float x) {
  float e;
  const float q = gelu_tail(x, e);
  float r;                                  // max(x, 0) without fmaxf's NaN-quieting v_max(x, x)
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return fmaf(-fabsf(x), q, r);
}
// gelu(x) (bitwise as gelu()) and gelu'(x) from one tail evaluation
GNOT_DEV float gelu_and_grad(float x, float& dg) {
  float e;
  const float q = gelu_tail(x, e);
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  dg = fmaf(x * kInvSqrt2Pi, e, 0.5f + copysignf(0.5f - q, x));
  return fmaf(-fabsf(x), q, r);
}
GNOT_DEV float gelu_grad(float x) {
  float e;
  const float q = gelu_tail(x, e);
  const float Phi = 0.5f + copysignf(0.5f - q, x);
  return fmaf(x * kInvSqrt2Pi, e, Phi);
}

GNOT_DEV float shfl_xor(float v, int m) { return __shfl_xor(v, m, 64); }

// ---- point-form loads / stores ------------------------------------------------------------
// load KT tiles of row p (features 16T + 4g + r); features >= ncols read as 0; invalid rows -> 0
// (16-byte loads when the row pitch allows it; X must then be 16-byte aligned)
template <int KT>
GNOT_DEV void load_rows(float (&a)[KT][4], const float* __restrict__ X, long ld, long p, bool valid,
                        int ncols, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int T = 0; T < KT; ++T) {
    const int f = 16 * T + 4 * g;
    if (valid && f + 3 < ncols && (ld & 3) == 0) {
      const float4 v = *reinterpret_cast<const float4*>(X + p * ld + f);
      a[T][0] = v.x; a[T][1] = v.y; a[T][2] = v.z; a[T][3] = v.w;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) a[T][r] = (valid && f + r < ncols) ? X[p * ld + f + r] : 0.f;
    }
  }
}

template <int KT>
GNOT_DEV void store_rows(const float (&a)[KT][4], float* __restrict__ Y, long ld, long p, bool valid,
                         int ncols, int lane) {
  if (!valid) return;
  const int g = lane >> 4;
#pragma unroll
  for (int T = 0; T < KT; ++T) {
    const int f = 16 * T + 4 * g;
    if (f + 3 < ncols && (ld & 3) == 0) {
      *reinterpret_cast<float4*>(Y + p * ld + f) = make_float4(a[T][0], a[T][1], a[T][2], a[T][3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (f + r < ncols) Y[p * ld + f + r] = a[T][r];
    }
  }
}

// OUT^T(16*OT x 16 points) = W(16*OT x 16*KT) * IN^T with W given in packed fragment order:
// Wp[(o*KT + T)*64 + lane] = { W[16o + (lane&15)][16T + 4(lane>>4) + r] : r = 0..3 }
// acc must be pre-initialised (bias or zero).
template <int KT, int OT>
GNOT_DEV void mm_tiles(const float4* __restrict__ Wp, const float (&in)[KT][4], f32x4 (&acc)[OT],
                       int lane) {
#pragma unroll
  for (int T = 0; T < KT; ++T) {
    float4 w[OT];
#pragma unroll
    for (int o = 0; o < OT; ++o) w[o] = Wp[(o * KT + T) * WAVE + lane];
#pragma unroll
    for (int o = 0; o < OT; ++o) acc[o] = mfma_k16(w[o], in[T], acc[o]);
  }
}

// ---- LDS-staged weight images ---------------------------------------------------------------
// A layer's packed A-operand image (OT x KT tiles of 1 KiB) is copied into LDS by the whole
// workgroup with global_load_lds (16 B per lane, one 1 KiB wave-instruction each, no VGPRs), then every
// wave of the workgroup reads its fragments with ds_read_b128 (contiguous -> conflict free).  Images
// larger than kLdsImageKB are processed in chunks of `och` output tiles.
constexpr int kLdsImageKB = 64;

constexpr int lds_och(int KT, int OT) {
  int c = OT;
  while (c > 1 && (c * KT > kLdsImageKB || OT % c != 0)) --c;
  return c;
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) const void* global_cvoid_ptr;

// LDS-DMA (global_load_lds) writes are tracked ONLY by the issuing wave's vmcnt: a barrier alone does
// not make them visible (the compiler's workgroup fence waits for stores, not loads).  Every barrier
// that hands DMA'd LDS to other waves is preceded by this wait.
GNOT_DEV void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// copy n4 float4 (a multiple of 64) from global to LDS; all threads of the workgroup call this.
// Buffer form: the source base in SGPRs (one descriptor per copy), the lane's 16-byte offset in one
// VGPR and the wave-instruction's base in soffset -- no 64-bit per-lane addresses to keep alive.
GNOT_DEV void stage_image(float4* lds, const float4* __restrict__ g, int n4, int nwaves, int wave, int lane) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(g), (short)0, n4 * 16, 0x00020000);
  for (int base = wave * WAVE; base < n4; base += nwaves * WAVE)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(lds + base), 16, lane * 16, base * 16, 0, 0);
}

// acc[o] (o < OT) += W x in  with W (OT x KT tiles, packed) streamed through the LDS buffer `lds`
// (capacity >= lds_och(KT,OT)*KT*64 float4).  Contains __syncthreads(): call uniformly.
template <int KT, int OT>
GNOT_DEV void mm_tiles_lds(const float4* __restrict__ Wg, float4* lds, const float (&in)[KT][4], f32x4 (&acc)[OT],
                           int nwaves, int wave, int lane) {
  constexpr int OCH = lds_och(KT, OT);
#pragma unroll
  for (int c = 0; c < OT / OCH; ++c) {
    __syncthreads();                                   // previous readers of lds are done
    stage_image(lds, Wg + c * OCH * KT * WAVE, OCH * KT * WAVE, nwaves, wave, lane);
    lds_dma_wait();
    __syncthreads();
    // fragments of k-tile T+1 are read from LDS while the MFMAs of k-tile T run; within a k-tile the
    // MFMA order is k-step-outer / output-tile-inner, so consecutive MFMAs use independent
    // accumulators (the f32 16x16x4 MFMA has a 40-cycle dependent latency vs 32-cycle issue)
    float4 wc[OCH], wn[OCH];
#pragma unroll
    for (int o = 0; o < OCH; ++o) wc[o] = lds[(o * KT + 0) * WAVE + lane];
#pragma unroll
    for (int T = 0; T < KT; ++T) {
      if (T + 1 < KT) {
#pragma unroll
        for (int o = 0; o < OCH; ++o) wn[o] = lds[(o * KT + T + 1) * WAVE + lane];
      }
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].x, in[T][0], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].y, in[T][1], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].z, in[T][2], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].w, in[T][3], acc[c * OCH + o]);
      if (T + 1 < KT) {
#pragma unroll
        for (int o = 0; o < OCH; ++o) wc[o] = wn[o];
      }
    }
  }
}

// ---- pipelined weight stream ------------------------------------------------------------------
// Two LDS buffers of kChunkKB each.  A layer's image is consumed in chunks of `och` output tiles; while
// chunk i is multiplied, chunk i+1 (of this layer, or the first chunk of the NEXT layer) is already
// landing in the other buffer by LDS-DMA, so the weight stream never stalls the MFMAs at a layer
// boundary.  One barrier per chunk (after an explicit vmcnt(0)): it retires chunk i's DMA and frees the
// buffer chunk i-1 used.  `cnt` counts consumed chunks (buffer parity).
constexpr int kChunkKB = 16;
constexpr int kChunkF4 = kChunkKB * WAVE;          // float4 per buffer

constexpr int chunk_och(int KT, int OT) {
  int c = OT;
  while (c > 1 && (c * KT > kChunkKB || OT % c != 0)) --c;
  return c;
}
constexpr int chunk_f4(int KT, int OT) { return chunk_och(KT, OT) * KT * WAVE; }
// float4 per buffer of a KT-deep weight stream: kChunkF4, or one whole output tile when that is larger
// (KT > kChunkKB: the layer-wise kernels at d > 256)
template <int KT>
constexpr int pipe_buf_f4() { return KT * WAVE > kChunkF4 ? KT * WAVE : kChunkF4; }

struct NoHook {
  GNOT_DEV void operator()() const {}
};

template <int KT, int OT, typename Hook = NoHook>
GNOT_DEV void mm_tiles_pipe(const float4* __restrict__ Wg, const float4* __restrict__ next_W, int next_f4,
                            float4* lds, int& cnt, const float (&in)[KT][4], f32x4 (&acc)[OT], int nwaves,
                            int wave, int lane, Hook hook = Hook()) {
  constexpr int OCH = chunk_och(KT, OT);
  constexpr int NC = OT / OCH;
  constexpr int CH4 = OCH * KT * WAVE;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    lds_dma_wait();                                    // this chunk's DMA (issued one chunk ago) has landed
    __syncthreads();
    float4* nb = lds + ((cnt + 1) & 1) * pipe_buf_f4<KT>();
    if (c + 1 < NC) stage_image(nb, Wg + (c + 1) * CH4, CH4, nwaves, wave, lane);
    else if (next_W) stage_image(nb, next_W, next_f4, nwaves, wave, lane);
    if (c == 0) hook();   // e.g. prefetch the next layer's saved rows: a whole layer of MFMAs to land
    const float4* cb = lds + (cnt & 1) * pipe_buf_f4<KT>();
    float4 wc[OCH], wn[OCH];
#pragma unroll
    for (int o = 0; o < OCH; ++o) wc[o] = cb[(o * KT + 0) * WAVE + lane];
#pragma unroll
    for (int T = 0; T < KT; ++T) {
      if (T + 1 < KT) {
#pragma unroll
        for (int o = 0; o < OCH; ++o) wn[o] = cb[(o * KT + T + 1) * WAVE + lane];
      }
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].x, in[T][0], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].y, in[T][1], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].z, in[T][2], acc[c * OCH + o]);
#pragma unroll
      for (int o = 0; o < OCH; ++o) acc[c * OCH + o] = mfma4(wc[o].w, in[T][3], acc[c * OCH + o]);
      if (T + 1 < KT) {
#pragma unroll
        for (int o = 0; o < OCH; ++o) wc[o] = wn[o];
      }
    }
    ++cnt;
  }
}

// ---- fp32 GEMM on bf16 MFMAs, split three ways ("bf16x6") --------------------------------------
// Every fp32 operand is written EXACTLY as the sum of three bf16 pieces by truncation
// (v = v0 + v1 + v2: each piece keeps the next 8 significant bits of the 24-bit mantissa), and a
// product as the six terms of order <= 2:  a.b ~ a0b0 + (a0b1 + a1b0) + (a0b2 + a1b1 + a2b0).  Each
// term is an exact product of 8-bit mantissas; the dropped terms (a1b2, a2b1, a2b2) are < 2^-23
// relative, i.e. fp32 rounding level, and the order-0 term accumulates separately from the small
// ones.  Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight v_mfma_f32_16x16x4_f32 (32
// cycles each) per 16x16x32 block: 2.7x fewer matrix-pipe cycles at fp32-level accuracy.
//
// Point form carries over unchanged: for k-block t (features 32t..32t+31) lane (p, g) feeds MFMA
// k-slots 8g+j with its own registers: j < 4 -> feature 32t+4g+j (tile 2t), j >= 4 -> feature
// 32t+16+4g+(j-4) (tile 2t+1).  Weight images (pack.hip, x6 jobs) use the same k order, k-major:
// image[((t*OT + o)*3 + q)*64 + lane] = 8 bf16 of piece q of rows 16o+(lane&15), k-slots 8(lane>>4)+j.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// LDS buffer of the bf16x6 weight stream: 24 KiB per buffer, double-buffered.
// Images are k-MAJOR: block (t, o) = output tile o, k-block t (32 contraction slots) at
//   image[((t*OT + o)*3 + q)*64 + lane]
// so a chunk is TCH whole k-blocks (all OT output tiles) or, when one k-block of all tiles exceeds the
// buffer (d = 256), OCH output tiles of one k-block.  Consuming a layer k-block by k-block means only
// the current block's three B pieces are live (12 VGPRs instead of 12*ceil(KT/2)), which with a
// single accumulator set keeps the d = 128 forward chain at 3 waves per SIMD.
constexpr int x6_buf_kb(int) { return 24; }
constexpr int x6_buf_f4(int D) { return x6_buf_kb(D) * WAVE; }   // 16-byte units per buffer

// NP: pieces per block (3: bf16x6, 1: one RNE bf16 piece, the bf16 arithmetic mode; pack x6 = 1 / 4)
template <int D, int NP = 3>
constexpr int x6_och(int KT, int OT) {                // output tiles per chunk (NP KiB per block)
  int c = OT;
  while (c > 1 && (c * NP > x6_buf_kb(D) || OT % c != 0)) --c;
  return c;
}
template <int D, int NP = 3>
constexpr int x6_tch(int KT, int OT) {                // k-blocks per chunk
  const int KB = (KT + 1) / 2;
  if (x6_och<D, NP>(KT, OT) != OT) return 1;
  int c = KB;
  while (c > 1 && (c * OT * NP > x6_buf_kb(D) || KB % c != 0)) --c;
  return c;
}
template <int D, int NP = 3>
constexpr int x6_chunk_f4(int KT, int OT) { return x6_och<D, NP>(KT, OT) * x6_tch<D, NP>(KT, OT) * NP * WAVE; }

GNOT_DEV unsigned f2u(float x) { return __builtin_bit_cast(unsigned, x); }
// (hi & 0xFFFF0000) | (lo >> 16) in one v_perm_b32: the high halves of two words as two bf16
GNOT_DEV unsigned pack_hi16(unsigned hi, unsigned lo) { return __builtin_amdgcn_perm(hi, lo, 0x07060302u); }
GNOT_DEV float u2f(unsigned x) { return __builtin_bit_cast(float, x); }

// ---- buffer loads: base + bound in SGPRs (reads past `bytes` return 0), wave-uniform row offset in
// an SGPR (soffset), only the lane's column offset in a VGPR
typedef __amdgpu_buffer_rsrc_t rsrc_t;
// cache-policy operand of the buffer load / store builtins: sc1 (gfx950: write-through stores, L1-bypassing
// loads -- the device-coherent form of an inter-workgroup hand-off, MI355X_MICROARCH.md)
constexpr int kCpolSc1 = 16;
// (base and bound are wave-uniform by construction; readfirstlane tells the compiler so, otherwise a
// descriptor built from a value it cannot prove uniform is used inside a waterfall loop)
GNOT_DEV rsrc_t make_rsrc(const void* p, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* up = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(up, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
GNOT_DEV float buf_load_f32(rsrc_t r, int voff, int soff) {
  return u2f(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
GNOT_DEV float4 buf_load_f32x4(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
// stores past the resource's `bytes` are dropped (tail lanes need no predicate).
// The whole offset goes in the VGPR and soffset stays the constant 0: a 128-bit buffer store whose
// soffset is an SGPR is not padded by the compiler's hazard recognizer (ROCm 7.2) against a VALU
// overwriting its data registers on the next cycle, and on gfx950 the tail lanes then store the new
// value (measured: element 0 of lanes 12-15 of every 16, chain2 saves, DESIGN.md "store-data hazard").
GNOT_DEV void buf_store_f32x4(float4 v, rsrc_t r, int voff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, 0, 0);
}

// exact 3-piece truncation split of 8 floats: p[q] = 8 bf16 (4 dwords, element j in the low half
// of dword j/2 for even j) of piece q; v == piece0 + piece1 + piece2 exactly
GNOT_DEV void split8_x6(const float (&v)[8], u32x4 (&p)[3]) {
  unsigned w0[8], w1[8], w2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned b = f2u(v[j]);
    const float r1 = v[j] - u2f(b & 0xFFFF0000u);
    const unsigned b1 = f2u(r1);
    const float r2 = r1 - u2f(b1 & 0xFFFF0000u);
    w0[j] = b;
    w1[j] = b1;
    w2[j] = f2u(r2);
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    p[0][d] = pack_hi16(w0[2 * d + 1], w0[2 * d]);
    p[1][d] = pack_hi16(w1[2 * d + 1], w1[2 * d]);
    p[2][d] = pack_hi16(w2[2 * d + 1], w2[2 * d]);
  }
}

// round-to-nearest-even bf16 of a float (bf16 arithmetic mode: one piece instead of three)
GNOT_DEV unsigned bf16_rne_bits(float x) {
  const unsigned u = f2u(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
// RNE bf16 of two floats in one word: ONE v_cvt_pk_bf16_f32, the bits of bf16_rne_bits for finite values (round
// 6: the one-piece operand splits used bf16_rne_bits, five VALU per element -- 16 % of the bf16-mode chain
// forward's VALU stream -- for the same bits)
GNOT_DEV unsigned pk_bf16(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
// 8 floats -> 8 RNE bf16 (4 dwords, element j in the low half of dword j/2 for even j)
GNOT_DEV void split8_bf16(const float (&v)[8], u32x4 (&p)[1]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) p[0][d] = pk_bf16(v[2 * d], v[2 * d + 1]);
}
// NP = 3: the exact bf16x6 split; NP = 1: RNE bf16
template <int NP>
GNOT_DEV void split8_np(const float (&v)[8], u32x4 (&p)[NP]) {
  if constexpr (NP == 3) split8_x6(v, p);
  else split8_bf16(v, p);
}

// the split of ONE element pair (elements 2d, 2d+1 of an 8-element group): dword d of every piece,
// the same bits split8_np writes
template <int NP>
GNOT_DEV void split2_np(float v0, float v1, u32x4 (&p)[NP], int d) {
  if constexpr (NP == 3) {
    const unsigned a0 = f2u(v0), b0 = f2u(v1);
    const float ra = v0 - u2f(a0 & 0xFFFF0000u), rb = v1 - u2f(b0 & 0xFFFF0000u);
    const unsigned a1 = f2u(ra), b1 = f2u(rb);
    const unsigned a2 = f2u(ra - u2f(a1 & 0xFFFF0000u)), b2 = f2u(rb - u2f(b1 & 0xFFFF0000u));
    p[0][d] = pack_hi16(b0, a0);
    p[1][d] = pack_hi16(b1, a1);
    p[2][d] = pack_hi16(b2, a2);
  } else {
    p[0][d] = pk_bf16(v0, v1);
  }
}

// ---- bf16 activation rows (bf16 arithmetic mode, soft-MoE chains at d = 256) ---------------------
// "Pair-interleaved" (PI) rows of 256 bf16 = 512 B per point: feature f = 16T + 4g + r sits in 16-byte
// chunk (T >> 1) * 4 + g, 8-byte half T & 1, element r.  Chunk (t, g) of a point is exactly the word a
// point-form lane of group g packs for k-block t (split_block_x6: tiles 2t, 2t+1), so the chains load and
// store whole 16-byte operand words, and every 4 consecutive features (f % 4 == 0) are 8 contiguous
// bytes: the row pieces ds_read_b64_tr_b16 gathers in the weight-gradient kernel (wgrad.hip).
constexpr int kB16Row = 512;
GNOT_DEV int b16_off(int T, int g) { return ((T >> 1) * 4 + g) * 16 + (T & 1) * 8; }
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
GNOT_DEV float bf16_lo(unsigned w) { return u2f(w << 16); }
GNOT_DEV float bf16_hi(unsigned w) { return u2f(w & 0xFFFF0000u); }
// 8-byte buffer store (whole offset in the VGPR, soffset 0: see buf_store_f32x4)
GNOT_DEV void buf_store_b64(u32x2 v, rsrc_t r, int voff) { __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, 0, 0); }
GNOT_DEV void buf_store_b128(u32x4 v, rsrc_t r, int voff) { __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 0); }
// one point-form tile (4 features of this lane) as RNE bf16 at its PI position; rowoff = point * 512
GNOT_DEV void store_tile_b16(const float (&v)[4], rsrc_t r, int rowoff, int T, int g) {
  buf_store_b64(u32x2{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}, r, rowoff + b16_off(T, g));
}
// KT point-form tiles from / to PI bf16 rows (KT even; rows past the resource bound read 0 / are dropped)
template <int KT>
GNOT_DEV void load_rows_b16(float (&a)[KT][4], rsrc_t r, int rowoff, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < KT / 2; ++t) {
    const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(r, rowoff + (t * 4 + g) * 16, 0, 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a[2 * t + h][0] = bf16_lo(w[2 * h]);
      a[2 * t + h][1] = bf16_hi(w[2 * h]);
      a[2 * t + h][2] = bf16_lo(w[2 * h + 1]);
      a[2 * t + h][3] = bf16_hi(w[2 * h + 1]);
    }
  }
}
template <int KT>
GNOT_DEV void store_rows_b16(const float (&a)[KT][4], rsrc_t r, int rowoff, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < KT / 2; ++t)
    buf_store_b128(u32x4{pk_bf16(a[2 * t][0], a[2 * t][1]), pk_bf16(a[2 * t][2], a[2 * t][3]),
                         pk_bf16(a[2 * t + 1][0], a[2 * t + 1][1]), pk_bf16(a[2 * t + 1][2], a[2 * t + 1][3])},
                   r, rowoff + (t * 4 + g) * 16);
}

// B pieces of k-block t of the point-form activations in[KT][4]: bp[q] = 8 bf16 (4 dwords) of piece q
template <int KT, int NP = 3>
GNOT_DEV void split_block_x6(const float (&in)[KT][4], int t, u32x4 (&bp)[NP]) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = in[2 * t][j];
    v[4 + j] = (2 * t + 1 < KT) ? in[2 * t + 1][j] : 0.f;
  }
  split8_np<NP>(v, bp);
}

GNOT_DEV f32x4 mfma_bf16(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}

// Same contract as mm_tiles_pipe (acc pre-initialised, chunks double-buffered in `lds` of
// 2*x6_buf_f4 units, next image staged across the layer boundary, hook after the first chunk's
// barrier), for k-major x6 weight images.  Per 16x16x32 block the six order <= 2 products go into
// the tile's one accumulator, smallest terms first (a single accumulation chain of
// v_mfma_f32_16x16x32_bf16 issues at full rate, MI355X_MICROARCH.md).  NP = 1 (bf16 mode, one-piece
// k-major images, pack x6 = 4): one product per block, the input rounded to bf16 (RNE).
// `late` runs after the LAST chunk's barrier, before its MFMAs (its VALU then issues beside them)
template <int D, int KT, int OT, int NP = 3, typename Hook = NoHook, typename Late = NoHook>
GNOT_DEV void mm_tiles_pipe_x6(const float4* __restrict__ Wg, const float4* __restrict__ next_W, int next_f4,
                               float4* lds, int& cnt, const float (&in)[KT][4], f32x4 (&acc)[OT], int nwaves,
                               int wave, int lane, Hook hook = Hook(), Late late = Late()) {
  constexpr int kBufF4 = x6_buf_f4(D);
  constexpr int KB = (KT + 1) / 2;
  constexpr int OCH = x6_och<D, NP>(KT, OT);
  constexpr int TCH = x6_tch<D, NP>(KT, OT);
  constexpr int NOG = OT / OCH;
  constexpr int NTG = KB / TCH;
  constexpr int CH4 = OCH * TCH * NP * WAVE;
#pragma unroll
  for (int tg = 0; tg < NTG; ++tg) {
    u32x4 bp[TCH][NP];
#pragma unroll
    for (int tt = 0; tt < TCH; ++tt) split_block_x6<KT, NP>(in, tg * TCH + tt, bp[tt]);
#pragma unroll
    for (int og = 0; og < NOG; ++og) {
      const int c = tg * NOG + og;
      lds_dma_wait();
      __syncthreads();
      float4* nb = lds + ((cnt + 1) & 1) * kBufF4;
      if (c + 1 < NTG * NOG) stage_image(nb, Wg + (c + 1) * CH4, CH4, nwaves, wave, lane);
      else if (next_W) stage_image(nb, next_W, next_f4, nwaves, wave, lane);
      if (c == 0) hook();
      if (c == NTG * NOG - 1) late();
      const u32x4* cb = reinterpret_cast<const u32x4*>(lds + (cnt & 1) * kBufF4);
#pragma unroll
      for (int tt = 0; tt < TCH; ++tt)
#pragma unroll
        for (int o = 0; o < OCH; ++o) {
          u32x4 a[NP];
#pragma unroll
          for (int q = 0; q < NP; ++q) a[q] = cb[((tt * OCH + o) * NP + q) * WAVE + lane];
          f32x4 r = acc[og * OCH + o];
          if constexpr (NP == 3) {
            r = mfma_bf16(a[2], bp[tt][0], r);
            r = mfma_bf16(a[1], bp[tt][1], r);
            r = mfma_bf16(a[0], bp[tt][2], r);
            r = mfma_bf16(a[1], bp[tt][0], r);
            r = mfma_bf16(a[0], bp[tt][1], r);
          }
          r = mfma_bf16(a[0], bp[tt][0], r);
          acc[og * OCH + o] = r;
        }
      ++cnt;
    }
  }
}

template <int OT>
GNOT_DEV void init_bias(f32x4 (&acc)[OT], const float* __restrict__ bias, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    if (bias) {
      const float4 b = *reinterpret_cast<const float4*>(bias + 16 * o + 4 * g);
      acc[o] = f32x4{b.x, b.y, b.z, b.w};
    } else {
      acc[o] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

template <int OT>
GNOT_DEV void acc_to_regs(const f32x4 (&acc)[OT], float (&h)[OT][4]) {
#pragma unroll
  for (int o = 0; o < OT; ++o) {
    h[o][0] = acc[o][0]; h[o][1] = acc[o][1]; h[o][2] = acc[o][2]; h[o][3] = acc[o][3];
  }
}

// Feature softmax over heads of `dh` consecutive features (model.py:59, 72, 93) applied to the
// point-form tile set h[OT][4] (features 16T + 4g + r).  Supported: dh = 4, 8 or a multiple of 16.
template <int OT>
GNOT_DEV void softmax_heads(float (&h)[OT][4], int dh, int g) {
  if (dh == 4) {
#pragma unroll
    for (int T = 0; T < OT; ++T) {
      float m = fmaxf(fmaxf(h[T][0], h[T][1]), fmaxf(h[T][2], h[T][3]));
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) { h[T][r] = __expf(h[T][r] - m); s += h[T][r]; }
      const float inv = 1.0f / s;
#pragma unroll
      for (int r = 0; r < 4; ++r) h[T][r] *= inv;
    }
  } else if (dh == 8) {
#pragma unroll
    for (int T = 0; T < OT; ++T) {
      float m = fmaxf(fmaxf(h[T][0], h[T][1]), fmaxf(h[T][2], h[T][3]));
      m = fmaxf(m, shfl_xor(m, 16));
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) { h[T][r] = __expf(h[T][r] - m); s += h[T][r]; }
      s += shfl_xor(s, 16);
      const float inv = 1.0f / s;
#pragma unroll
      for (int r = 0; r < 4; ++r) h[T][r] *= inv;
    }
  } else if ((dh & 15) != 0) {
    // any other dh (a multiple of 4): the 4 features of tile T in lane group g, 16T + 4g .. +3, lie in
    // ONE head, (16T + 4g) / dh (the chunk starts at a head boundary, linear.hip linear_oc).  Per head:
    // this lane's max / sum over its groups in the head, then a butterfly over the 4 lane groups of the
    // point (a lane with no feature of the head contributes -inf / 0)
    int hT[OT];
#pragma unroll
    for (int T = 0; T < OT; ++T) hT[T] = (16 * T + 4 * g) / dh;
    const int nh = 16 * OT / dh;
    for (int hd = 0; hd < nh; ++hd) {
      float m = -INFINITY;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (hT[T] == hd) m = fmaxf(m, fmaxf(fmaxf(h[T][0], h[T][1]), fmaxf(h[T][2], h[T][3])));
      m = fmaxf(m, shfl_xor(m, 16));
      m = fmaxf(m, shfl_xor(m, 32));
      float s = 0.f;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (hT[T] == hd) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { h[T][r] = __expf(h[T][r] - m); s += h[T][r]; }
        }
      s += shfl_xor(s, 16);
      s += shfl_xor(s, 32);
      const float inv = 1.0f / s;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (hT[T] == hd) {
#pragma unroll
          for (int r = 0; r < 4; ++r) h[T][r] *= inv;
        }
    }
  } else {
    const int tph = dh >> 4;  // tiles per head
    for (int T0 = 0; T0 < OT; T0 += tph) {
      float m = -INFINITY;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (T >= T0 && T < T0 + tph)
          m = fmaxf(m, fmaxf(fmaxf(h[T][0], h[T][1]), fmaxf(h[T][2], h[T][3])));
      m = fmaxf(m, shfl_xor(m, 16));
      m = fmaxf(m, shfl_xor(m, 32));
      float s = 0.f;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (T >= T0 && T < T0 + tph) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { h[T][r] = __expf(h[T][r] - m); s += h[T][r]; }
        }
      s += shfl_xor(s, 16);
      s += shfl_xor(s, 32);
      const float inv = 1.0f / s;
#pragma unroll
      for (int T = 0; T < OT; ++T)
        if (T >= T0 && T < T0 + tph) {
#pragma unroll
          for (int r = 0; r < 4; ++r) h[T][r] *= inv;
        }
    }
  }
}

}  // namespace gnot
