// Fused MLP chains for hidden width d >= 128 (reference MLP, model.py:5-18): forward and backward on
// bf16x6 MFMA, OUTPUT-MAJOR.
//
// Same point form as chain.hip (a wave carries 16 points through all nl+1 Linears with the
// activations in registers; grid.y = chain, e.g. the E experts of a soft-MoE), but the layer is
// computed one 16-feature OUTPUT tile at a time instead of one input block at a time:
//   * the layer input is held as its exact three-piece bf16 split (gnot_common.h split8_x6), 12
//     registers per 32-feature k-block, so every output tile is 6 x KB v_mfma_f32_16x16x32_bf16 with
//     nothing but the weight pieces read from LDS;
//   * a tile's result is final as soon as its MFMAs retire: bias, save store, GELU (forward) or
//     GELU'(saved pre-activation) and the dZ store (backward) of tile o run beside the MFMAs of tile
//     o+1, instead of a whole-layer VALU burst between two MFMA phases;
//   * the next layer's input accumulates as fp32 (4 registers per tile) and is split once per layer.
// 8 waves (128 points) share one weight stream: one LDS chunk = one output tile's image (KB k-blocks
// x 3 pieces x 1 KiB, output-major pack, pack.hip x6 = 2), double-buffered, the next chunk's DMA
// (next tile, or the next layer's first tile) issued one chunk ahead.  <= 256 registers: two waves per
// SIMD, so one wave's epilogue VALU runs beside its partner's MFMAs.
//   forward : h_l = W_l a_l + b_l, a_{l+1} = gelu(h_l); saves h_l (training); epilogue of the last
//             layer: CH_STORE / CH_SOFTMAX (gating) / CH_MOE (score-scaled expert output)
//   backward: dz_{nl-1} = dy (x score for CH_MOE), g_l = W_l^T dz_l, dz_{l-1} = g_l * gelu'(h_{l-1});
//             writes every dz_l (weight gradients, wgrad.hip) and optionally dX = W_0^T dz_0.
#include "gnot_kernels.h"
#include "x6_core.h"

namespace gnot {

// backward: weight chunks in flight ahead of the one being consumed (1 .. kC2Ring - 1), per arithmetic.
// In-step (r03x): bf16x6 lead 1 / 2 / 3 = 232.2 / 235.0 / 234.7 ms per configs[2] step (the concurrent
// weight gradients take the slack); the one-piece bf16 chains lead 3 (a tile's MFMA work is far shorter
// than a chunk's L2 -> LDS latency)
// Round 4 (no concurrent weight gradients, microbench r04ld, one box): bf16x6 lead 2 / 3 = 8.39 / 8.42 ms
// against 8.26-8.29 for lead 1, with the wait + barrier share of the tile unchanged at 0.30 (stamp build):
// the wait is the barrier's skew between the 8 waves, not the chunk's latency
template <int NP>
constexpr int c2b_lead() { return NP == 3 ? 1 : 3; }
// output tiles per weight chunk of the backward: two in the bf16-storage chains (one counted wait and
// barrier per pair; the ring buffers of the one-piece chains already hold two tiles, C2Lds::WB)
template <int NP, bool B16>
constexpr int c2b_ch() { return (B16 && NP == 1) ? 2 : 1; }
// bf16-storage backward: saved-row tile pairs requested this many pairs ahead (r03r: 6 vs 1 neutral)
constexpr int kC2bPairsAhead = 6;

// diagnostic builds only (make microbench EXTRA=-DGNOT_DIAG_STAMP): runtime switches that make the chains
// compute WRONG results, to price one part of their work -- bit 1: no GELU (identity), bit 2: every save /
// dZ / stage store dropped by a zero-size buffer resource (still issued and counted), bit 4: no weight-chunk
// DMA after the prologue
#ifdef GNOT_DIAG_STAMP
__constant__ int c2_diag;
hipError_t set_chain2_diag(int v) { return hipMemcpyToSymbol(HIP_SYMBOL(c2_diag), &v, sizeof(int)); }
#define C2D(bit) (c2_diag & (bit))
#else
#define C2D(bit) 0
#endif


// LDS of one workgroup (u32x4 units): two weight-chunk buffers, two 1 KiB bias buffers (layer parity,
// forward) and per wave four 1 KiB slots of saved pre-activation tiles (backward).
// forward pair mode: two output tiles per weight chunk, one barrier per pair.  Measured (`r02bf`):
// bf16 mode chain forward 348 -> 388 TFLOP/s; bf16x6 unchanged (202), so only the one-piece mode
template <int NP>
constexpr bool c2f_pair() { return NP == 1; }

template <int D, int NP>
struct C2Lds {
  // one weight chunk: one output tile of a D x D image (two in the forward's pair mode)
  static constexpr int WB = c2_tile_u4(D / 32, NP) * (c2f_pair<NP>() ? 2 : 1);
  static constexpr int kBias = kC2Ring * WB;            // offset of the bias buffers
  static constexpr int kHs = kBias + 2 * 64;            // offset of the saved-row slots
  // saved-row slots per wave: 4 (bf16x6), 8 at one piece (the bf16-storage backward keeps up to
  // kC2bPairsAhead + 1 tile pairs in flight; a power of two dividing the 8 pairs of a layer)
  static constexpr int kSlots = NP == 1 ? 8 : 4;
  static constexpr int kBytes = (kHs + kC2Waves * kSlots * 64) * 16;
};


// ------------------------------------------------------------------------------------------ expert grid
// Workgroup -> (128-point block, expert).  Workgroups are dealt round-robin over the 8 XCDs (w and w + 8
// share one, MI355X_MICROARCH.md "Workgroup dispatch"); speed only, nothing depends on placement.
//   mode 1 "grouped" (E > 1): w = 8 (E (b / 8) + e) + b % 8 -- the E experts of a block run at the same
//          time on ONE XCD and read the block's input rows (forward: the MoE input; backward: dquery, the
//          scores) once from HBM into its L2; every XCD streams all E experts' weights;
//   mode 0: blockIdx.x = block, blockIdx.y = chain (single chains).
// Measured at configs[2] (262,144 points, E = 8, d = 256; profiles/r04_chain_grid.txt): grouped against
// mode 0, bf16x6 forward 6.76 / 6.81 ms, backward 8.27 / 9.02; bf16 storage 4.01 / 4.31 and 3.84 / 4.12.
// Fewer experts per XCD (each XCD's L2 holding fewer experts' weights) measured within +-2 % (round 5,
// profiles/r05u_chain_xcd_experts_sweep.log) and is gone.
GNOT_DEV void c2_grid_pos(int E, int mode, int& blk, int& e) {
  if (mode == 0 || gridDim.y > 1) {
    blk = (int)blockIdx.x;
    e = (int)blockIdx.y;
    return;
  }
  const int w = (int)blockIdx.x, x = w & 7, s = w >> 3;
  e = s % E;
  blk = (s / E) * 8 + x;
}
static int c2_grid_mode(int E) { return E <= 1 ? 0 : 1; }
// 1-D grid of the grouped deal (the ids past the last block exit at once)
inline unsigned c2_grid_size(int nblocks, int E) { return 8u * (unsigned)E * (unsigned)((nblocks + 7) / 8); }

// in place: each value rounded to bf16 (RNE, the bits store_rows_b16_sc1 writes)
template <int KT>
GNOT_DEV void round_rows_bf16(float (&a)[KT][4]) {
#pragma unroll
  for (int T = 0; T < KT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) a[T][r] = bf16_lo(pk_bf16(a[T][r], 0.f));
}

// ------------------------------------------------------------------------------------------ forward
// One forward layer: OT output tiles h = W a + b of the split input `in`; saves h (SAVE) and returns
// gelu(h) (GELU) or h.  Entry: this layer's tile-0 weights sit in pp.cur() and its bias in bias buffer
// `bsel`, DMA'd before exactly `pend0` later vector-memory ops of this wave.  Per tile o: counted wait
// + barrier, DMA of tile o+1 (or of the next layer's bias then tile 0), the 6 x KB MFMAs, then the
// epilogue of tile o-1 (its save store is the ONLY vector-memory op after the DMA, so the next wait is
// vmcnt(1)).
// B16: the save is the RNE bf16 tile at its pair-interleaved position (voff = the lane's row * 512 B)
template <int OT, int KBI, bool GELU, bool SAVE, int NP, bool B16 = false>
GNOT_DEV void c2f_layer(C2Pipe& pp, const u32x4* W, const u32x4 (&in)[KBI][NP], int bsel, rsrc_t rs, int voff,
                        const u32x4* nextW, int next_n16, const float* next_bias, int next_bias_bytes, int pend0,
                        int g, float (&out)[OT][4]) {
  constexpr int TU = c2_tile_u4(KBI, NP);
  const u32x4* bias = pp.lds + C2Lds<256, NP>::kBias + bsel * 64;
  f32x4 prev;
  // B16 saves in pair mode: the two 8-byte halves of a 16-byte pair-interleaved chunk (tiles 2t, 2t+1) go out
  // as ONE store once the odd tile's epilogue is done (the even tile's half waits in `held`): half the store
  // instructions of 8-byte tile stores (MI355X_MICROARCH.md: narrow stores are issue-bound)
  constexpr bool COMB = B16 && SAVE && c2f_pair<NP>();
  u32x2 held;
  auto save_tile = [&](int o, const f32x4& acc) {
    if constexpr (COMB) {
      const u32x2 w = u32x2{pk_bf16(acc[0], acc[1]), pk_bf16(acc[2], acc[3])};
      if ((o & 1) == 0) held = w;
      else buf_store_b128(u32x4{held[0], held[1], w[0], w[1]}, rs, voff + ((o >> 1) * 4 + g) * 16);
    } else if constexpr (B16) {
      const float v[4] = {acc[0], acc[1], acc[2], acc[3]};
      store_tile_b16(v, rs, voff, o, g);
    } else {
      buf_store_f32x4(make_float4(acc[0], acc[1], acc[2], acc[3]), rs, voff + 64 * o);
    }
  };
  // B16 GELU layers save gelu'(h) instead of h (bf16 mode: the backward then multiplies instead of
  // evaluating gelu', and the weight gradients read the stored Linear inputs, not h), from the same tail
  // evaluation as gelu(h); stored after the tile's last value
  constexpr bool SGRAD = B16 && GELU;
  float gd[4];
  auto epi = [&](int o, const f32x4& acc) {
    if (SAVE && !SGRAD) save_tile(o, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (C2D(1)) { out[o][r] = acc[r]; gd[r] = acc[r]; }
      else if constexpr (SGRAD) out[o][r] = gelu_and_grad(acc[r], gd[r]);
      else out[o][r] = GELU ? gelu(acc[r]) : acc[r];
    }
    pin4(out[o]);
    if (SAVE && SGRAD) save_tile(o, f32x4{gd[0], gd[1], gd[2], gd[3]});
  };
  // one part of tile o's epilogue (inside the next tile's MFMA stream): part 0 the save store (SGRAD:
  // part 3)
  auto epi_part = [&](int o, const f32x4& acc, int r) {
    if (SAVE && !SGRAD && r == 0) save_tile(o, acc);
    if (C2D(1)) {
      out[o][r] = acc[r]; gd[r] = acc[r];
      asm volatile("" : "+v"(out[o][r]), "+v"(gd[r]));
      if (SAVE && SGRAD && r == 3) save_tile(o, f32x4{gd[0], gd[1], gd[2], gd[3]});
    } else if constexpr (SGRAD) {
      out[o][r] = gelu_and_grad(acc[r], gd[r]);
      asm volatile("" : "+v"(out[o][r]), "+v"(gd[r]));
      if (SAVE && r == 3) save_tile(o, f32x4{gd[0], gd[1], gd[2], gd[3]});
    } else {
      out[o][r] = GELU ? gelu(acc[r]) : acc[r];
      asm volatile("" : "+v"(out[o][r]));
    }
  };
  if constexpr (c2f_pair<NP>()) {
  // pair mode: one chunk = tiles o, o+1; the wait at pair o retires the DMA issued at pair o-2, after
  // which this wave issued the save stores of the epilogues inside tiles o-2 (if o-2 > 0) and o-1
#pragma unroll
  for (int o = 0; o < OT; o += 2) {
#ifdef GNOT_DIAG_STAMP
    const unsigned long long t0 = pp.stamp_in();
#endif
    // stores issued after the DMA being retired (issued at pair o-2): the saves of tiles o-3 and o-2 (COMB: the
    // one combined store of tiles o-4, o-3)
    if (o == 0) c2_sync_n(pend0);
    else c2_sync_n(SAVE ? (COMB ? (o >= 4 ? 1 : 0) : (o >= 4 ? 2 : 1)) : 0);
#ifdef GNOT_DIAG_STAMP
    pp.stamp_out(t0);
#endif
    const u32x4* cb = pp.cur();
    u32x4* nb = pp.nxt();
    ++pp.cnt;
    auto issue = [&]() __attribute__((always_inline)) {
      if (C2D(4)) return;
      if (o + 3 < OT) {
        dma_image_n<2 * TU, kC2Waves>(nb, W + (size_t)(o + 2) * TU, pp.wave, pp.lane);
      } else if (o + 2 < OT) {
        dma_image_n<TU, kC2Waves>(nb, W + (size_t)(o + 2) * TU, pp.wave, pp.lane);
      } else if (nextW) {
        if (pp.wave == 0)
          dma16(make_rsrc(next_bias, (unsigned)next_bias_bytes), pp.lds + C2Lds<256, NP>::kBias + (bsel ^ 1) * 64,
                pp.lane * 16, 0);
        dma_image(nb, nextW, next_n16, kC2Waves, pp.wave, pp.lane);
      }
    };
    {
      const u32x4 bb = bias[4 * o + g];
      f32x4 acc;
      if (o > 0) {
        const f32x4 pv = prev;
        auto ep = [&](int r) { epi_part(o - 1, pv, r); };
        acc = c2_tile_epi<KBI, NP, true>(cb, in, __builtin_bit_cast(f32x4, bb), pp.lane, ep, issue);
      } else {
        issue();
        acc = c2_tile<KBI, false, NP>(cb, in, __builtin_bit_cast(f32x4, bb), pp.lane);
      }
      prev = acc;
    }
    if (o + 1 < OT) {
      const u32x4 bb = bias[4 * (o + 1) + g];
      const f32x4 pv = prev;
      auto ep = [&](int r) { epi_part(o, pv, r); };
      prev = c2_tile_epi<KBI, NP, true>(cb + TU, in, __builtin_bit_cast(f32x4, bb), pp.lane, ep);
    }
  }
  epi(OT - 1, prev);
  return;
  }
#pragma unroll
  for (int o = 0; o < OT; ++o) {
#ifdef GNOT_DIAG_STAMP
    const unsigned long long t0 = pp.stamp_in();
#endif
    if (o == 0) c2_sync_n(pend0);
    else c2_sync_n((SAVE && o >= 2) ? 1 : 0);
#ifdef GNOT_DIAG_STAMP
    pp.stamp_out(t0);
#endif
    const u32x4* cb = pp.cur();
    u32x4* nb = pp.nxt();
    ++pp.cnt;
    auto issue = [&]() __attribute__((always_inline)) {
      if (C2D(4)) return;
      if (o + 1 < OT) {
        dma_image_n<TU, kC2Waves>(nb, W + (size_t)(o + 1) * TU, pp.wave, pp.lane);
      } else if (nextW) {
        // the next layer's bias first: the next layer's first wait only counts ops after its weights
        if (pp.wave == 0)
          dma16(make_rsrc(next_bias, (unsigned)next_bias_bytes), pp.lds + C2Lds<256, NP>::kBias + (bsel ^ 1) * 64,
                pp.lane * 16, 0);
        dma_image(nb, nextW, next_n16, kC2Waves, pp.wave, pp.lane);
      }
    };
    const u32x4 bb = bias[4 * o + g];
    f32x4 acc;
    if (o > 0) {
      const f32x4 pv = prev;
      auto ep = [&](int r) { epi_part(o - 1, pv, r); };
      acc = c2_tile_epi<KBI, NP, true>(cb, in, __builtin_bit_cast(f32x4, bb), pp.lane, ep, issue);
    } else {
      issue();
      acc = c2_tile<KBI, false, NP>(cb, in, __builtin_bit_cast(f32x4, bb), pp.lane);
    }
    prev = acc;
  }
  epi(OT - 1, prev);
}

// B16 (bf16 mode, ChainArgs::b16s): bf16 pair-interleaved saves, plus each Linear's RNE bf16 input (the
// split the MFMAs consume, stored as it is made) for the weight gradients
template <int D, int KT0, int OTL, bool SAVE, int NP, bool B16 = false>
__global__ void __launch_bounds__(64 * kC2Waves, 2) chain2_fwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16, KB = DT / 2, KB0 = (KT0 + 1) / 2;
  using LD = C2Lds<D, NP>;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  int blk, eg;
  c2_grid_pos(a.nchains, a.grid_mode, blk, eg);
  if ((long)blk * kC2Waves * 16 >= a.P) return;       // past the last block (whole workgroup, before any barrier)
  const long p = ((long)blk * kC2Waves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int nl = a.nlin;
  // Every buffer resource of a layer starts at this workgroup's first row (64-bit base in SGPRs), so the
  // 32-bit offsets only span the workgroup's 128 rows: no bound on the point count of a launch.  Rows
  // past P read 0 / are dropped by the resource's bound (the workgroup's rows that exist).
  const long row0 = (long)blk * kC2Waves * 16;
  const int nrows = (int)min((long)kC2Waves * 16, (long)a.P - row0);
  const unsigned lay_bytes = (unsigned)nrows * (unsigned)(D * 4);   // this workgroup's rows of a [P, D] layer
  // byte offset of this lane's row within the workgroup's rows
  const int voff = (int)(((unsigned)wave * 16u + (unsigned)(lane & 15)) * (unsigned)(D * 4) + 16u * (unsigned)g);
  // B16: this lane's row in the bf16 layers (512 B per point)
  const int rowb = (int)(((unsigned)wave * 16u + (unsigned)(lane & 15)) * (unsigned)kB16Row);
  const unsigned lay_b16 = (unsigned)nrows * (unsigned)kB16Row;
  // float offset of the workgroup's first row in a layer (fp32: D floats per row; B16: 512 B = 128 floats)
  const long rbase = row0 * (B16 ? kB16Row / 4 : D);
  C2Pipe pp{c2lds, LD::WB, 0, wave, lane};
  constexpr int CH = c2f_pair<NP>() ? 2 : 1;         // output tiles per weight chunk
  // a layer's first wait: the saves the previous layer issued after its last weight DMA (its last
  // tile's stream + the final epilogue; pair mode: its last pair's two tiles + the final epilogue; B16 pair
  // mode: the combined stores of tiles 12-13 and 14-15)
  constexpr int pend_next = SAVE ? (CH == 2 ? (B16 ? 2 : 3) : 2) : 0;
  const int e = eg;
  const ChainLayer* L = a.layers + e * nl;
  float* save = SAVE ? a.save + e * a.save_chain_stride : nullptr;
  const u32x4* W0 = reinterpret_cast<const u32x4*>(L[0].Wp);
  if (wave == 0) dma16(make_rsrc(L[0].bias, 16 * DT * 4), c2lds + LD::kBias, lane * 16, 0);
  dma_image(c2lds, W0, CH * c2_tile_u4(KB0, NP), kC2Waves, wave, lane);
  auto wp = [&](int l) { return reinterpret_cast<const u32x4*>(L[l].Wp); };
  auto rs = [&](int l) {
    return make_rsrc(SAVE ? save + l * a.save_layer_stride + rbase : nullptr,
                     SAVE && !C2D(2) ? (B16 ? lay_b16 : lay_bytes) : 0u);
  };
  const int svoff = B16 ? rowb : voff;
  // B16: a Linear's bf16 input words (k-blocks 0 .. nkb-1) into save slot `slot`; returns the stores issued
  auto store_in = [&](const float* slot, const u32x4 (&w)[KB][NP], int nkb) __attribute__((always_inline)) {
    const rsrc_t r = make_rsrc(slot + rbase, C2D(2) ? 0u : lay_b16);
#pragma unroll
    for (int t = 0; t < KB; ++t)
      if (t < nkb) buf_store_b128(w[t][0], r, rowb + (t * 4 + g) * 16);
    return nkb;
  };

  float nx[DT][4];                                   // next layer input (fp32), then split
  u32x4 bp[KB][NP];
  int bsel = 0;
  {
    float x0[KT0][4];
    load_rows<KT0>(x0, a.X, a.ldx, p, valid, a.in_dim, lane);
    u32x4 b0[KB0][NP];
    c2_split<KT0, NP>(x0, b0);
    int pend0 = 0;
    if constexpr (B16 && SAVE) {
      // the shared MoE input (Linear 0's operand): chain 0 only
      if (e == 0) {
        if constexpr (KB0 == KB) pend0 = store_in(a.save + nl * a.save_layer_stride, b0, KB0);
      }
    }
    const int nb = nl - 1 == 1 ? 16 * OTL * 4 : 16 * DT * 4;
    c2f_layer<DT, KB0, true, SAVE, NP, B16>(pp, W0, b0, bsel, rs(0), svoff, wp(1),
                                            (nl - 1 == 1 ? (OTL < CH ? OTL : CH) : CH) * c2_tile_u4(KB, NP), L[1].bias,
                                            nb, pend0, g, nx);
    bsel ^= 1;
  }
  for (int l = 1; l < nl - 1; ++l) {
    c2_split<DT, NP>(nx, bp);
    const int pin = B16 && SAVE ? store_in(save + (nl + l) * a.save_layer_stride, bp, KB) : 0;
    const int nb = l + 1 == nl - 1 ? 16 * OTL * 4 : 16 * DT * 4;
    c2f_layer<DT, KB, true, SAVE, NP, B16>(pp, wp(l), bp, bsel, rs(l), svoff, wp(l + 1),
                                           (l + 1 == nl - 1 ? (OTL < CH ? OTL : CH) : CH) * c2_tile_u4(KB, NP),
                                           L[l + 1].bias, nb, pend_next + pin, g, nx);
    bsel ^= 1;
  }
  float y[OTL][4];
  c2_split<DT, NP>(nx, bp);
  const int pin_last = B16 && SAVE ? store_in(save + (2 * nl - 1) * a.save_layer_stride, bp, KB) : 0;
  // B16: the last Linear's output is not saved as such: slot nl-1 receives the bf16 score-scaled expert term
  // below (the stage row itself; the backward divides d score by the score)
  c2f_layer<OTL, KB, false, SAVE && !B16, NP, B16>(pp, wp(nl - 1), bp, bsel, rs(nl - 1), svoff, nullptr, 0, nullptr, 0,
                                                   pend_next + pin_last, g, y);
  if (a.mode == CH_SOFTMAX) {
    // softmax over the first out_dim outputs (features 16T + 4g + r); padded features excluded
    float m = -INFINITY;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 * T + 4 * g + r < a.out_dim) m = fmaxf(m, y[T][r]);
    m = fmaxf(m, shfl_xor(m, 16));
    m = fmaxf(m, shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool in = 16 * T + 4 * g + r < a.out_dim;
        y[T][r] = in ? __expf(y[T][r] - m) : 0.f;
        sum += y[T][r];
      }
    sum += shfl_xor(sum, 16);
    sum += shfl_xor(sum, 32);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[T][r] *= inv;
  } else if (a.mode == CH_MOE) {
    const float s = valid ? a.scores[p * a.ldsc + e] : 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[T][r] *= s;
    // B16: the stage term in bf16 (the bf16 stage rows the combine pass sums; the recompute and inference
    // forms round the same values, so every soft-MoE form is bitwise equal)
    if constexpr (B16) round_rows_bf16<OTL>(y);
  }
  if (OTL == 16 && B16 && SAVE && a.mode == CH_MOE) {
    // bf16 training forward: the score-scaled term goes to save slot nl-1 (the backward's d score operand);
    // the engine points Y at that same slot, so it is also the stage row of the combine pass
    store_rows_b16<OTL>(y, rs(nl - 1), rowb, lane);
  } else if (OTL == 16 && B16 && a.stage_b16 && a.Y != nullptr) {   // bf16 stage rows for moe_combine_b16
    store_rows_b16<OTL>(y, make_rsrc(a.Y + e * a.y_chain_stride + rbase, C2D(2) ? 0u : lay_b16), rowb, lane);
  } else if (a.Y != nullptr) {
    store_rows<OTL>(y, a.Y + e * a.y_chain_stride, a.ldy, p, valid, a.out_dim, lane);
  }
#ifdef GNOT_DIAG_STAMP
  if (a.dbg && lane == 0) {
    unsigned long long* d = a.dbg + ((size_t)(blockIdx.x + (size_t)blockIdx.y * gridDim.x) * kC2Waves + wave) * 3;
    d[0] = pp.ts_body; d[1] = pp.ts_sync; d[2] = pp.ts_n;
  }
#endif
}

// ------------------------------------------------------------------------------------------ backward
// One backward layer l: g = W_l^T dz_l (DT output tiles of the split input `in`), dz_{l-1} = g *
// gelu'(h_{l-1}) stored (rz) and kept in nx.  Weight chunks stream through the ring c2b_lead<NP>() tiles
// ahead (the last tiles request the next image's first chunks); each tile's wait retires its own chunk
// and leaves every younger op of the wave in flight (C2Pipe::issued / mark).  The saved pre-activation tiles
// h_{l-1} arrive by LDS-DMA two tiles ahead into this wave's slots (tile o in slot o % kSlots; the next
// layer's tiles 0 and 1 are requested by this layer's last two tiles).  Entry: the layer's first
// c2b_lead<NP>() chunks and its h tiles 0 and 1 requested.
// B16 (bf16 storage, voff = the lane's row * 512 B): h and dz are pair-interleaved bf16 rows; one 16-byte
// DMA brings the h of a tile PAIR (pair m into slot m % 4, requested at tile 2m - 2), dz stores are 8 B
template <int KBI, int NP, bool B16 = false>
GNOT_DEV void c2b_layer(C2Pipe& pp, const u32x4* Wt, const u32x4 (&in)[KBI][NP], rsrc_t rh, rsrc_t rz, rsrc_t rh_next,
                        bool has_next_h, int voff, const u32x4* nextW, int next_n16, int next_tiles,
                        float (&nx)[16][4]) {
  constexpr int DT = 16, TU = c2_tile_u4(KBI, NP), LEAD = c2b_lead<NP>(), CH = c2b_ch<NP, B16>(), NC = DT / CH;
  static_assert(LEAD >= 1 && LEAD < kC2Ring, "weight ring too small");
  static_assert(CH == 1 || (B16 && kC2bPairsAhead >= LEAD), "pair mode: a pair's saved rows must be requested no "
                                                             "later than the chunk whose wait retires them");
  constexpr int SL = C2Lds<256, NP>::kSlots;
  // B16: pairs requested PK pairs ahead (pair m of a layer in slot m % SL; the next layer's pairs
  // continue the numbering, SL divides the 8 pairs of a layer); fp32 saves: tiles two ahead
  constexpr int PK = B16 ? kC2bPairsAhead : 1;
  static_assert(!B16 || (PK >= 1 && PK + 2 <= SL), "slot ring too small for the prefetch distance");
  u32x4* slots = pp.lds + C2Lds<256, NP>::kHs + pp.wave * SL * 64;
  const int g = pp.lane >> 4;
  f32x4 prev;
  // one part of tile o's epilogue (inside the next tile's MFMA stream): part 0 waits for the saved
  // pre-activation tile
  f32x4 hc;
  u32x2 hb;
  auto epi_part = [&](int o, const f32x4& acc, int r) {
    // the saved tile was read at the top of this tile (lds_read16_issue); wait for it here
    float h;
    if constexpr (B16) {
      if (r == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(hb) :: "memory");
      h = (r & 1) ? bf16_hi(hb[r >> 1]) : bf16_lo(hb[r >> 1]);
    } else {
      if (r == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(hc) :: "memory");
      h = hc[r];
    }
    // B16: the forward stored gelu'(h_{l-1}) itself (c2f_layer SGRAD)
    nx[o][r] = acc[r] * ((B16 || C2D(1)) ? h : gelu_grad(h));
    asm volatile("" : "+v"(nx[o][r]));
  };
  // the saved tile of tile o's epilogue, read from its slot
  auto read_h = [&](int o) {
    if constexpr (B16) hb = lds_read8_issue(slots + ((o >> 1) % SL) * 64 + pp.lane, 8 * (o & 1));
    else hc = lds_read16_issue(slots + (o % SL) * 64 + pp.lane);
  };
  // tile o's dz store is issued at the top of tile o+2, after that tile's DMAs: a counted wait only
  // retires the ops issued before the DMA it waits for, so each store gets two tiles to drain
  // B16: one 16-byte store per tile PAIR (the pair-interleaved chunk of tiles o-1, o), at odd o
  auto stores = [&](int o) {
    if constexpr (B16) {
      if (o & 1) {
        buf_store_b128(u32x4{pk_bf16(nx[o - 1][0], nx[o - 1][1]), pk_bf16(nx[o - 1][2], nx[o - 1][3]),
                             pk_bf16(nx[o][0], nx[o][1]), pk_bf16(nx[o][2], nx[o][3])},
                       rz, voff + ((o >> 1) * 4 + g) * 16);
        ++pp.issued;
      }
    } else {
      buf_store_f32x4(make_float4(nx[o][0], nx[o][1], nx[o][2], nx[o][3]), rz, voff + 64 * o);
      ++pp.issued;
    }
  };
  // does tile t request saved rows (fp32: tile t + 2; B16: at even t, pair t / 2 + PK)?
  auto hdma = [&](int t) { return B16 ? ((t & 1) == 0 && (t / 2 + PK < DT / 2 || has_next_h))
                                      : (t + 2 < DT || has_next_h); };
#pragma unroll
  for (int o = 0; o < DT; ++o) {
    // this tile's chunk c (DMA'd LEAD chunks back): every op of this wave younger than it may stay in
    // flight.  Ring positions are static: every backward layer has 16 / CH chunks and starts at buffer 0
    // (the mark array must only ever be indexed by constants, or it goes to scratch memory).  Pair mode:
    // the wait and the weight DMA at the chunk's first tile only
    const int c = o / CH;
    const bool first = o % CH == 0;
    if (first) {
#ifdef GNOT_DIAG_STAMP
      const unsigned long long t0 = pp.stamp_in();
#endif
      c2_sync_n(pp.issued - pp.mark[c % kC2Ring]);
#ifdef GNOT_DIAG_STAMP
      pp.stamp_out(t0);
#endif
    }
    const u32x4* cb = pp.lds + (c % kC2Ring) * pp.WB + (o % CH) * TU;
    u32x4* nb = pp.lds + ((c + LEAD) % kC2Ring) * pp.WB;
    const int nmark = (c + LEAD) % kC2Ring;
    // the weight DMA of chunk o + LEAD (this layer's, or the next image's first tiles) in its loop form
    // (unrolled measured 149 -> 141 TFLOP/s), then this tile's h DMA and the dz store of tile o - 2
    // (h first: the counted wait of tile o + 1 retires only ops OLDER than chunk o + 1's weight DMA,
    // issued LEAD tiles back, and must retire the h of tile o requested then too)
    auto issue = [&]() __attribute__((always_inline)) {
      if (hdma(o)) ++pp.issued;
      if constexpr (B16) {
        const int m = o / 2 + PK;
        if ((o & 1) == 0) {
          if (m < DT / 2) dma16(rh, slots + (m % SL) * 64, voff + 16 * g, 64 * m);
          else if (has_next_h) dma16(rh_next, slots + (m % SL) * 64, voff + 16 * g, 64 * (m - DT / 2));
        }
      } else {
        if (o + 2 < DT) dma16(rh, slots + ((o + 2) % SL) * 64, voff, 64 * (o + 2));
        else if (has_next_h) dma16(rh_next, slots + ((o + 2) % SL) * 64, voff, 64 * (o + 2 - DT));
      }
      if (first) {
        const int t = c + LEAD;            // chunk to request
        if (C2D(4)) {
        } else if (t < NC) {
          dma_image(nb, Wt + (size_t)t * CH * TU, CH * TU, kC2Waves, pp.wave, pp.lane);
          pp.issued += dma_image_count(CH * TU, kC2Waves, pp.wave);
        } else if (nextW && (t - NC) * CH < next_tiles) {
          const int nt = min(CH, next_tiles - (t - NC) * CH);
          dma_image(nb, nextW + (size_t)(t - NC) * CH * next_n16, nt * next_n16, kC2Waves, pp.wave, pp.lane);
          pp.issued += dma_image_count(nt * next_n16, kC2Waves, pp.wave);
        }
        pp.mark[nmark] = pp.issued;
      }
      if (o >= 2) stores(o - 2);
    };
    f32x4 acc;
    if (o > 0) {
      // the saved h tile of the epilogue below, read now so its LDS latency hides behind the first
      // k-blocks' MFMAs (its DMA, three tiles back, was retired by the counted wait above)
      read_h(o - 1);
      const f32x4 pv = prev;
      auto ep = [&](int r) { epi_part(o - 1, pv, r); };
      // the DMA issue first, then the tile (issuing it after k-block 0's fragment reads, as the forward
      // does, measured 155.0 -> 152.3 TFLOP/s here, r02ax)
      issue();
      acc = c2_tile_epi<KBI, NP, true>(cb, in, f32x4{0.f, 0.f, 0.f, 0.f}, pp.lane, ep);
    } else {
      issue();
      acc = c2_tile<KBI, false, NP>(cb, in, f32x4{0.f, 0.f, 0.f, 0.f}, pp.lane);
    }
    prev = acc;
    __builtin_amdgcn_sched_barrier(0);      // no code motion across tiles (register pressure)
  }
  stores(DT - 2);
  read_h(DT - 1);
#pragma unroll
  for (int r = 0; r < 4; ++r) epi_part(DT - 1, prev, r);
  stores(DT - 1);
}

// B16 (bf16 mode, ChainArgs::b16s): saves and dz as bf16 pair-interleaved rows
template <int D, int KT0, int OTL, int NP, bool B16 = false>
__global__ void __launch_bounds__(64 * kC2Waves, 2) chain2_bwd_kernel(ChainArgs a) {
  constexpr int DT = D / 16, KB = DT / 2, KBL = (OTL + 1) / 2;
  using LD = C2Lds<D, NP>;
  extern __shared__ __attribute__((aligned(16))) u32x4 c2lds[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4;
  int blk, eg;
  c2_grid_pos(a.nchains, a.grid_mode, blk, eg);
  if ((long)blk * kC2Waves * 16 >= a.P) return;       // past the last block (whole workgroup, before any barrier)
  const long p = ((long)blk * kC2Waves + wave) * 16 + (lane & 15);
  const bool valid = p < a.P;
  const int nl = a.nlin;
  // buffer resources start at this workgroup's first row (chain2_fwd_kernel): 32-bit offsets span 128 rows
  const long row0 = (long)blk * kC2Waves * 16;
  const int nrows = (int)min((long)kC2Waves * 16, (long)a.P - row0);
  const unsigned lay_bytes = (unsigned)nrows * (unsigned)(D * 4);
  const int voff = (int)(((unsigned)wave * 16u + (unsigned)(lane & 15)) * (unsigned)(D * 4) + 16u * (unsigned)g);
  // B16: this lane's row in the bf16 layers (512 B per point)
  const int rowb = (int)(((unsigned)wave * 16u + (unsigned)(lane & 15)) * (unsigned)kB16Row);
  const unsigned lay_b16 = (unsigned)nrows * (unsigned)kB16Row;
  const long rbase = row0 * (B16 ? kB16Row / 4 : D);
  const int lvoff = B16 ? rowb : voff;               // what the layers address rows with
  C2Pipe pp{c2lds, LD::WB, 0, wave, lane};
  const int e = eg;
  const ChainLayer* L = a.layers + e * nl;
  const float* save = a.save + e * a.save_chain_stride;
  float* dz = a.dz + e * a.dz_chain_stride;
  auto wt = [&](int l) { return reinterpret_cast<const u32x4*>(L[l].WpT); };
  const unsigned lb = B16 ? lay_b16 : lay_bytes;
  auto rh = [&](int l) { return make_rsrc(save + l * a.save_layer_stride + rbase, lb); };   // h_l
  auto rz = [&](int l) { return make_rsrc(dz + l * a.dz_layer_stride + rbase, C2D(2) ? 0u : lb); };      // dz_l
  // prologue DMA: the last Linear's first c2b_lead<NP>() weight chunks (ring buffers 0 ..) and the first
  // two h_{nl-2} tiles (B16: pairs 0 .. kC2bPairsAhead - 1)
  // (h first: a chunk's counted wait retires only the ops older than its DMA)
  {
    u32x4* slots = c2lds + LD::kHs + wave * LD::kSlots * 64;
    const rsrc_t r = rh(nl - 2);
    if constexpr (B16) {
#pragma unroll
      for (int m = 0; m < kC2bPairsAhead; ++m) dma16(r, slots + m * 64, rowb + 16 * g, 64 * m);
      pp.issued += kC2bPairsAhead;
    } else {
      dma16(r, slots, voff, 0);
      dma16(r, slots + 64, voff, 64);
      pp.issued += 2;
    }
    constexpr int C1 = c2b_ch<NP, B16>() * c2_tile_u4(KBL, NP);   // the last Linear's chunk
#pragma unroll
    for (int t = 0; t < c2b_lead<NP>(); ++t) {
      dma_image(c2lds + t * LD::WB, wt(nl - 1) + (size_t)t * C1, C1, kC2Waves, wave, lane);
      pp.issued += dma_image_count(C1, kC2Waves, wave);
      pp.mark[t] = pp.issued;
    }
  }
  // ---- gradient at the chain output
  float dy[OTL][4];
  if (a.mode == CH_MOE) {
    // query_out = query_in + sum_e s_e * y_e : dy_e = s_e * dq ; ds_e = dq . y_e (model.py:128-131)
    float yv[OTL][4];
    load_rows<OTL>(dy, a.dY, a.lddy, p, valid, 16 * OTL, lane);
    if constexpr (B16) load_rows_b16<OTL>(yv, rh(nl - 1), rowb, lane);
    else load_rows<OTL>(yv, save + (nl - 1) * a.save_layer_stride, D, p, valid, 16 * OTL, lane);
    float ds = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) ds += dy[T][r] * yv[T][r];
    ds += shfl_xor(ds, 16);
    ds += shfl_xor(ds, 32);
    const float s = valid ? a.scores[p * a.ldsc + e] : 0.f;
    // B16: slot nl-1 holds bf16(s y) (the stage row, forward); d score = dq . y = (dq . s y) / s.  s = 0 (an
    // underflowed softmax weight) contributes nothing to the gating gradient either way (it is scaled by s)
    if constexpr (B16) ds = s != 0.f ? ds / s : 0.f;
    if (valid && g == 0) a.dscore[p * a.ldsc + e] += ds;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dy[T][r] *= s;
  } else if (a.mode == CH_SOFTMAX) {
    // d logits = s * (ds - <s, ds>)   (softmax over experts, model.py:156)
    float sv[OTL][4];
    load_rows<OTL>(sv, a.scores, a.ldsc, p, valid, a.out_dim, lane);
    load_rows<OTL>(dy, a.dscore, a.ldsc, p, valid, a.out_dim, lane);
    float dot = 0.f;
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dot += sv[T][r] * dy[T][r];
    dot += shfl_xor(dot, 16);
    dot += shfl_xor(dot, 32);
#pragma unroll
    for (int T = 0; T < OTL; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) dy[T][r] = sv[T][r] * (dy[T][r] - dot);
  } else {
    load_rows<OTL>(dy, a.dY, a.lddy, p, valid, a.out_dim, lane);
  }
  if constexpr (B16) store_rows_b16<OTL>(dy, rz(nl - 1), rowb, lane);
  else store_rows<OTL>(dy, dz + (nl - 1) * a.dz_layer_stride, D, p, valid, 16 * OTL, lane);

  float nx[DT][4];
  u32x4 bp[KB][NP];
  // next image after layer l's tiles: layer l-1's W^T, or the first Linear's (dX) when l - 1 == 0
  auto next_img = [&](int l) -> const u32x4* { return (l - 1 >= 1 || a.dX) ? wt(l - 1) : nullptr; };
  // output tiles of the next image (hidden Linear: DT; the first Linear's dX: KT0)
  auto next_tiles = [&](int l) { return l - 1 >= 1 ? DT : KT0; };
  {
    u32x4 bl[KBL][NP];
    c2_split<OTL, NP>(dy, bl);
    const int l = nl - 1;
    c2b_layer<KBL, NP, B16>(pp, wt(l), bl, rh(l - 1), rz(l - 1), rh(l >= 2 ? l - 2 : 0), l - 1 >= 1, lvoff,
                            next_img(l), c2_tile_u4(KB, NP), next_tiles(l), nx);
  }
  for (int l = nl - 2; l >= 1; --l) {
    c2_split<DT, NP>(nx, bp);
    c2b_layer<KB, NP, B16>(pp, wt(l), bp, rh(l - 1), rz(l - 1), rh(l >= 2 ? l - 2 : 0), l - 1 >= 1, lvoff,
                           next_img(l), c2_tile_u4(KB, NP), next_tiles(l), nx);
  }
  // ---- first Linear: dX = W_0^T dz_0 (KT0 output tiles); its first c2b_lead<NP>() chunks were requested
  // by the last layer above
  if (a.dX) {
    c2_split<DT, NP>(nx, bp);
    const u32x4* W0 = wt(0);
    constexpr int TU0 = c2_tile_u4(KB, NP);
    float dx[KT0][4];
#pragma unroll
    for (int o = 0; o < KT0; ++o) {
      constexpr int CH = c2b_ch<NP, B16>(), LEAD = c2b_lead<NP>();
      const int c = o / CH;
      if (o % CH == 0) {
        c2_sync_n(pp.issued - pp.mark[c % kC2Ring]);
        const int t = c + LEAD;
        if (t * CH < KT0) {
          const int nt = min(CH, KT0 - t * CH);
          dma_image(c2lds + (t % kC2Ring) * LD::WB, W0 + (size_t)t * CH * TU0, nt * TU0, kC2Waves, wave, lane);
          pp.issued += dma_image_count(nt * TU0, kC2Waves, wave);
        }
        pp.mark[t % kC2Ring] = pp.issued;
      }
      const u32x4* cb = c2lds + (c % kC2Ring) * LD::WB + (o % CH) * TU0;
      f32x4 acc = c2_tile<KB, false, NP>(cb, bp, f32x4{0.f, 0.f, 0.f, 0.f}, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) dx[o][r] = acc[r];
    }
    if (B16 && KT0 == 16 && a.stage_b16) {           // bf16 stage rows for the moe_combine_b16 pass
      store_rows_b16<KT0>(dx, make_rsrc(a.dX + e * a.dx_chain_stride + rbase, C2D(2) ? 0u : lay_b16), rowb, lane);
    } else {
      if constexpr (B16) round_rows_bf16<KT0>(dx);   // the bf16 stage value (see the forward)
      store_rows<KT0>(dx, a.dX + e * a.dx_chain_stride, a.lddx, p, valid, a.in_dim, lane);
    }
  }
#ifdef GNOT_DIAG_STAMP
  if (a.dbg && lane == 0) {
    unsigned long long* d = a.dbg + ((size_t)(blockIdx.x + (size_t)blockIdx.y * gridDim.x) * kC2Waves + wave) * 3;
    d[0] = pp.ts_body; d[1] = pp.ts_sync; d[2] = pp.ts_n;
  }
#endif
}

template <int D, int NP>
static hipError_t launch_chain2_d(const ChainArgs& a, bool bwd, hipStream_t s) {
  constexpr int DT = D / 16;
  const int nblocks = (a.P + 16 * kC2Waves - 1) / (16 * kC2Waves);
  const int mode = c2_grid_mode(a.nchains);
  const dim3 grid = mode ? dim3(c2_grid_size(nblocks, a.nchains)) : dim3(nblocks, a.nchains);
  ChainArgs b = a;
  b.grid_mode = mode;
  const dim3 block(64 * kC2Waves);
  if (a.stage_b16 && (!a.b16s ||
                      (bwd ? (!a.dX || a.dx_chain_stride % 4) : (a.y_chain_stride % 4))))
    return hipErrorInvalidValue;
  const size_t lds = C2Lds<D, NP>::kBytes;
#define GNOT_C2_ATTR(K)                                                                                  \
  do {                                                                                                   \
    static bool attr = false;                                                                            \
    if (!attr) {                                                                                         \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)lds);                                                               \
      attr = true;                                                                                       \
    }                                                                                                    \
  } while (0)
  if (a.b16s) {
    // bf16 storage: soft-MoE experts (d x d chains) in bf16 mode.  The expert terms are bf16 in every form
    // (the bf16 stage rows; the recompute and inference forms' rounding), so they give the same bits
    if constexpr (NP == 1) {
      if (a.mode != CH_MOE || a.KT0 != DT || a.OTL != DT) return hipErrorInvalidValue;
      if (bwd) {
        GNOT_C2_ATTR((chain2_bwd_kernel<D, DT, DT, 1, true>));
        hipLaunchKernelGGL((chain2_bwd_kernel<D, DT, DT, 1, true>), grid, block, lds, s, b);
      } else if (a.save) {
        GNOT_C2_ATTR((chain2_fwd_kernel<D, DT, DT, true, 1, true>));
        hipLaunchKernelGGL((chain2_fwd_kernel<D, DT, DT, true, 1, true>), grid, block, lds, s, b);
      } else {
        GNOT_C2_ATTR((chain2_fwd_kernel<D, DT, DT, false, 1, true>));
        hipLaunchKernelGGL((chain2_fwd_kernel<D, DT, DT, false, 1, true>), grid, block, lds, s, b);
      }
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
#define GNOT_C2_CASE(K0, OL)                                                                             \
  if (a.KT0 == K0 && a.OTL == OL) {                                                                      \
    if (bwd) {                                                                                           \
      GNOT_C2_ATTR((chain2_bwd_kernel<D, K0, OL, NP>));                                           \
      hipLaunchKernelGGL((chain2_bwd_kernel<D, K0, OL, NP>), grid, block, lds, s, b);             \
    } else if (a.save) {                                                                                 \
      GNOT_C2_ATTR((chain2_fwd_kernel<D, K0, OL, true, NP>));                                     \
      hipLaunchKernelGGL((chain2_fwd_kernel<D, K0, OL, true, NP>), grid, block, lds, s, b);       \
    } else {                                                                                             \
      GNOT_C2_ATTR((chain2_fwd_kernel<D, K0, OL, false, NP>));                                    \
      hipLaunchKernelGGL((chain2_fwd_kernel<D, K0, OL, false, NP>), grid, block, lds, s, b);      \
    }                                                                                                    \
    return hipGetLastError();                                                                            \
  }
  GNOT_C2_CASE(1, 1)
  GNOT_C2_CASE(1, DT)
  GNOT_C2_CASE(DT, 1)
  GNOT_C2_CASE(DT, DT)
#undef GNOT_C2_CASE
#undef GNOT_C2_ATTR
  return hipErrorInvalidValue;
}

// The soft-MoE experts run as an expert grid (one workgroup per (128-point block, expert)) writing an
// [E, P, d] stage that moe_combine sums.  Two other forms were measured slower and are gone: a "walk"
// form (one workgroup runs every expert of its block and sums in place: 236.2 vs 233.0 ms per fp32
// configs[2] step, 127 vs 112 ms in bf16 mode, round 3) and a fused combine (the last expert workgroup of
// a block sums the stage: 230.0-232.9 vs 229.9-230.4 ms fp32, 95.9 vs 92.6-93.3 ms bf16, round 5).
hipError_t launch_chain2(const ChainArgs& a, bool bwd, hipStream_t s) {
  if (a.P <= 0 || a.nchains <= 0) return hipSuccess;
  if (a.nlin < 2) return hipErrorInvalidValue;
  switch (a.D) {
    case 256: return a.np == 1 ? launch_chain2_d<256, 1>(a, bwd, s) : launch_chain2_d<256, 3>(a, bwd, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gnot
