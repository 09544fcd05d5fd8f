// Weight packing: nn.Linear weights -> MFMA A-operand fragment-order images.
//
// Every Linear of the model (reference model.py:9-14, 43-51) is re-laid out once per step (after
// the optimizer touched the parameters) into two images:
//   forward  A = W   : lane l of tile (o, T) holds W[16o + (l&15)][16T + 4(l>>4) + 0..3]
//   backward A = W^T : lane l of tile (o, T) holds W[16T + 4(l>>4) + 0..3][16o + (l&15)]
// so that a kernel's A-operand read is one contiguous 1 KiB wave-instruction (16 B per lane).
// Out-of-range rows/columns are written as zeros, which is what lets the chain/linear kernels run
// every layer on whole 16-wide tiles (odd in/out widths such as input_dim+theta_dim = 3 or
// n_expert = 3 cost nothing but padding).
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

// W row of image row / contraction index i (padded heads: PackJob::hr / hp), or -1 for a zero row
GNOT_DEV int pack_row(const PackJob& J, int i) {
  if (i >= J.out) return -1;
  if (J.hp == 0) return i;
  const int h = i / J.hp, j = i - h * J.hp;
  return j < J.hr ? h * J.hr + j : -1;
}

// one wave per (job, tile)
__global__ void __launch_bounds__(64) pack_kernel(const PackJob* __restrict__ jobs,
                                                  const int* __restrict__ prefix, int njobs) {
  const int tile_id = blockIdx.x;
  // binary search: last job with prefix[j] <= tile_id
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= tile_id) lo = mid; else hi = mid - 1;
  }
  const PackJob& J = jobs[lo];
  const int t = tile_id - prefix[lo];
  const int lane = threadIdx.x;
  const int r16 = lane & 15, g = lane >> 4;
  if (J.x6) {
    // bf16x6 image block (o, kb): lane holds row 16o + r16 at k-slots 8g + j of k-block kb; blocks are
    // k-major (x6 = 1: chain.hip, a k-block of every output tile together) or output-major (x6 = 2:
    // chain2.hip / linear2.hip / linear.hip, an output tile's k-blocks together); x6 = 3 / 4: output-major /
    // k-major with ONE RNE bf16 piece (the bf16 arithmetic mode)
    const int KB = (J.KTp + 1) / 2;
    const int o = t / KB, kb = t % KB;
    unsigned w[3][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 32 * kb + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));   // contraction index
      const int row = 16 * o + r16;
      float v = 0.f;
      if (!J.transposed) {
        const int wr = pack_row(J, row);
        v = (wr >= 0 && f < J.in) ? J.W[(long)wr * J.in + f] : 0.f;
      } else {
        const int wr = pack_row(J, f);
        v = (wr >= 0 && row < J.in) ? J.W[(long)wr * J.in + row] : 0.f;
      }
      const unsigned b = __builtin_bit_cast(unsigned, v);
      const float r1 = v - __builtin_bit_cast(float, b & 0xFFFF0000u);
      const unsigned b1 = __builtin_bit_cast(unsigned, r1);
      const float r2 = r1 - __builtin_bit_cast(float, b1 & 0xFFFF0000u);
      w[0][j] = b;
      w[1][j] = b1;
      w[2][j] = __builtin_bit_cast(unsigned, r2);
    }
    uint4* dst = reinterpret_cast<uint4*>(J.dst);
    const bool omaj = J.x6 == 2 || J.x6 == 3;
    const long blk = omaj ? (long)(J.o0 + o) * ((J.ktot + 1) / 2) + J.t0 / 2 + kb    // output-major
                          : (long)(J.t0 / 2 + kb) * J.otot + J.o0 + o;               // k-major
    if (J.x6 >= 3) {
      // bf16 arithmetic mode: one round-to-nearest-even piece (w[0] holds the fp32 bits)
      uint4 u;
      u.x = (bf16_rne_bits(u2f(w[0][1])) << 16) | bf16_rne_bits(u2f(w[0][0]));
      u.y = (bf16_rne_bits(u2f(w[0][3])) << 16) | bf16_rne_bits(u2f(w[0][2]));
      u.z = (bf16_rne_bits(u2f(w[0][5])) << 16) | bf16_rne_bits(u2f(w[0][4]));
      u.w = (bf16_rne_bits(u2f(w[0][7])) << 16) | bf16_rne_bits(u2f(w[0][6]));
      dst[blk * WAVE + lane] = u;
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        uint4 u;
        u.x = (w[q][1] & 0xFFFF0000u) | (w[q][0] >> 16);
        u.y = (w[q][3] & 0xFFFF0000u) | (w[q][2] >> 16);
        u.z = (w[q][5] & 0xFFFF0000u) | (w[q][4] >> 16);
        u.w = (w[q][7] & 0xFFFF0000u) | (w[q][6] >> 16);
        dst[blk * 3 * WAVE + q * WAVE + lane] = u;
      }
    }
    if (J.bias_dst && t == 0) {
      const int nb = 16 * J.OTp;
      for (int i = lane; i < nb; i += WAVE) {
        const int br = pack_row(J, i);
        J.bias_dst[i] = (br >= 0 && J.b) ? J.b[br] : 0.f;
      }
    }
    return;
  }
  float v[4];
  int o, T;
  if (!J.transposed) {
    o = t / J.KTp; T = t % J.KTp;
    const int wr = pack_row(J, 16 * o + r16);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = 16 * T + 4 * g + r;
      v[r] = (wr >= 0 && col < J.in) ? J.W[(long)wr * J.in + col] : 0.f;
    }
  } else {                              // contraction runs over W's rows
    o = t / J.KTp; T = t % J.KTp;
    const int col = 16 * o + r16;       // W column (input feature)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int wr = pack_row(J, 16 * T + 4 * g + r);
      v[r] = (wr >= 0 && col < J.in) ? J.W[(long)wr * J.in + col] : 0.f;
    }
  }
  const int Ta = J.t0 + T;
  const long di = J.kh > 0 ? ((long)(Ta / J.kh) * J.otot + J.o0 + o) * J.kh + Ta % J.kh
                           : (long)(J.o0 + o) * J.ktot + Ta;
  J.dst[di * WAVE + lane] = make_float4(v[0], v[1], v[2], v[3]);
  // padded bias copy, done by the job's first tile
  if (J.bias_dst && t == 0) {
    const int nb = 16 * J.OTp;
    for (int i = lane; i < nb; i += WAVE) {
      const int br = pack_row(J, i);
      J.bias_dst[i] = (br >= 0 && J.b) ? J.b[br] : 0.f;
    }
  }
}

hipError_t launch_pack(const PackJob* jobs_dev, const int* tile_prefix_dev, int njobs,
                       int total_tiles, hipStream_t s) {
  if (total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_kernel, dim3(total_tiles), dim3(64), 0, s, jobs_dev, tile_prefix_dev, njobs);
  return hipGetLastError();
}

}  // namespace gnot
