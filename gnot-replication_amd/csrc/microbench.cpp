// Kernel microbenchmark (diagnostics, not part of libgnot_hip.so): times the internal launchers on
// synthetic cfg2-sized operands with hipEvents, one kernel class at a time, no contention.
//   make microbench && ./microbench [points] [D] [experts]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "gnot_kernels.h"

using namespace gnot;
#ifdef GNOT_DIAG_STAMP
namespace gnot {
hipError_t set_chain2_diag(int v);
}
#endif

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

static float* dalloc(size_t n, float scale) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((float)((i * 2654435761u) % 2001) / 1000.0f - 1.0f);
  float* d = nullptr;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

template <typename F>
static double time_us(F&& f, int reps = 50) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
  CK(hipEventRecord(a, nullptr));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, nullptr));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

#ifdef GNOT_DIAG_STAMP
// diagnostic build (make microbench EXTRA=-DGNOT_DIAG_STAMP): one extra launch with ChainArgs::dbg set;
// per wave the shader-clock ticks spent in the chunk waits + barriers (sync) and between them (body)
static void stamp_report(const char* name, ChainArgs a, bool bwd) {
  static unsigned long long* dbg = nullptr;
  const size_t n = (size_t)65536 * 8 * 3;
  if (!dbg) CK(hipMalloc(&dbg, n * sizeof(unsigned long long)));
  CK(hipMemset(dbg, 0, n * sizeof(unsigned long long)));
  a.dbg = dbg;
  CK(bwd ? launch_chain_bwd(a, nullptr) : launch_chain_fwd(a, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(n);
  CK(hipMemcpy(h.data(), dbg, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double body = 0, sync = 0, cnt = 0, waves = 0;
  for (size_t i = 0; i < n; i += 3)
    if (h[i + 2]) { body += (double)h[i]; sync += (double)h[i + 1]; cnt += (double)h[i + 2]; waves += 1; }
  std::printf("stamp %-28s waves %8.0f  syncs/wave %6.1f  sync share %5.3f  ticks/sync %7.1f  body ticks/interval %8.1f\n",
              name, waves, cnt / std::max(waves, 1.0), sync / std::max(body + sync, 1.0), sync / std::max(cnt, 1.0),
              body / std::max(cnt - waves, 1.0));
}
#define STAMP(name, args, bwd) stamp_report(name, args, bwd)
#else
#define STAMP(name, args, bwd) (void)0
#endif

int main(int argc, char** argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 10000;
  const int D = argc > 2 ? std::atoi(argv[2]) : 128;
  const int E = argc > 3 ? std::atoi(argv[3]) : 4, NL = 5, DT = D / 16;
  // packed weight images: NL layers x E chains, fwd and transposed (values arbitrary, finite)
  const size_t img4 = (size_t)DT * ((DT + 1) / 2) * 3 * 64;   // float4 per DxD image (bf16x6 >= fp32)
  float4* W = reinterpret_cast<float4*>(dalloc(img4 * 4 * NL * E * 2, 0.05f));
  float* bias = dalloc((size_t)NL * E * D, 0.01f);
  std::vector<ChainLayer> layers;
  for (int e = 0; e < E; ++e)
    for (int j = 0; j < NL; ++j) {
      const size_t k = (size_t)e * NL + j;
      layers.push_back(ChainLayer{W + 2 * k * img4, W + (2 * k + 1) * img4, bias + k * D});
    }
  ChainLayer* dlayers = nullptr;
  CK(hipMalloc(&dlayers, layers.size() * sizeof(ChainLayer)));
  CK(hipMemcpy(dlayers, layers.data(), layers.size() * sizeof(ChainLayer), hipMemcpyHostToDevice));
  float* X = dalloc((size_t)P * D, 1.0f);
  float* Y = dalloc((size_t)E * P * D, 0.0f);
  float* save = dalloc((size_t)E * NL * P * D, 1.0f);
  float* dz = dalloc((size_t)E * NL * P * D, 0.0f);
  float* scores = dalloc((size_t)P * 16, 0.25f);
  float* dscore = dalloc((size_t)P * 16, 0.0f);
  float* dX = dalloc((size_t)E * P * D, 0.0f);

  ChainArgs a{};
  a.D = D; a.KT0 = DT; a.OTL = DT; a.nlin = NL; a.in_dim = D; a.out_dim = D; a.P = P; a.nchains = E;
  a.layers = dlayers; a.X = X; a.ldx = D; a.Y = Y; a.ldy = D; a.y_chain_stride = (long)P * D;
  a.scores = scores; a.ldsc = 16; a.mode = CH_MOE;
  a.save = save; a.save_layer_stride = (long)P * D; a.save_chain_stride = (long)NL * P * D;
  const double fl = 2.0 * E * P * NL * (double)D * D;
  double t = time_us([&] { CK(launch_moe_combine(X, Y, (long)P * D, E, dX, (long)P * D, nullptr)); });
  std::printf("moe_combine E=%d P=%d D=%d: %8.2f us  %6.0f GB/s\n", E, P, D, t, (E + 2.0) * P * D * 4 / t / 1e3);
  t = time_us([&] { CK(launch_chain_fwd(a, nullptr)); });
  std::printf("chain_fwd  MoE E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
  STAMP("chain_fwd MoE x6", a, false);
  {  // the same chains without the training saves (inference form)
    ChainArgs an = a;
    an.save = nullptr;
    t = time_us([&] { CK(launch_chain_fwd(an, nullptr)); });
    std::printf("chain_fwd  MoE no-save E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
  }
  ChainArgs bw = a;
  bw.dY = X; bw.lddy = D; bw.dscore = dscore; bw.dz = dz; bw.dz_layer_stride = (long)P * D;
  bw.dz_chain_stride = (long)NL * P * D; bw.dX = dX; bw.lddx = D; bw.dx_chain_stride = (long)P * D;
  t = time_us([&] { CK(launch_chain_bwd(bw, nullptr)); });
  std::printf("chain_bwd  MoE E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
  STAMP("chain_bwd MoE x6", bw, true);
  if (D == 256) {   // bf16 arithmetic mode (one operand piece)
    ChainArgs a1 = a, b1 = bw;
    a1.np = 1; b1.np = 1;
    t = time_us([&] { CK(launch_chain_fwd(a1, nullptr)); });
    std::printf("chain_fwd  bf16 E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
    t = time_us([&] { CK(launch_chain_bwd(b1, nullptr)); });
    std::printf("chain_bwd  bf16 E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
    // bf16 storage (ChainArgs::b16s, the bf16-mode soft-MoE chains): bf16 saves / inputs / dZ rows
    ChainArgs a2 = a1, b2 = b1;
    a2.b16s = 1; a2.save_layer_stride = (long)P * D / 2; a2.save_chain_stride = (long)NL * P * D;
    b2.b16s = 1; b2.save_layer_stride = a2.save_layer_stride; b2.save_chain_stride = a2.save_chain_stride;
    b2.dz_layer_stride = (long)P * D / 2; b2.dz_chain_stride = (long)NL * P * D / 2;
    // the saves-only forward (MoE recompute's first pass)
    a2.Y = nullptr;
    t = time_us([&] { CK(launch_chain_fwd(a2, nullptr)); });
    std::printf("chain_fwd  b16s saves-only E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
    a2.Y = Y;
    // the bf16 mode's default soft-MoE form: bf16 stage rows for the moe_combine_b16 pass
    ChainArgs a3 = a2, b3 = b2;
    a3.stage_b16 = 1; a3.y_chain_stride = (long)P * D / 2;
    b3.stage_b16 = 1; b3.dx_chain_stride = (long)P * D / 2;
#ifdef GNOT_DIAG_STAMP
    // priced parts (set_chain2_diag bits: 1 no GELU, 2 stores dropped, 4 no weight DMA); wrong results
    for (int dg : {0, 1, 2, 4, 3, 6, 7}) {
      CK(set_chain2_diag(dg));
      t = time_us([&] { CK(launch_chain_fwd(a3, nullptr)); });
      const double tf = t;
      t = time_us([&] { CK(launch_chain_bwd(b3, nullptr)); });
      std::printf("diag %d  b16s stage   fwd %8.2f us  bwd %8.2f us\n", dg, tf, t);
      t = time_us([&] { CK(launch_chain_fwd(a, nullptr)); });
      const double tx = t;
      t = time_us([&] { CK(launch_chain_bwd(bw, nullptr)); });
      std::printf("diag %d  fp32 (x6)    fwd %8.2f us  bwd %8.2f us\n", dg, tx, t);
    }
    CK(set_chain2_diag(0));
#else
    t = time_us([&] { CK(launch_chain_fwd(a3, nullptr)); });
    std::printf("chain_fwd  b16s stage E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
    t = time_us([&] { CK(launch_chain_bwd(b3, nullptr)); });
    std::printf("chain_bwd  b16s stage E=%d P=%d D=%d: %8.2f us  %6.1f TFLOP/s\n", E, P, D, t, fl / t / 1e6);
#endif
  }

  if (argc > 4 && std::atoi(argv[4]) == 1) return 0;   // chains only
  for (int NO : {D, 3 * D}) {
    LinearArgs l{};
    l.nseg = 1; l.X[0] = X; l.Wp[0] = W; l.ldx = D; l.nsum = 1; l.K = D; l.bias = bias; l.Y = Y; l.ldy = NO;
    l.NO = NO; l.P = P; l.epi = EPI_STORE; l.nsoft = 0; l.dh = 16;
    t = time_us([&] { CK(D == 256 ? launch_linear2(l, nullptr) : launch_linear(l, D, nullptr)); });
    std::printf("linear     P=%d K=%d NO=%d: %8.2f us  %6.1f TFLOP/s\n", P, D, NO, t, 2.0 * P * D * NO / t / 1e6);
    if (D == 256) {
      l.np = 1;
      t = time_us([&] { CK(launch_linear2(l, nullptr)); });
      std::printf("linear     P=%d K=%d NO=%d bf16: %8.2f us  %6.1f TFLOP/s\n", P, D, NO, t, 2.0 * P * D * NO / t / 1e6);
      l.np = 3;
    }
    if (D == 256 && NO == D) {
      l.epi = EPI_ACCUM;
      t = time_us([&] { CK(launch_linear2(l, nullptr)); });
      std::printf("linear     P=%d K=%d NO=%d accum: %8.2f us  %6.1f TFLOP/s\n", P, D, NO, t, 2.0 * P * D * NO / t / 1e6);
      l.nseg = 3; l.X[1] = X; l.X[2] = X; l.Wp[1] = W; l.Wp[2] = W; l.bias = nullptr;
      t = time_us([&] { CK(launch_linear2(l, nullptr)); });
      std::printf("linear     P=%d K=3x%d NO=%d accum: %8.2f us  %6.1f TFLOP/s\n", P, D, NO, t, 6.0 * P * D * NO / t / 1e6);
    }
  }
  {  // finite dZ for the weight-gradient runs (the chain_bwd above wrote arbitrary values)
    float* fresh = dalloc((size_t)E * NL * P * D, 0.5f);
    CK(hipMemcpy(dz, fresh, (size_t)E * NL * P * D * 4, hipMemcpyDeviceToDevice));
    CK(hipFree(fresh));
    fresh = dalloc((size_t)E * NL * P * D, 2.0f);
    CK(hipMemcpy(save, fresh, (size_t)E * NL * P * D * 4, hipMemcpyDeviceToDevice));
    CK(hipFree(fresh));
  }
  // weight-gradient point-reduction GEMM of one MoE chain group: E*NL jobs of D x D over P points,
  // split-K exactly as the engine sizes it (<= 512 workgroups, >= 128 points per split)
  {
    std::vector<WgradJob> jobs;
    std::vector<int> wg_pre, red_pre;
    int wg = 0, red = 0;
    long slab_off = 0;
    float* dW = dalloc((size_t)E * NL * (D * D + D), 0.f);
    const int njobs = E * NL;
    const int tiles = ((D + 127) / 128) * ((D + 127) / 128);
    const long want = std::max<long>(1, 512 / ((long)njobs * tiles));
    for (int k = 0; k < njobs; ++k) {
      WgradJob J{};
      J.dz = dz + (size_t)k * P * D; J.lddz = D; J.x = save + (size_t)k * P * D; J.ldx = D; J.x_gelu = 1;
      J.out = D; J.in = D; J.dW = dW + (size_t)k * (D * D + D); J.db = J.dW + D * D; J.P = P;
      J.tiles_o = (D + 127) / 128; J.tiles_i = J.tiles_o;
      J.splits = (int)std::min<long>(std::min<long>(want, std::max<long>(1, P / 128)), 256);
      J.slab_off = slab_off;
      slab_off += (long)J.splits * tiles * 128 * 129;
      wg_pre.push_back(wg); wg += tiles * J.splits;
      red_pre.push_back(red); red += tiles * 128 * 129;
      jobs.push_back(J);
    }
    WgradJob* djobs = nullptr;
    int* dpre = nullptr;
    CK(hipMalloc(&djobs, jobs.size() * sizeof(WgradJob)));
    CK(hipMemcpy(djobs, jobs.data(), jobs.size() * sizeof(WgradJob), hipMemcpyHostToDevice));
    std::vector<int> pre(wg_pre);
    pre.insert(pre.end(), red_pre.begin(), red_pre.end());
    CK(hipMalloc(&dpre, pre.size() * sizeof(int)));
    CK(hipMemcpy(dpre, pre.data(), pre.size() * sizeof(int), hipMemcpyHostToDevice));
    float* slab = dalloc((size_t)slab_off, 0.f);
    t = time_us([&] { CK(launch_wgrad(djobs, dpre, njobs, wg, dpre + njobs, red, slab, nullptr)); }, 20);
    std::printf("wgrad MoE  %d jobs P=%d D=%d (%d WGs): %8.2f us  %6.1f TFLOP/s\n", njobs, P, D, wg, t, fl / t / 1e6);
    const size_t ndw = (size_t)E * NL * (D * D + D);
    std::vector<float> ref(ndw), got(ndw);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), dW, ndw * 4, hipMemcpyDeviceToHost));
    t = time_us([&] { CK(launch_wgrad(djobs, dpre, njobs, wg, dpre + njobs, red, slab, nullptr, true)); }, 20);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), dW, ndw * 4, hipMemcpyDeviceToHost));
    double num = 0, den = 0;
    for (size_t i = 0; i < ndw; ++i) { num += (got[i] - ref[i]) * (double)(got[i] - ref[i]); den += (double)ref[i] * ref[i]; }
    std::printf("wgrad MoE  bf16x6:                     %8.2f us  %6.1f TFLOP/s  (rel-L2 vs fp32 %.2e)\n", t, fl / t / 1e6,
                std::sqrt(num / (den + 1e-30)));
    if (D == 256) {   // the 256 x 256-tile kernel: one workgroup per (job, split)
      for (int wgs : {256, 512}) {
        std::vector<WgradJob> wj(jobs);
        std::vector<int> wpre;
        long soff = 0;
        const int splits = std::max(1, wgs / njobs);
        for (int k = 0; k < njobs; ++k) {
          wj[k].splits = splits;
          wj[k].slab_off = soff;
          soff += (long)splits * tiles * 128 * 129;
          wpre.push_back(k * splits);
        }
        wpre.insert(wpre.end(), red_pre.begin(), red_pre.end());
        WgradJob* dwj = nullptr;
        int* dwpre = nullptr;
        float* wslab = nullptr;
        CK(hipMalloc(&dwj, wj.size() * sizeof(WgradJob)));
        CK(hipMemcpy(dwj, wj.data(), wj.size() * sizeof(WgradJob), hipMemcpyHostToDevice));
        CK(hipMalloc(&dwpre, wpre.size() * sizeof(int)));
        CK(hipMemcpy(dwpre, wpre.data(), wpre.size() * sizeof(int), hipMemcpyHostToDevice));
        CK(hipMalloc(&wslab, soff * sizeof(float)));
        t = time_us([&] { CK(launch_wgrad(dwj, dwpre, njobs, njobs * splits, dwpre + njobs, red, wslab, nullptr, true, true)); }, 20);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), dW, ndw * 4, hipMemcpyDeviceToHost));
        double n2 = 0, d2 = 0;
        for (size_t i = 0; i < ndw; ++i) { n2 += (got[i] - ref[i]) * (double)(got[i] - ref[i]); d2 += (double)ref[i] * ref[i]; }
        std::printf("wgrad MoE  bf16x6 wide 256x256 (%d WGs):  %8.2f us  %6.1f TFLOP/s  (rel-L2 vs fp32 %.2e)\n",
                    njobs * splits, t, fl / t / 1e6, std::sqrt(n2 / (d2 + 1e-30)));
        t = time_us([&] { CK(launch_wgrad(dwj, dwpre, njobs, njobs * splits, dwpre + njobs, red, wslab, nullptr, true, true, 1)); }, 20);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), dW, ndw * 4, hipMemcpyDeviceToHost));
        n2 = 0; d2 = 0;
        for (size_t i = 0; i < ndw; ++i) { n2 += (got[i] - ref[i]) * (double)(got[i] - ref[i]); d2 += (double)ref[i] * ref[i]; }
        std::printf("wgrad MoE  bf16 wide 256x256 (%d WGs):    %8.2f us  %6.1f TFLOP/s  (rel-L2 vs fp32 %.2e)\n",
                    njobs * splits, t, fl / t / 1e6, std::sqrt(n2 / (d2 + 1e-30)));
        if (wgs == 512) {
          // diagnostics of the wide x6 kernel: without the GELU of the B operand, with every point
          // reading row 0 (L2-resident rows: no HBM latency), and both
          const char* what[3] = {"no-GELU operand", "L2-resident rows", "no-GELU + L2 rows"};
          for (int v = 0; v < 3; ++v) {
            std::vector<WgradJob> dj(wj);
            for (auto& J : dj) {
              if (v != 1) J.x_gelu = 0;
              if (v != 0) { J.lddz = 0; J.ldx = 0; }
            }
            CK(hipMemcpy(dwj, dj.data(), dj.size() * sizeof(WgradJob), hipMemcpyHostToDevice));
            t = time_us([&] { CK(launch_wgrad(dwj, dwpre, njobs, njobs * splits, dwpre + njobs, red, wslab, nullptr, true, true)); }, 20);
            std::printf("wgrad MoE  bf16x6 wide, %-18s   %8.2f us  %6.1f TFLOP/s\n", what[v], t, fl / t / 1e6);
          }
        }
        CK(hipFree(dwj));
        CK(hipFree(dwpre));
        CK(hipFree(wslab));
      }
    }
    {
      std::vector<WgradJob> ng(jobs);
      for (auto& J : ng) J.x_gelu = 0;
      WgradJob* dng = nullptr;
      CK(hipMalloc(&dng, ng.size() * sizeof(WgradJob)));
      CK(hipMemcpy(dng, ng.data(), ng.size() * sizeof(WgradJob), hipMemcpyHostToDevice));
      t = time_us([&] { CK(launch_wgrad(dng, dpre, njobs, wg, dpre + njobs, red, slab, nullptr)); }, 20);
      std::printf("wgrad MoE  no-GELU operand:            %8.2f us  %6.1f TFLOP/s\n", t, fl / t / 1e6);
      for (auto& J : ng) { J.x_gelu = 1; J.lddz = 0; J.ldx = 0; }   // every point reads row 0: no HBM traffic
      CK(hipMemcpy(dng, ng.data(), ng.size() * sizeof(WgradJob), hipMemcpyHostToDevice));
      t = time_us([&] { CK(launch_wgrad(dng, dpre, njobs, wg, dpre + njobs, red, slab, nullptr)); }, 20);
      std::printf("wgrad MoE  L2-resident rows (diag):    %8.2f us  %6.1f TFLOP/s\n", t, fl / t / 1e6);
    }

    // attention apply pass (H = 8 heads of D/8), alone and under a concurrent MoE wgrad stream
    const int H = 8, dh = D / H;
    std::vector<int4> ch;
    for (int s0 = 0; s0 < P; s0 += 64) ch.push_back(make_int4(0, s0, std::min(64, P - s0), 0));
    int4* dch = nullptr;
    CK(hipMalloc(&dch, ch.size() * sizeof(int4)));
    CK(hipMemcpy(dch, ch.data(), ch.size() * sizeof(int4), hipMemcpyHostToDevice));
    long* doff = nullptr;
    const long hoff[2] = {0, P};
    CK(hipMalloc(&doff, sizeof(hoff)));
    CK(hipMemcpy(doff, hoff, sizeof(hoff), hipMemcpyHostToDevice));
    float* st = dalloc((size_t)2 * H * (dh * dh + dh), 0.1f);
    float* q = dalloc((size_t)P * 3 * D, 0.05f);
    float* dres = dalloc((size_t)P * D, 0.3f);
    float* du = dalloc((size_t)2 * P * D, 0.f);
    float* dden = dalloc((size_t)2 * P * H, 0.f);
    float* dq = dalloc((size_t)P * 3 * D, 0.f);
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int nsrc : {1, 2}) {
      AttnApplyArgs ap{};
      ap.q = q; ap.ldq = nsrc == 1 ? 3 * D : D; ap.nsrc = nsrc; ap.chunks = dch; ap.nchunks = (int)ch.size();
      ap.off = doff; ap.H = H; ap.dh = dh; ap.res = Y; ap.dres = dres; ap.dq_pre = dq; ap.lddq = ap.ldq; ap.lddu = D;
      for (int i = 0; i < nsrc; ++i) {
        ap.state[i] = st + (size_t)i * H * (dh * dh + dh);
        ap.du[i] = du + (size_t)i * P * D;
        ap.dden[i] = dden + (size_t)i * P * H;
      }
      // algorithmic HBM bytes: fwd reads q, writes res; bwd reads q, dres, writes du (per source), dq, dden
      const double bf = 2.0 * P * D * 4, bb = (3.0 + nsrc) * P * D * 4 + 4.0 * nsrc * P * H;
      t = time_us([&] { CK(launch_attn_apply_fwd(ap, nullptr)); });
      std::printf("apply_fwd  nsrc=%d P=%d H=%d dh=%d: %8.2f us  %6.0f GB/s\n", nsrc, P, H, dh, t, bf / t / 1e3);
      t = time_us([&] { CK(launch_attn_apply_bwd(ap, nullptr)); });
      std::printf("apply_bwd  nsrc=%d P=%d H=%d dh=%d: %8.2f us  %6.0f GB/s\n", nsrc, P, H, dh, t, bb / t / 1e3);
      if (nsrc == 1) {   // K/V backward of the self attention (k, v = the 2nd/3rd thirds of the qkv rows)
        AttnKVBwdArgs kb{};
        kb.k = q + D; kb.v = q + 2 * D; kb.ldkv = 3 * D; kb.dstate = st; kb.chunks = dch; kb.nchunks = (int)ch.size();
        kb.H = H; kb.dh = dh; kb.dk = dq + D; kb.dv = dq + 2 * D; kb.lddkv = 3 * D;
        t = time_us([&] { CK(launch_attn_kv_bwd(kb, nullptr)); });
        std::printf("kv_bwd     P=%d H=%d dh=%d: %8.2f us  %6.0f GB/s\n", P, H, dh, t, 4.0 * P * D * 4 / t / 1e3);
      }
      // contention: wgrad launches queued on s2 while apply_bwd is timed on the null stream
      for (int i = 0; i < 30; ++i) CK(launch_wgrad(djobs, dpre, njobs, wg, dpre + njobs, red, slab, s2));
      t = time_us([&] { CK(launch_attn_apply_bwd(ap, nullptr)); }, 20);
      std::printf("apply_bwd  nsrc=%d under concurrent wgrad: %8.2f us\n", nsrc, t);
      CK(hipStreamSynchronize(s2));
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
