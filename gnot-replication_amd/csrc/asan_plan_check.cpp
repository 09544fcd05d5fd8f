// Host-side planning check, built with AddressSanitizer on the HOST code only (csrc/Makefile `asan`):
// exercises every C-ABI entry point that needs no GPU -- plan creation for the supported widths, packed
// batch geometries (ragged, empty samples, many meshes, padded-equal strides), MoE recompute and
// precision switches, workspace sizing, gradient offsets, the point-shard exchange tables and the
// error paths -- so heap overflows / use-after-free in engine.cpp's table building show up on the CPU.
// Run by tests/test_asan.py; exit status 0 = every check passed and ASan reported nothing.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "gnot_hip.h"

static int g_fail = 0;
#define CHECK(cond)                                                                      \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond,   \
                   gnot_last_error());                                                   \
      ++g_fail;                                                                          \
    }                                                                                    \
  } while (0)

static int fake_allreduce(void*, float*, int64_t, void*) { return 0; }
static int fake_alltoallv(void*, const float*, const int64_t*, float*, const int64_t*, void*) { return 0; }

static std::vector<int64_t> offsets(const std::vector<int64_t>& n) {
  std::vector<int64_t> o(1, 0);
  for (int64_t v : n) o.push_back(o.back() + v);
  return o;
}

// one plan: several batch geometries, both precisions and recompute settings, sharded geometries
static void exercise(const gnot_config& cfg, std::mt19937& rng) {
  gnot_plan* p = nullptr;
  CHECK(gnot_plan_create(&cfg, &p) == GNOT_OK);
  if (!p) return;
  const int nlin = gnot_plan_num_linears(p);
  CHECK(nlin > 0);
  std::vector<int32_t> dims(2 * nlin);
  CHECK(gnot_plan_linear_dims(p, dims.data()) == GNOT_OK);
  const int I = cfg.n_input_functions;
  for (int trial = 0; trial < 12; ++trial) {
    const int B = 1 + (int)(rng() % (trial < 6 ? 4 : 64));
    std::vector<int64_t> n(B), m(B);
    for (int b = 0; b < B; ++b) {
      n[b] = (trial == 2 && b == 0) ? 0 : 1 + (int64_t)(rng() % 3000);   // an empty sample once
      m[b] = 1 + (int64_t)(rng() % 900);
    }
    if (trial == 1) for (int b = 0; b < B; ++b) n[b] = n[0] ? n[0] : 1;  // padded-equal strides
    const auto xo = offsets(n);
    std::vector<int64_t> fo;
    for (int i = 0; i < I; ++i) {
      const auto o = offsets(m);
      fo.insert(fo.end(), o.begin(), o.end());
    }
    for (int rc = 0; rc < 2; ++rc)
      for (int bf = 0; bf < 2; ++bf) {
        CHECK(gnot_plan_set_moe_recompute(p, rc) == GNOT_OK);
        CHECK(gnot_plan_set_precision(p, bf) == GNOT_OK);
        for (int tr = 0; tr < 2; ++tr) {
          const int st = gnot_plan_set_batch(p, B, xo.data(), I ? fo.data() : nullptr, tr);
          if (xo.back() == 0) {
            CHECK(st == GNOT_E_INVALID);
            continue;
          }
          CHECK(st == GNOT_OK);
          CHECK(gnot_plan_workspace_bytes(p) > 0);
          std::vector<int64_t> go(2 * nlin);
          CHECK(gnot_plan_grad_offsets(p, go.data()) == GNOT_OK);
          int64_t expect = 0;
          for (int k = 0; k < nlin; ++k) {
            CHECK(go[2 * k] == expect);
            expect += (int64_t)dims[2 * k] * dims[2 * k + 1];
            CHECK(go[2 * k + 1] == expect);
            expect += dims[2 * k];
          }
        }
      }
    // point sharding: every rank's local geometry of the same global batch
    const int world = 2 + (int)(rng() % 7);
    gnot_comm comm{nullptr, fake_allreduce, fake_alltoallv};
    for (int r = 0; r < world; ++r) {
      CHECK(gnot_plan_set_shard(p, r, world, B, n.data(), &comm) == GNOT_OK);
      std::vector<int64_t> loc(B);
      for (int b = 0; b < B; ++b) {
        int64_t lo, hi;
        CHECK(gnot_shard_range(n[b], r, world, &lo, &hi) == GNOT_OK);
        loc[b] = hi - lo;
      }
      const auto lo = offsets(loc);
      const int st = gnot_plan_set_batch(p, B, lo.data(), I ? fo.data() : nullptr, 1);
      CHECK(st == GNOT_OK || lo.back() == 0);
      // a geometry that does not match the declared shard is refused
      if (lo.back() > 0) {
        auto bad = lo;
        bad.back() += 1;
        CHECK(gnot_plan_set_batch(p, B, bad.data(), I ? fo.data() : nullptr, 1) == GNOT_E_INVALID);
      }
    }
    CHECK(gnot_plan_set_shard(p, 0, 1, B, n.data(), nullptr) == GNOT_OK);
  }
  gnot_plan_destroy(p);
}

// the scramble exchange tables: what rank r sends to t is what t receives from r, and the segments
// cover the local buffers exactly
static void exchange(std::mt19937& rng) {
  for (int trial = 0; trial < 40; ++trial) {
    const int B = 1 + (int)(rng() % 5), world = 1 + (int)(rng() % 8);
    const int H = 1 + (int)(rng() % 8), dh = 4 * (1 + (int)(rng() % 8));
    std::vector<int64_t> n(B);
    for (int b = 0; b < B; ++b) n[b] = (int64_t)(rng() % 5000);
    std::vector<std::vector<int64_t>> sc(world, std::vector<int64_t>(world)), rc = sc;
    for (int r = 0; r < world; ++r) {
      int64_t nseg = 0;
      CHECK(gnot_shard_exchange(B, n.data(), H, dh, r, world, sc[r].data(), rc[r].data(), nullptr, 0, &nseg) ==
            GNOT_OK);
      std::vector<int64_t> segs(4 * (nseg + 1));
      int64_t nseg2 = 0;
      CHECK(gnot_shard_exchange(B, n.data(), H, dh, r, world, nullptr, nullptr, segs.data(), nseg, &nseg2) ==
            GNOT_OK);
      CHECK(nseg2 == nseg);
      int64_t local = 0, sent = 0, recvd = 0, tot_s = 0, tot_r = 0;
      for (int b = 0; b < B; ++b) {
        int64_t lo, hi;
        gnot_shard_range(n[b], r, world, &lo, &hi);
        local += (hi - lo) * H * dh;
      }
      for (int64_t k = 0; k < nseg; ++k) {
        CHECK(segs[4 * k + 3] >= 0);
        (segs[4 * k] == 0 ? sent : recvd) += segs[4 * k + 3];
      }
      for (int t = 0; t < world; ++t) {
        tot_s += sc[r][t];
        tot_r += rc[r][t];
      }
      CHECK(sent == tot_s && recvd == tot_r);
      CHECK(tot_s == local && tot_r == local);
    }
    for (int r = 0; r < world; ++r)
      for (int t = 0; t < world; ++t) CHECK(sc[r][t] == rc[t][r]);
  }
  // argument errors
  int64_t lo, hi, nseg;
  CHECK(gnot_shard_range(10, 2, 2, &lo, &hi) == GNOT_E_INVALID);
  CHECK(gnot_shard_exchange(0, nullptr, 8, 32, 0, 1, nullptr, nullptr, nullptr, 0, &nseg) == GNOT_E_INVALID);
}

int main() {
  std::mt19937 rng(12345);
  const int widths[] = {16, 32, 48, 64, 96, 128, 144, 192, 256};
  for (int d : widths)
    for (int I = 0; I <= 2; ++I) {
      gnot_config c{};
      c.input_dim = 2 + (d & 1);
      c.theta_dim = 1;
      c.input_func_dim = 3;
      c.out_dim = 1 + I;
      c.n_attn_layers = 1 + (d % 3);
      c.n_attn_hidden_dim = c.n_mlp_hidden_dim = c.n_input_hidden_dim = d;
      c.n_mlp_num_layers = 2 + (d % 3);
      c.n_expert = d == 32 ? 2 : d == 48 ? 3 : d == 256 ? 8 : 4;
      c.n_head = d == 48 || d == 144 ? 3 : d >= 64 ? 8 : 4;   // 96 / 192: head width 12 / 24
      c.n_input_functions = I;
      exercise(c, rng);
    }
  // bad configurations are refused without leaking
  gnot_config bad{};
  bad.input_dim = 2; bad.theta_dim = 1; bad.input_func_dim = 3; bad.out_dim = 1; bad.n_attn_layers = 1;
  bad.n_attn_hidden_dim = 32; bad.n_mlp_num_layers = 2; bad.n_mlp_hidden_dim = 64; bad.n_input_hidden_dim = 32;
  bad.n_expert = 2; bad.n_head = 4;
  gnot_plan* p = nullptr;
  CHECK(gnot_plan_create(&bad, &p) == GNOT_E_INVALID);
  exchange(rng);
  std::printf("asan_plan_check: %s (%d failed checks)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
