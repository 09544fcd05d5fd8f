"""Hidden and head widths beyond the BASELINE configs: the reference accepts any n_embed divisible by
n_head (model.py:41).  This core takes every (d, n_head) with a head width up to 256 whose internal width
is at most 1024 (engine.cpp gnot_plan_create): the chain.hip / linear.hip kernels at any multiple of 16 up to
192 (whole 16-wide MFMA tiles; a d that is not a multiple of 16 runs padded with exact-zero pad columns),
chain2.hip / linear2.hip at 256 (heads of 16 / 32 / 64 / 128 / 256), and everything else at the next
multiple of 64 from 320 on the one-Linear-at-a-time chains (chainw.hip, linear.hip's whole-row projection
tilings), above 512 at the next multiple of 128 with every full-width contraction split in two halves.  The attention passes split a head into 4-aligned lane slices up to 64 and into 4-feature quads
over 16 lanes above; the projections' feature softmax reduces a head that straddles 16-feature tiles
across the 4 lane groups of a point (gnot_common.h softmax_heads); a head width that is not a multiple of
4 runs on heads padded to one.

Each case is checked against the float64 oracle (oracle/gnot_oracle.py, pinned to the reference's
fixtures) at north_star's 1e-4: output and every parameter gradient (golden_util.check_parity), on a
packed two-sample batch with input functions where the case has them.  The head widths other than
16 / 32 / 64 run the VALU attention forms only (no MFMA variant), so both the size-based choice and the
forced-MFMA setting (attn_path) reach the same kernels for them."""
import functools

import pytest

from golden_util import check_parity
from test_gpu_parity import _random_case, attn_path, build_model, run_packed  # noqa: F401

pytestmark = pytest.mark.gpu


def _cfg(d, H, E, I, L=1, nl=3, out=2):
    return dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=out, n_attn_layers=L, d=d,
                n_mlp_num_layers=nl, n_expert=E, n_head=H, n_input_functions=I)


CASES = {
    "d16_h4": _cfg(16, 4, 2, 1),          # dh 4, the narrowest hidden width
    "d80_h5": _cfg(80, 5, 2, 0, L=2),     # dh 16 with an odd tile count (5 tiles)
    "d96_h8": _cfg(96, 8, 3, 1),          # dh 12: heads straddle 16-feature tiles
    "d112_h4": _cfg(112, 4, 2, 2),        # dh 28, two input functions
    "d144_h3": _cfg(144, 3, 2, 1),        # dh 48 above d = 128
    "d144_h4": _cfg(144, 4, 2, 1),        # dh 36: only the whole 9-tile row keeps a head in one projection workgroup
    "d176_h4": _cfg(176, 4, 2, 0),        # dh 44: 11 tiles, self-attention (fused q|k|v softmax) only
    "d160_h8": _cfg(160, 8, 2, 1),        # dh 20
    "d192_h8": _cfg(192, 8, 2, 0),        # dh 24, self-attention only
    "d192_h6": _cfg(192, 6, 2, 1, nl=4),  # dh 32 (fp32-MFMA attention forms at d = 192)
    "d192_h12": _cfg(192, 12, 2, 1),      # dh 16, 12 heads: 3 per wave has no MFMA state form (VALU state)
    # widths that are not a multiple of 16 run padded to the next one (engine.cpp gnot_plan_create: zero pad
    # columns, the feature softmax's pad columns zeroed, the scramble rows at the real width)
    "d36_h3": _cfg(36, 3, 2, 1),          # dh 12, kernels at d = 48
    "d100_h5": _cfg(100, 5, 3, 2, L=2),   # dh 20, kernels at d = 112, two input functions, two blocks
    "d60_h15": _cfg(60, 15, 2, 0),        # dh 4, kernels at d = 64, self-attention (fused q|k|v) only
    "d208_h13": _cfg(208, 13, 2, 1),      # dh 16, the d = 256 kernels (chain2 / linear2 / wide wgrad) padded
    "d224_h7": _cfg(224, 7, 3, 0),        # dh 32, d = 256 kernels, self-attention only
    # head widths that are not a multiple of 4 run on heads padded to one (engine.cpp gnot_plan::head_padded:
    # q / k / v rows at h * dh', the feature softmax masked to the real features, the scramble at the real
    # head width, per-head weight-gradient jobs)
    "d100_h4": _cfg(100, 4, 2, 1),        # dh 25 -> 28, kernels at d = 112, batched input-function K/V
    "d90_h6": _cfg(90, 6, 2, 0, L=2),     # dh 15 -> 16, kernels at d = 96, fused q|k|v in both attentions
    "d30_h2": _cfg(30, 2, 2, 2),          # dh 15 -> 16, kernels at d = 32, two input functions
    "d21_h7": _cfg(21, 7, 2, 0),          # dh 3 -> 4, kernels at d = 32
    "d150_h6": _cfg(150, 6, 2, 1),        # dh 25 -> 28: H dh' = 168 > 160, kernels at d = 176
    # d > 256: the chains one Linear at a time (chainw.hip) on the fp32-MFMA projection kernel
    "d320_h10": _cfg(320, 10, 2, 1),      # dh 32
    "d288_h18": _cfg(288, 18, 3, 0, nl=2),  # dh 16, padded to 320, self-attention only
    "d512_h16": _cfg(512, 16, 2, 1),      # dh 32, the widest
    # heads of 64 above 256: d * dh = 20,480 / 32,768 (round 5 refused d * dh > 16,384: the VALU state kernel
    # now loops over any number of its 4 x 4 blocks per thread); H = 8 also runs the MFMA state kernel
    "d320_h5": _cfg(320, 5, 2, 1),
    "d512_h8": _cfg(512, 8, 2, 1),
    # heads wider than 64 (round 6): attn.hip's wide forms (16 lanes per head, 4-feature quads round-robin,
    # the q / k row read through the L1), linear2.hip's 128- and 256-feature softmax heads at d = 256
    "d128_h1": _cfg(128, 1, 2, 1),        # dh 128: one head (two 64-feature blocks)
    "d256_h2": _cfg(256, 2, 2, 1),        # dh 128 on the d = 256 kernels
    "d256_h1": _cfg(256, 1, 3, 1, nl=2),  # dh 256 (four blocks; batched input-function K / V at oc 16)
    "d192_h2": _cfg(192, 2, 2, 0),        # dh 96: a half-filled second block, self-attention only
    "d136_h2": _cfg(136, 2, 2, 2),        # dh 68 (one quad in block 1), kernels at d = 144, two input functions
    "d150_h1": _cfg(150, 1, 2, 1),        # dh 150 -> 152: a padded wide head, kernels at d = 160
    "d184_h2": _cfg(184, 2, 2, 1),        # dh 92 at a padded width (kernels at d = 192)
    # (round 6) every width the d = 256 kernels cannot take runs at the next multiple of 64 from 320 on the
    # one-Linear-at-a-time chains, linear.hip's whole-row projection tilings keeping any head in one workgroup
    "d250_h10": _cfg(250, 10, 2, 1),      # heads of 25 -> 28: 280 internal columns, kernels at d = 320
    "d200_h5": _cfg(200, 5, 2, 0),        # heads of 40 (no d = 256 softmax group): kernels at d = 320
    "d256_h32": _cfg(256, 32, 2, 1, nl=2),  # heads of 8 at d = 256: kernels at d = 320
    "d384_h3": _cfg(384, 3, 2, 1, nl=2),  # heads of 128 above d = 256 (wide attention, whole-row projections)
    "d300_h5": _cfg(300, 5, 2, 0),        # heads of 60 at a padded 320
    # (round 6) above 512: the next multiple of 128 up to 1024, every full-width contraction in two halves on the
    # 320 .. 512 kernels (launch_linear's K-split over half images; the batched input-function K / V and their
    # backward-data split on the host)
    "d576_h9": _cfg(576, 9, 2, 1),        # heads of 64, kernels at 640 (fc_out contracts 576 = 320 + 256 columns)
    "d768_h24": _cfg(768, 24, 2, 0, nl=2),  # heads of 32, self-attention only
    "d1024_h16": _cfg(1024, 16, 2, 2, nl=2),  # heads of 64, two input functions
    "d640_l3": _cfg(640, 10, 2, 1, L=3, nl=1),  # three blocks: the d(fn) backward-data in two accumulating launches
}


@functools.lru_cache(maxsize=None)
def _case(name):
    """the oracle result of a case (computed once for both attention paths)"""
    cfg = CASES[name]
    Ms = [[120, 77], [64, 31]][: cfg["n_input_functions"]]
    return _random_case(13, cfg, [300, 173], Ms)


@pytest.mark.parametrize("name", sorted(CASES))
def test_width_vs_oracle(name, attn_path):
    fx, G = _case(name)
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs


@pytest.mark.parametrize("name", ["d208_h13", "d224_h7"])
def test_padded_256_width_bf16_mode(name):
    """bf16 mode (one RNE bf16 piece per MFMA operand, bf16 storage of the soft-MoE chains) on a width
    padded to the d = 256 kernels: north_star's 1e-2 norm-wise against the fp64 oracle (tests/test_gpu_bf16.py
    bar), and really a different arithmetic from the fp32 result."""
    import numpy as np
    fx, G = _case(name)
    m = build_model(fx["params"], fx["cfg"])
    out32, g32 = run_packed(m, fx, G)
    m.set_precision("bf16")
    m.zero_grad(set_to_none=True)
    out16, g16 = run_packed(m, fx, G)
    keys = list(fx["grads"].keys())
    cat = lambda g: np.concatenate([g[k].ravel() for k in keys])
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
    e_out, e_grad = rel(out16, fx["out"]), rel(cat(g16), cat(fx["grads"]))
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)
    assert rel(out16, out32) > 1e-6


# wide input / output widths at d > 256: the first and last Linears of the chains run the projection kernel
# at the plan's full padded width (engine.cpp kt_of: one tile, or every tile of the hidden width)
CASES["d320_wide_io"] = dict(input_dim=150, theta_dim=60, input_func_dim=200, out_dim=200, n_attn_layers=1, d=320,
                             n_mlp_num_layers=2, n_expert=2, n_head=10, n_input_functions=1)


def test_wide_io_widths_above_256():
    """input_dim + theta_dim = 210, input_func_dim = 200 and out_dim = 200 beside a d = 320 hidden width
    (chainw.hip: every first / last Linear at the 320-wide projection instantiation) vs the oracle."""
    fx, G = _case("d320_wide_io")
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs


@pytest.mark.parametrize("name", ["d100_h5", "d208_h13", "d288_h18", "d100_h4"])
def test_padded_width_pad_columns_stay_zero_across_steps(name):
    """Padded widths keep their pad columns at exact zero only because the workspace is cleared at bind
    and no kernel writes a non-zero pad value.  Three steps on one bound plan: the
    first and third on the case's inputs, the second on other inputs (other values in every reused
    buffer); the third step's output and gradients must be bitwise the first's."""
    import numpy as np
    import torch
    fx, G = _case(name)
    m = build_model(fx["params"], fx["cfg"])
    out1, g1 = run_packed(m, fx, G)
    rng = np.random.default_rng(99)
    fx2 = dict(fx, x=rng.random(fx["x"].shape) * 3 - 1, theta=rng.random(fx["theta"].shape) * 5,
               fns=[rng.random(f.shape) * 4 - 2 for f in fx["fns"]])
    run_packed(m, fx2, rng.standard_normal(G.shape) * 10)
    out3, g3 = run_packed(m, fx, G)
    assert np.array_equal(out1, out3)
    assert all(np.array_equal(g1[k], g3[k]) for k in g1), [k for k in g1 if not np.array_equal(g1[k], g3[k])]
    torch.cuda.synchronize()


@pytest.mark.parametrize("name", ["d16_h4", "d96_h8", "d100_h5", "d144_h4", "d176_h4", "d192_h6", "d100_h4", "d90_h6"])
def test_width_bf16_mode(name):
    """The bf16 arithmetic mode at d <= 192 (chain.hip / linear.hip / the 128-tile weight gradients on one
    RNE bf16 piece per operand), padded widths included: north_star's 1e-2 norm-wise vs the fp64 oracle, and
    really another arithmetic than the fp32 path."""
    import numpy as np
    fx, G = _case(name)
    m = build_model(fx["params"], fx["cfg"])
    out32, g32 = run_packed(m, fx, G)
    m.set_precision("bf16")
    out16, g16 = run_packed(m, fx, G)
    keys = list(fx["grads"].keys())
    cat = lambda g: np.concatenate([g[k].ravel() for k in keys])
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
    e_out, e_grad = rel(out16, fx["out"]), rel(cat(g16), cat(fx["grads"]))
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)
    assert rel(out16, out32) > 1e-6


@pytest.mark.parametrize("name", ["d320_h10", "d200_h5", "d576_h9"])
def test_bf16_mode_above_256_runs_the_fp32_path(name):
    """Above an internal width of 256 (chainw.hip, fp32-MFMA projections: d > 256, and head layouts the d = 256
    kernels cannot take, e.g. d = 200 with heads of 40) the bf16 mode has no one-piece kernels: the results
    are the fp32 path's, bit for bit."""
    import numpy as np
    fx, G = _case(name)
    m = build_model(fx["params"], fx["cfg"])
    out32, g32 = run_packed(m, fx, G)
    m.set_precision("bf16")
    out16, g16 = run_packed(m, fx, G)
    assert np.array_equal(out16, out32) and all(np.array_equal(g16[k], g32[k]) for k in g32)
