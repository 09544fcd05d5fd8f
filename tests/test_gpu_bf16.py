"""bf16 arithmetic mode (GNOT.set_precision('bf16'), gnot_plan_set_precision): BASELINE configs[2]'s
bf16 training.  The d = 256 MLP chains, attention projections and weight gradients take ONE
round-to-nearest bf16 piece per MFMA operand (fp32 accumulation).  Bar: north_star's "1e-2 in bf16",
norm-wise against the float64 oracle -- the whole output and all gradients concatenated within 1e-2
relative (the reference's own bf16-autocast error is 3.3e-3 / 2.6e-3) -- and the mode
must really differ from the fp32 path (a silent fallback to bf16x6 would pass the bar trivially)."""
import numpy as np
import pytest
import torch

from test_gpu_configs import CFG_3D, CFG_CFG2
from test_gpu_parity import _random_case, build_model, run_packed

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.mark.parametrize("n_attn_layers", [1, 4])
def test_bf16_mode_within_1e2_of_fp64_reference(n_attn_layers):
    cfg = dict(CFG_3D, n_attn_layers=n_attn_layers)
    fx, G = _random_case(21, cfg, [1500, 548], [[805, 300]])
    m = build_model(fx["params"], fx["cfg"])
    out32, g32 = run_packed(m, fx, G)
    m.set_precision("bf16")
    m.zero_grad(set_to_none=True)
    out16, g16 = run_packed(m, fx, G)
    keys = list(fx["grads"].keys())
    cat = lambda g: np.concatenate([g[k].ravel() for k in keys])
    e_out = _rel(out16, fx["out"])
    e_grad = _rel(cat(g16), cat(fx["grads"]))
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)
    # the bf16 path is a different arithmetic: visibly less exact than fp32 (which meets 1e-4) ...
    assert _rel(out16, out32) > 1e-6 and _rel(cat(g16), cat(g32)) > 1e-6
    # ... and switching back restores the fp32 results
    m.set_precision("fp32")
    m.zero_grad(set_to_none=True)
    out32b, g32b = run_packed(m, fx, G)
    assert np.array_equal(out32b, out32)
    assert all(np.array_equal(g32b[k], g32[k]) for k in keys)


def _bf16_vs_oracle(fx, G):
    """(e_out, e_grad) of the bf16 mode vs the float64 oracle, after checking that the mode changes the
    arithmetic and that switching back restores the fp32 bits"""
    m = build_model(fx["params"], fx["cfg"])
    out32, g32 = run_packed(m, fx, G)
    m.set_precision("bf16")
    m.zero_grad(set_to_none=True)
    out16, g16 = run_packed(m, fx, G)
    keys = list(fx["grads"].keys())
    cat = lambda g: np.concatenate([g[k].ravel() for k in keys])
    assert _rel(out16, out32) > 1e-6 and _rel(cat(g16), cat(g32)) > 1e-6
    m.set_precision("fp32")
    m.zero_grad(set_to_none=True)
    out32b, g32b = run_packed(m, fx, G)
    assert np.array_equal(out32b, out32) and all(np.array_equal(g32b[k], g32[k]) for k in keys)
    return _rel(out16, fx["out"]), _rel(cat(g16), cat(fx["grads"]))


@pytest.mark.timeout(300)
def test_bf16_mode_configs1_exact_shape():
    """configs[1] ("fp32 and bf16") in the bf16 mode at bench.py --workload cfg2's shape:
    d = 128, 4 experts, 8 heads, 4 blocks, two 805-point input functions, one 10,000-point mesh.  At d <= 192
    the mode runs chain.hip (k-major one-piece images, forward AND backward-data), linear.hip (output-major
    one-piece projections) and the 128-tile weight gradients on one RNE bf16 piece per operand, fp32
    accumulation; the attention contractions stay fp32 (as at d = 256).  north_star's 1e-2 vs float64."""
    fx, G = _random_case(9, CFG_CFG2, [10000], [[805], [805]])
    e_out, e_grad = _bf16_vs_oracle(fx, G)
    print(f"\nconfigs[1] bf16 mode: output {e_out:.2e}, gradients {e_grad:.2e}")
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)


@pytest.mark.parametrize("d,H", [(256, 2), (256, 1), (128, 1)])
def test_bf16_mode_wide_heads(d, H):
    """Heads wider than 64 (round 6) in the bf16 mode: the d = 256 projections' 128- and 256-feature softmax
    heads on the one-piece linear2 forms, d = 128 on linear.hip's; the attention contractions run attn.hip's
    wide forms in fp32.  north_star's 1e-2 vs float64, on the data of the one-block case above (heads of 32
    there).  (The norm-wise bar depends on the data: with meshes of 900 + 300 points the decoder's gradients
    dominate the norm and carry 17-18 % errors in bf16 at EVERY head count -- the reference's own
    torch.autocast run shows the same, scripts/diag_bf16_heads_autocast.py -- so that data tests nothing
    about the heads.)"""
    cfg = dict(CFG_3D, d=d, n_head=H, n_attn_layers=1)
    fx, G = _random_case(21, cfg, [1500, 548], [[805, 300]])
    e_out, e_grad = _bf16_vs_oracle(fx, G)
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)


def test_set_precision_rejects_unknown_dtype():
    from gnot_amd import GNOT
    m = GNOT(3, 1, 3, 1, 1, 256, 2, 256, 256, 2, 8, 1)
    with pytest.raises(ValueError):
        m.set_precision("fp16")


@pytest.mark.parametrize("cast", ["bfloat16", "float64"])
def test_module_casts_raise_with_the_route(cast):
    """The reference runs whatever dtype its module is cast to (model.py:142-173).  Here the parameters stay
    fp32: a bf16 (or fp16) cast raises pointing at set_precision('bf16'), the bf16 arithmetic mode, and a
    float64 cast raises naming the fp32 MFMA path."""
    import torch
    from gnot_amd import GNOT
    m = GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1).cuda().to(getattr(torch, cast))
    x = torch.rand(1, 50, 2, device="cuda")
    th = torch.rand(1, 1, device="cuda")
    fn = torch.rand(1, 20, 3, device="cuda")
    with pytest.raises(RuntimeError, match="set_precision" if cast == "bfloat16" else "float64"):
        m(x, th, [fn])
