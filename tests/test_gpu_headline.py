"""Oracle parity at the size and kernel selection of the headline (bench.py's configs[2] line).

The small-mesh parity tests (test_gpu_parity.py, test_gpu_configs.py) run below the size thresholds
at which the engine switches kernels, so they check the VALU attention forms and short split-K
reductions.  These tests run the configs[2] model widths (d=256, 8 heads, 8 experts, 4-layer MLPs,
one 805-point input function) on meshes large enough that the DEFAULT (unforced) choice is the one
the 262,144-point bench takes:

* 70,000 points >= 65,536 per state group: the fp32-MFMA state kernel (state.hip `state_mfma`,
  ceil(70,000 / 256) = 274 partial states per sample, fixed-order reduce) instead of the VALU
  partials;
* >= 8,192 points: the MFMA attention apply / K-V backward kernels (attn_mfma.hip);
* the wide weight-gradient kernel with the SAME split counts as at 262,144 points (fixed target of
  256 workgroups: 6 splits per MoE job group of 40 Linears, 51 per single-chain group of 5), and an
  odd number of 16-point stages in the last split (70,000 - 5 * 11,680 = 11,600 points = 725
  stages), the case of the stage-buffer reuse the db column sums once raced on;
* the soft-MoE expert grid + moe_combine (the form the bench runs);
* 70,000 is not a multiple of 128 (a partial last chain workgroup) nor of 256 (a partial state block).

Checked against the float64 CPU oracle (oracle/gnot_oracle.py, pinned to the reference fixtures):
output and every parameter gradient at north_star's 1e-4 in fp32 (golden_util.check_parity), the bf16
mode at 1e-2, and two steps bitwise equal.  L = 1 block keeps the oracle in tens of seconds; every
kernel of a block (cross + self attention, both MoE calls, all weight-gradient groups) runs.

The FULL 262,144-point configs[2] model (L = 4) is checked on its forward against the stock-torch CPU
port (oracle/torch_port.py, fixture-validated) in fp32 under no_grad, the only form of the whole mesh
that fits host memory.  Anchor of the all-point sums these sizes stress:
/root/reference/model.py:77-80, 98-101.
"""
import numpy as np
import pytest
import torch

from golden_util import check_parity, rel
from test_gpu_configs import CFG_3D
from test_gpu_parity import build_model, run_packed

pytestmark = pytest.mark.gpu

N_MID, M = 70000, 805    # the session fixture mid_case (conftest.py): one 70,000-point mesh, L = 1


@pytest.mark.timeout(900)
def test_configs2_widths_70k_points_fp32(mid_case):
    """the expert grid + moe_combine, fp32."""
    fx, G = mid_case
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    keys = sorted(fx["grads"])
    cat = lambda g: np.concatenate([np.ravel(g[k]) for k in keys])
    print(f"\n70k fp32: out rel {rel(out, fx['out']):.3e}, all-grad rel {rel(cat(grads), cat(fx['grads'])):.3e}")
    assert not errs, errs
    out2, grads2 = run_packed(m, fx, G)
    assert np.array_equal(out, out2)
    for k in grads:
        assert np.array_equal(grads[k], grads2[k]), f"{k} differs between two identical steps"


@pytest.mark.timeout(900)
def test_configs2_widths_70k_points_bf16_mode(mid_case):
    """bf16 mode at 1e-2 of the fp64 oracle, in the soft-MoE form the bench runs."""
    fx, G = mid_case
    m = build_model(fx["params"], fx["cfg"])
    m.set_precision("bf16")
    out, grads = run_packed(m, fx, G)
    keys = sorted(fx["grads"])
    cat = lambda g: np.concatenate([np.ravel(g[k]) for k in keys])
    e_out, e_grad = rel(out, fx["out"]), rel(cat(grads), cat(fx["grads"]))
    print(f"\n70k bf16 mode: out rel {e_out:.3e}, all-grad rel {e_grad:.3e}")
    assert e_out < 1e-2 and e_grad < 1e-2, (e_out, e_grad)


@pytest.mark.timeout(900)
def test_configs2_full_262144_point_forward_vs_cpu_port():
    """The bench's exact model and mesh (bench.py make_batch seed 100, weights of torch.manual_seed(1234))
    through the HIP forward vs the stock-torch CPU port on the same fp32 weights: whole output within
    1e-4 relative (norm-wise)."""
    from gnot_amd import GNOT
    from oracle import torch_port
    N = 262144
    cfg = dict(CFG_3D, n_attn_hidden_dim=256)
    torch.manual_seed(1234)
    model = GNOT(3, 1, 3, 1, 4, 256, 4, 256, 256, 8, 8, 1)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    g = torch.Generator(device="cpu").manual_seed(100)
    x = torch.rand(N, 3, generator=g)
    theta = torch.rand(1, 1, generator=g)
    fn = torch.rand(M, 3, generator=g)
    dev = torch.device("cuda")
    model = model.to(dev)
    with torch.no_grad():
        got = model.forward_packed(x.to(dev), [0, N], theta.to(dev), [fn.to(dev)], [[0, M]]).cpu()
        del model
        torch.cuda.empty_cache()
        ref = torch_port.gnot_forward(sd, dict(cfg, d=256), x[None], theta, [fn[None]])[0]
    e = rel(got.double().numpy(), ref.double().numpy())
    print(f"\n262,144-point forward vs CPU port: rel {e:.3e}")
    assert torch.isfinite(got).all()
    assert e < 1e-4, e
