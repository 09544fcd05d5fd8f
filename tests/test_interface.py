"""CPU-side checks of the drop-in boundary: state_dict layout, the C ABI library, plan logic."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from golden_util import fixture_names, load, model_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnot_hip.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|size_t|const char\*)\s+(gnot_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from gnot_amd import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(_lib.EXPORTS) == names
    assert b"gfx950" in lib.gnot_version()


@pytest.mark.parametrize("name", fixture_names())
def test_state_dict_matches_reference(name):
    """Same keys, order and shapes as the reference module -> checkpoints interchange."""
    from gnot_amd import GNOT
    fx = load(name)
    m = GNOT(*model_args(fx["cfg"]))
    sd = m.state_dict()
    assert list(sd.keys()) == list(fx["params"].keys())
    for k, v in sd.items():
        assert tuple(v.shape) == fx["params"][k].shape, k
    m.load_state_dict({k: torch.from_numpy(v).float() for k, v in fx["params"].items()})


@pytest.mark.parametrize("name", fixture_names())
def test_plan_linear_order_matches_module(name):
    """The native plan's canonical Linear list == the module's named_parameters order."""
    from gnot_amd import GNOT
    from gnot_amd import _lib
    fx = load(name)
    m = GNOT(*model_args(fx["cfg"]))
    lin = m.linears()
    names = [k[:-len(".weight")] for k in m.state_dict() if k.endswith(".weight")]
    assert len(names) == len(lin)
    lib = _lib.load()
    cfg = _lib.GnotConfig(**m._cfg)
    plan = ctypes.c_void_p()
    _lib.check(lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan)))
    try:
        n = lib.gnot_plan_num_linears(plan)
        dims = (ctypes.c_int32 * (2 * n))()
        _lib.check(lib.gnot_plan_linear_dims(plan, dims))
        assert n == len(lin)
        for k, l in enumerate(lin):
            assert (dims[2 * k], dims[2 * k + 1]) == tuple(l.weight.shape)
        # batch geometry + workspace sizing are host-only
        B = len(fx["x_off"]) - 1
        xo = (ctypes.c_int64 * (B + 1))(*[int(v) for v in fx["x_off"]])
        flat = [int(v) for o in fx["fn_offs"] for v in o]
        fo = (ctypes.c_int64 * max(1, len(flat)))(*flat)
        _lib.check(lib.gnot_plan_set_batch(plan, B, xo, fo if flat else None, 1))
        need = lib.gnot_plan_workspace_bytes(plan)
        assert need > 0
        offs = (ctypes.c_int64 * (2 * n))()
        _lib.check(lib.gnot_plan_grad_offsets(plan, offs))
        total = sum(o * i + o for o, i in (tuple(l.weight.shape) for l in lin))
        assert offs[2 * n - 1] + lin[-1].weight.shape[0] == total
    finally:
        lib.gnot_plan_destroy(plan)


def test_constructor_errors_mirror_reference():
    from gnot_amd import GNOT
    with pytest.raises(AssertionError, match="divisible by head"):
        GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 5, 1)


def test_plan_rejects_bad_config_and_batch():
    from gnot_amd import _lib
    lib = _lib.load()
    good = dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, n_attn_hidden_dim=32,
                n_mlp_num_layers=2, n_mlp_hidden_dim=32, n_input_hidden_dim=32, n_expert=2, n_head=4,
                n_input_functions=1)
    plan = ctypes.c_void_p()
    for bad in (dict(n_mlp_hidden_dim=64), dict(n_head=5),
                dict(n_attn_hidden_dim=264, n_mlp_hidden_dim=264, n_input_hidden_dim=264, n_head=1)):   # dh 264 > 256
        cfg = _lib.GnotConfig(**{**good, **bad})
        assert lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan)) == -1
        assert lib.gnot_last_error()
    cfg = _lib.GnotConfig(**good)
    _lib.check(lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan)))
    try:
        xo = (ctypes.c_int64 * 3)(0, 5, 3)         # decreasing
        fo = (ctypes.c_int64 * 3)(0, 2, 4)
        assert lib.gnot_plan_set_batch(plan, 2, xo, fo, 1) == -1
        xo = (ctypes.c_int64 * 3)(0, 5, 9)
        assert lib.gnot_plan_set_batch(plan, 2, xo, None, 1) == -1   # fn offsets required
        assert lib.gnot_forward(plan, None, None, None, None, None) == -3   # not bound
    finally:
        lib.gnot_plan_destroy(plan)


def test_padded_widths():
    """A hidden width that is not a multiple of 16 (up to 192) runs on the next multiple's kernels: the
    plan accepts it and its canonical Linears keep the model's width (the parameter shapes); d in
    (192, 256) runs on the d = 256 kernels (head widths 16 / 32 / 64 there), d in (256, 512] on the
    one-Linear-at-a-time chains (chainw.hip; head widths dividing 64); a head width that is not a multiple
    of 4 runs on heads padded to one (d = 100 with 4 heads of 25: kernels at 112; d = 190 with 10 heads of
    19: 10 x 20 = 200 columns, kernels at 320); everything the d = 256 kernels cannot take (heads other than
    16 / 32 / 64 / 128 / 256, padded heads) runs at the next multiple of 64 from 320, above 512 at the next
    multiple of 128 (heads dividing 64); head widths above 256 and internal widths above 1024 are refused (round 6: d * dh is no longer bounded -- d = 512 / 320 with heads of 64 run).  (Point sharding takes every width the plan takes, tests/test_gpu_shard.py.)"""
    from gnot_amd import _lib
    lib = _lib.load()
    base = dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, n_mlp_num_layers=2,
                n_expert=2, n_input_functions=1)
    plan = ctypes.c_void_p()
    for d, H, ok in ((36, 3, True), (100, 5, True), (60, 15, True), (208, 13, True), (224, 7, True),
                     (320, 10, True), (288, 18, True), (512, 16, True), (512, 8, True),
                     (100, 4, True), (21, 7, True), (150, 6, True), (190, 10, True),
                     (200, 5, True), (184, 2, True), (300, 5, True), (576, 9, True),
                     (320, 5, True),                   # heads of 64 above 256 (d * dh up to 32,768)
                     # heads wider than 64 (round 6): up to 256 at d <= 256 (128 / 256 on the d = 256 kernels)
                     (128, 1, True), (136, 2, True), (192, 2, True), (150, 1, True), (256, 2, True), (256, 1, True),
                     (240, 2, True), (384, 3, True),
                     # (round 6) widths the d = 256 kernels cannot take run at the next multiple of 64 from 320 on
                     # the one-Linear-at-a-time chains: heads padded past an internal 192 (250 = 10 x 25 -> 10 x 28),
                     # d = 256 with heads of 8 (-> 320); refused: d > 512, heads above 256, 10 x 52 = 520 > 512
                     (250, 10, True), (256, 32, True), (512, 1, False), (300, 1, False),
                     # above 512: the next multiple of 128 up to 1024 (K-split projections), heads dividing 64
                     (510, 10, False), (1024, 16, True), (768, 24, True), (640, 5, False), (1100, 11, False)):
        cfg = _lib.GnotConfig(**base, n_attn_hidden_dim=d, n_mlp_hidden_dim=d, n_input_hidden_dim=d, n_head=H)
        rc = lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan))
        assert (rc == 0) == ok, (d, H, rc)
        if not ok:
            continue
        try:
            n = lib.gnot_plan_num_linears(plan)
            dims = (ctypes.c_int32 * (2 * n))()
            _lib.check(lib.gnot_plan_linear_dims(plan, dims))
            assert max(dims) == d                  # every hidden Linear is d x d (no pad in the parameters)
        finally:
            lib.gnot_plan_destroy(plan)


def test_plan_accepts_meshes_past_the_old_32bit_offset_limit():
    """The streaming kernels base their buffer resources per workgroup / per split-K range (64-bit base,
    32-bit in-tile offsets), so a plan takes configs[4]'s ~1.6M points and configs[3]'s 1M-point mesh at
    d = 256 on one GPU (round 3 refused more than 0xFFFFFFFF / (12 d) = 1,398,101 points).  Only the
    32-bit point indices of the job tables bound a plan (2^29 points)."""
    from gnot_amd import _lib
    lib = _lib.load()
    cfg = _lib.GnotConfig(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1,
                          n_attn_hidden_dim=256, n_mlp_num_layers=4, n_mlp_hidden_dim=256, n_input_hidden_dim=256,
                          n_expert=8, n_head=8, n_input_functions=1)
    plan = ctypes.c_void_p()
    _lib.check(lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan)))
    try:
        fo = (ctypes.c_int64 * 2)(0, 805)
        for n in (1398102, 4_000_000):
            _lib.check(lib.gnot_plan_set_batch(plan, 1, (ctypes.c_int64 * 2)(0, n), fo, 1))
            assert lib.gnot_plan_workspace_bytes(plan) > n * 256 * 4
        assert lib.gnot_plan_set_batch(plan, 1, (ctypes.c_int64 * 2)(0, 1 << 29), fo, 0) == -1
        assert b"32-bit" in lib.gnot_last_error()
        assert lib.gnot_plan_set_batch(plan, 1, (ctypes.c_int64 * 2)(0, 1000),
                                       (ctypes.c_int64 * 2)(0, 1 << 29), 0) == -1
    finally:
        lib.gnot_plan_destroy(plan)


def test_forward_refuses_cpu_tensors():
    from gnot_amd import GNOT
    m = GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 0)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m(torch.rand(1, 10, 2), torch.rand(1, 1))


def test_missing_input_functions_raises_like_reference():
    from gnot_amd import GNOT
    m = GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1)
    with pytest.raises(NotImplementedError):
        m(torch.rand(1, 10, 2), torch.rand(1, 1))


def test_moe_recompute_shrinks_training_workspace():
    """gnot_plan_set_moe_recompute: the per-MoE-call saves (E*nl*P*d each, 2 per block) become one
    shared buffer; it invalidates the batch (set_batch must run again)."""
    from gnot_amd import _lib
    lib = _lib.load()
    cfg = _lib.GnotConfig(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                          n_attn_hidden_dim=64, n_mlp_num_layers=4, n_mlp_hidden_dim=64, n_input_hidden_dim=64,
                          n_expert=8, n_head=4, n_input_functions=1)
    plan = ctypes.c_void_p()
    _lib.check(lib.gnot_plan_create(ctypes.byref(cfg), ctypes.byref(plan)))
    try:
        P, M, E, NL, L, d = 4096, 100, 8, 5, 4, 64
        xo, fo = (ctypes.c_int64 * 2)(0, P), (ctypes.c_int64 * 2)(0, M)
        _lib.check(lib.gnot_plan_set_batch(plan, 1, xo, fo, 1))
        plain = lib.gnot_plan_workspace_bytes(plan)
        _lib.check(lib.gnot_plan_set_moe_recompute(plan, 1))
        assert lib.gnot_plan_workspace_bytes(plan) == 0          # batch invalidated
        _lib.check(lib.gnot_plan_set_batch(plan, 1, xo, fo, 1))
        rc = lib.gnot_plan_workspace_bytes(plan)
        saves = E * NL * P * d * 4
        assert plain - rc >= (2 * L - 1) * saves * 0.99, (plain, rc)
        _lib.check(lib.gnot_plan_set_batch(plan, 1, xo, fo, 0))  # inference: no saves either way
        inf_rc = lib.gnot_plan_workspace_bytes(plan)
        _lib.check(lib.gnot_plan_set_moe_recompute(plan, 0))
        _lib.check(lib.gnot_plan_set_batch(plan, 1, xo, fo, 0))
        assert lib.gnot_plan_workspace_bytes(plan) == inf_rc
    finally:
        lib.gnot_plan_destroy(plan)
