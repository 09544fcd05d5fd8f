"""NS2d format, safe loading and batching, CPU only."""
import os
import pickle

import numpy as np
import pytest
import torch

from gnot_amd import data


def _samples(rng, n=5, I=2):
    return [data.synthetic_sample(rng, int(rng.integers(3, 40)), fn_points=tuple(int(rng.integers(2, 9)) for _ in range(I)))
            for _ in range(n)]


def test_roundtrip_reference_format(tmp_path):
    rng = np.random.default_rng(0)
    s = _samples(rng)
    p = os.path.join(tmp_path, "ns2d.pkl")
    data.write_ns2d(p, s)
    raw = pickle.load(open(p, "rb"))            # our own file: the reference loader's view of it
    assert len(raw) == len(s) and len(raw[0]) == 4 and isinstance(raw[0][3], list)
    ds = data.NS2dData(p)
    for (x, y, th, fns), ref in zip(ds, s):
        assert torch.equal(x, torch.from_numpy(ref[0]).float()) and torch.equal(y, torch.from_numpy(ref[1]).float())
        assert np.array_equal(th, ref[2]) and len(fns) == len(ref[3])


def test_safe_loader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    p = os.path.join(tmp_path, "evil.pkl")
    pickle.dump([[np.zeros((2, 2)), np.zeros((2, 1)), np.zeros(1), [Evil()]]], open(p, "wb"))
    with pytest.raises(pickle.UnpicklingError):
        data.safe_load(p)


def test_packed_and_padded_collate_match_the_reference_batching():
    rng = np.random.default_rng(1)
    batch = list(data.NS2dData(_samples(rng, n=4, I=2)))
    pk = data.collate_packed(batch)
    pd = data.collate_padded(batch)
    counts = [b[0].shape[0] for b in batch]
    assert pk["x_off"] == list(np.concatenate([[0], np.cumsum(counts)]))
    # the padded batch holds the packed rows followed by zeros (utils.py:3-4, main.py:63-82)
    N = max(counts)
    M = max(f.shape[0] for b in batch for f in b[3])
    assert pd["x"].shape == (4, N, 2) and pd["fns"].shape == (2, 4, M, 3)
    for b in range(4):
        rows = pk["x"][pk["x_off"][b]:pk["x_off"][b + 1]]
        assert torch.equal(pd["x"][b, :counts[b]], rows) and not pd["x"][b, counts[b]:].any()
        for i in range(2):
            f = pk["fns"][i][pk["fn_offs"][i][b]:pk["fn_offs"][i][b + 1]]
            assert torch.equal(pd["fns"][i, b, :f.shape[0]], f) and not pd["fns"][i, b, f.shape[0]:].any()
    assert torch.equal(pd["y"], pk["y"]) and pk["theta"].shape == (4, 1)
