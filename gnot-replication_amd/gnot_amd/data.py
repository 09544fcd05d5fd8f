"""NS2d-format data and batching without dgl.

Reference format (dataset.py:7, 19-36): a pickled list of samples `[X (N x in), Y (N x out), theta
(length theta_dim), [f_1 (M_1 x F), f_2, ...]]` of numpy arrays.  `NS2dData` mirrors
`NS2dDataset.__getitem__` (dataset.py:43-44) with plain tensors instead of a DGLGraph, and reads the
pickle with a restricted unpickler that only rebuilds numpy arrays and plain containers (a pickle
cannot run code through it).  `collate_packed` is the packed-offsets batch the engine consumes
(replacing the padding of main.py:60-82 and utils.py:3-4); `collate_padded` reproduces the
reference's padded tensors exactly, for parity runs.  `synthetic_sample` / `write_ns2d` generate
meshes in the same on-disk format.
"""
import io
import pickle

import numpy as np
import torch

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("builtins", "list"), ("builtins", "tuple"),
}


class _ArrayUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"NS2d files may only hold numpy arrays; refusing {module}.{name}")


def safe_load(path):
    with open(path, "rb") as f:
        return _ArrayUnpickler(io.BytesIO(f.read())).load()


def write_ns2d(path, samples):
    """Write samples [[X, Y, theta, [f...]], ...] (numpy) in the reference's pickle format."""
    with open(path, "wb") as f:
        pickle.dump([[np.asarray(s[0]), np.asarray(s[1]), np.asarray(s[2]), [np.asarray(v) for v in s[3]]]
                     for s in samples], f, protocol=4)


def synthetic_sample(rng, n_points, input_dim=2, out_dim=1, theta_dim=1, fn_points=(805,), fn_dim=3):
    """One synthetic mesh in the NS2d layout: coordinates U[0,1]^input_dim, a smooth field as target,
    theta U[0,1], input functions U[0,1]^fn_dim."""
    x = rng.random((n_points, input_dim))
    theta = rng.random(theta_dim)
    y = np.stack([np.sin(np.pi * (c + 1) * x.sum(1)) * (1 + theta[0]) for c in range(out_dim)], 1)
    fns = [rng.random((m, fn_dim)) for m in fn_points]
    return [x.astype(np.float64), y.astype(np.float64), theta, fns]


class NS2dData(torch.utils.data.Dataset):
    """dataset.py:6-44 without dgl: item = (x [N, in], y [N, out], theta, [f_i [M_i, F]])."""

    def __init__(self, path_or_samples):
        self.data = safe_load(path_or_samples) if isinstance(path_or_samples, str) else path_or_samples
        self.items = []
        for s in self.data:
            fns = [torch.from_numpy(np.asarray(f)).float() for f in s[3]] if s[3] else []
            self.items.append((torch.from_numpy(np.asarray(s[0])).float(), torch.from_numpy(np.asarray(s[1])).float(),
                               s[2], fns))

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def collate_packed(batch):
    """Packed batch (no padding): x [sum N, in], x_off [B+1], y, theta [B, theta_dim], fns[i] packed with
    fn_offs[i] [B+1].  GNOT.forward_packed(x, x_off, theta, fns, fn_offs) on it equals one unpadded
    B=1 reference call per sample."""
    xs, ys, thetas, fnl = zip(*batch)
    off = [0]
    for x in xs:
        off.append(off[-1] + x.shape[0])
    I = len(fnl[0])
    fns, fn_offs = [], []
    for i in range(I):
        parts = [f[i] for f in fnl]
        o = [0]
        for p in parts:
            o.append(o[-1] + p.shape[0])
        fns.append(torch.cat(parts))
        fn_offs.append(o)
    theta = torch.tensor(np.stack([np.asarray(t, dtype=np.float64) for t in thetas])).float()
    return dict(x=torch.cat(xs), x_off=off, y=torch.cat(ys), theta=theta, fns=fns, fn_offs=fn_offs)


def collate_padded(batch):
    """The reference's batch exactly (main.py:60-82, utils.py:3-4): x zero-padded to the batch max N,
    every input function zero-padded to ONE common max M over all functions and samples, stacked
    [I, B, M, F]; y is returned packed ([sum N, out], main.py:89/93) with the real counts."""
    xs, ys, thetas, fnl = zip(*batch)
    pad = lambda t, L: torch.nn.functional.pad(t, (0, 0, 0, L - t.shape[0]))
    mmax = max((t.shape[0] for arrays in fnl for t in arrays), default=0)
    I = len(fnl[0])
    fns = torch.stack([torch.stack([pad(arrays[i], mmax) for arrays in fnl]) for i in range(I)]) if I else None
    nmax = max(t.shape[0] for t in xs)
    x = torch.stack([pad(t, nmax) for t in xs])
    theta = torch.tensor(np.stack([np.asarray(t, dtype=np.float64) for t in thetas])).float()
    return dict(x=x, theta=theta, fns=fns, y=torch.cat(ys), counts=[t.shape[0] for t in xs])
