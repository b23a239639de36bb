"""Synthetic coexpression datasets for the benchmark configurations.

Per module m of k_m genes: an eigengene E_m ~ N(0,1)^S and per-gene loadings
r ~ U(0.3, 0.9) * (+-1); gene = r * E_m + sqrt(1 - r^2) * eps. Background genes
(label "0") are pure noise. Discovery and test draw independent noise; the
test dataset keeps the eigengene structure of every other module (preserved)
and replaces the rest by noise. corr = Pearson correlation of the data,
net = |corr|^5 (the bundled example's construction, R/example-data.R).

Small cases are built with numpy on the host; benchmark-size cases with torch
on the GPU (``device="cuda"``) so the 20k x 20k matrices never leave HBM.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

CONFIGS = {
    # name: (n_nodes, n_samples, module sizes, n_perm, data?)
    "C1": None,  # the bundled data, tests/golden/netrep_bundled.npz
    "C2": (5000, 100, np.round(np.linspace(30, 300, 20)).astype(int), 10_000, True),
    "C3": (20000, 500, np.round(np.linspace(30, 300, 50)).astype(int), 100_000, True),
    "C4": (20000, 500, np.round(np.linspace(30, 300, 50)).astype(int), 1_000_000, False),
    "C5": (40000, 1000, np.round(np.geomspace(30, 2000, 40)).astype(int), 100, True),
    # small case of the same shape for the multi-rank GPU test (tests/test_gpu_distributed.py)
    "CT": (3000, 120, np.round(np.linspace(30, 300, 8)).astype(int), 192, True),
}


@dataclass
class Layout:
    n_nodes: int
    module_sizes: np.ndarray
    names: list = field(default_factory=list)
    labels: list = field(default_factory=list)
    modules: list = field(default_factory=list)
    members: dict = field(default_factory=dict)   # label -> node positions (assignment order)


def make_layout(n_nodes: int, module_sizes, seed: int) -> Layout:
    rng = np.random.default_rng(seed)
    sizes = np.asarray(module_sizes, dtype=int)
    if sizes.sum() > n_nodes:
        raise ValueError("modules larger than the network")
    perm = rng.permutation(n_nodes)
    labels = np.full(n_nodes, "0", dtype=object)
    members = {}
    o = 0
    for i, k in enumerate(sizes):
        lab = str(i + 1)
        pos = np.sort(perm[o:o + k])
        labels[pos] = lab
        members[lab] = pos
        o += k
    names = [f"G{i + 1}" for i in range(n_nodes)]
    return Layout(n_nodes, sizes, names, list(labels), [str(i + 1) for i in range(len(sizes))], members)


def _gen_numpy(layout: Layout, n_samples: int, rng, preserved: set):
    x = rng.standard_normal((n_samples, layout.n_nodes))
    for lab, pos in layout.members.items():
        if lab not in preserved:
            continue
        e = rng.standard_normal(n_samples)
        r = rng.uniform(0.3, 0.9, size=pos.size) * rng.choice([-1.0, 1.0], size=pos.size)
        x[:, pos] = np.outer(e, r) + np.sqrt(1 - r * r) * x[:, pos]
    return x


def numpy_dataset(layout: Layout, n_samples: int, seed: int, preserve_all: bool = True):
    """(data S x N, corr N x N, net N x N) as numpy arrays."""
    rng = np.random.default_rng(seed)
    mods = layout.modules
    preserved = set(mods) if preserve_all else set(mods[::2])
    x = _gen_numpy(layout, n_samples, rng, preserved)
    corr = np.corrcoef(x, rowvar=False)
    corr = np.triu(corr) + np.triu(corr, 1).T     # exactly symmetric, as R's cor() returns
    net = np.abs(corr) ** 5
    return x, corr, net


def torch_dataset(layout: Layout, n_samples: int, seed: int, preserve_all: bool = True,
                  device="cuda"):
    """Same construction on the GPU with torch (fp64). Returns (data, corr, net) tensors,
    column-major as R expects: data is stored (N, S) row-major == (S, N) column-major."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n, s = layout.n_nodes, n_samples
    mods = layout.modules
    preserved = set(mods) if preserve_all else set(mods[::2])
    xt = torch.randn((n, s), generator=g, device=device, dtype=torch.float64)  # row j = gene j
    for lab, pos in layout.members.items():
        if lab not in preserved:
            continue
        p = torch.as_tensor(pos, device=device)
        e = torch.randn(s, generator=g, device=device, dtype=torch.float64)
        r = (torch.rand(p.numel(), generator=g, device=device, dtype=torch.float64) * 0.6 + 0.3)
        sign = torch.where(torch.rand(p.numel(), generator=g, device=device) < 0.5, -1.0, 1.0).double()
        r = r * sign
        xt[p] = r[:, None] * e[None, :] + torch.sqrt(1 - r * r)[:, None] * xt[p]
    xc = xt - xt.mean(dim=1, keepdim=True)
    xc = xc / xc.norm(dim=1, keepdim=True)
    corr = xc @ xc.T
    corr = torch.triu(corr) + torch.triu(corr, 1).T   # bitwise symmetric, as R's cor() returns
    corr.diagonal().fill_(1.0)
    net = corr.abs().pow(5)
    return xt, corr, net


def scale_rows_torch(x):
    """Scale (src/scale.cpp:21) applied to genes stored as rows of x (N x S):
    (x - mean) / sd with n-1 normalisation, on the tensor's device."""
    mu = x.mean(dim=1, keepdim=True)
    sd = x.std(dim=1, unbiased=True, keepdim=True)
    return (x - mu) / sd


def csr_of(layout: Layout):
    """(node_off, idx) of the layout's modules in `modules` order (CSR)."""
    mods = layout.modules
    node_off = np.concatenate([[0], np.cumsum([layout.members[m].size for m in mods])]).astype(np.int64)
    idx = np.concatenate([layout.members[m] for m in mods]).astype(np.int32)
    return node_off, idx
