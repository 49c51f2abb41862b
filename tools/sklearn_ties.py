"""How sklearn's kneighbors orders EXACT distance ties, against the (fp64
distance, index) rule the engine and oracle/refcpu.knn_query follow.
Sources: a 48x48 lattice; queries: 200 lattice points and 200 cell centres
(every query has tied neighbours at the 30-th boundary).  Run in the container
(sklearn is importable here, not on the GPU box); DESIGN.md §2 quotes it."""
import os
import sys

import numpy as np
import torch
from sklearn.neighbors import NearestNeighbors

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import refcpu  # noqa: E402

g = np.arange(48, dtype=np.float32) / 47
src = np.stack(np.meshgrid(g, g), -1).reshape(-1, 2).astype(np.float32)
rng = np.random.default_rng(0)
qry = np.concatenate([src[rng.choice(len(src), 200, replace=False)],
                      (src[rng.choice(len(src), 200, replace=False)] + np.float32(0.5 / 47)).clip(0, 1)])
qry = qry.astype(np.float32)
nn = NearestNeighbors(n_neighbors=30).fit(src)
_, sk = nn.kneighbors(qry)
ours = refcpu.knn_query(torch.from_numpy(src), torch.from_numpy(qry), 1, 30).numpy().reshape(sk.shape)
print(f"sklearn fit method {nn._fit_method}: same 30-set {np.mean([set(a) == set(b) for a, b in zip(sk, ours)]):.3f}, "
      f"same order {np.mean([np.array_equal(a, b) for a, b in zip(sk, ours)]):.3f} of {len(qry)} tie-bearing queries")
