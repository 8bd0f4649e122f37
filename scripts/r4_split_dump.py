"""SPLIT diagnosis: the mains' and the helpers' layer-1 hidden-tile-1 partial
of the first step (libfedmx_hip_splitd2.so dumps both into the stamps buffer)."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/tests")
from test_kernels_gpu import _setup_pair  # noqa: E402

from fedmse_decentralized_amd.engine.base import TrainHParams  # noqa: E402
from fedmse_decentralized_amd.ops import _hip  # noqa: E402

_, a = _setup_pair(n_train=(12, 12), n_valid=(14, 9), seed=13)
st = torch.zeros(2048, dtype=torch.int64, device="cuda")
hp = TrainHParams(epochs=1, batch_size=12, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.0, patience=10 ** 6)
_hip.train(a.store, [0, 1], hp, a.dims, stamps=st, helper=True)
torch.cuda.synchronize()
v = st.cpu().numpy().astype(np.uint32).view(np.float32).reshape(2, 4, 64, 4)   # role, wave, lane, r
m, h = v[0], v[1]
d = np.abs(m - h)
print("sample main", m[0, :2].tolist(), "helper", h[0, :2].tolist(), "nonzero", int((m != 0).sum()))
print("max |main - helper|", float(d.max()), "mismatches", int((m != h).sum()), "of", m.size)
for w in range(4):
    bad = np.argwhere(m[w] != h[w])
    print("wave", w, "mismatching (lane, r):", bad[:8].tolist(), "main", m[w][tuple(bad[:3].T)] if len(bad) else "",
          "helper", h[w][tuple(bad[:3].T)] if len(bad) else "")
