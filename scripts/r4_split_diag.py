"""Where does a training-kernel variant first differ from the 4-wave kernel?
Runs the helper-wave kernel (this process's library, FEDMX_HIP_LIB) and the
4-wave kernel from identical state for 1..K steps and prints the max abs
difference of every state tensor (split by W1 hidden tile) and of the
tracked losses."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/tests")

from test_kernels_gpu import _setup_pair  # noqa: E402

from fedmse_decentralized_amd.engine.base import TrainHParams  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS, padded_index  # noqa: E402
from fedmse_decentralized_amd.ops import _hip  # noqa: E402

DEV = torch.device("cuda", 0)
idx, segs = padded_index(DEFAULT_DIMS)
# W1 rows 0..15 (main waves) and 16..26 (SPLIT: helper waves) reported apart
segs = [(0, 16 * 115), (16 * 115, segs[0][1])] + list(segs[1:])
for n_train, epochs in ((12, 1), (24, 1), (53, 2)):
    _, a = _setup_pair(n_train=(n_train, n_train), n_valid=(14, 9), seed=13)
    _, b = _setup_pair(n_train=(n_train, n_train), n_valid=(14, 9), seed=13)
    hp = TrainHParams(epochs=epochs, batch_size=12, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.0, patience=10 ** 6)
    ta, ea, ba = _hip.train(a.store, [0, 1], hp, a.dims, helper=True)
    tb, eb, bb = _hip.train(b.store, [0, 1], hp, b.dims, helper=False)
    torch.cuda.synchronize()
    _hip.runtime(DEV).sync()
    out = {"steps": (n_train + 11) // 12 * epochs}
    for name in ("params", "adam_m", "adam_v", "best"):
        d = (getattr(a.store, name) - getattr(b.store, name)).abs()[:, idx.to(DEV)].cpu()
        out[name] = [float(d[:, s:e].max()) for s, e in segs]
    out["tracking"] = float(np.max(np.abs(np.array(ta) - np.array(tb))))
    out["train_loss_diff"] = np.abs(np.array(ta)[:, :, 0] - np.array(tb)[:, :, 0]).max(axis=1).tolist()
    out["valid_loss_diff"] = np.abs(np.array(ta)[:, :, 1] - np.array(tb)[:, :, 1]).max(axis=1).tolist()
    out["w1_rows_per_client"] = [float((a.store.params[k] - b.store.params[k]).abs().max()) for k in range(2)]
    print(out, flush=True)
