"""Process environment the multi-rank path needs, exported before HIP starts.

HSA and the HIP runtime read their environment once, when the runtime is
initialised (the first ``torch.cuda`` query that touches the driver, e.g.
``torch.cuda.is_available()``).  A variable set after that point is seen by
nothing below PyTorch.  The entry points (``bench.py``, ``main.py``) therefore
call :func:`export_comm_env` as their first statement, before ``import
torch``; :func:`parallel.launch.init_comm` calls it again (a no-op then) and
warns when it had to set a variable in a process whose HIP runtime was
already up.

This module imports nothing heavy (no torch) so it can run first.
"""
from __future__ import annotations

import os

# name -> value; setdefault semantics (a value the user exported wins)
COMM_ENV = {
    # RCCL's intra-node transport on this platform: the host driver supports
    # dmabuf IPC only; the legacy IPC handle path fails with
    # "hipIpcGetMemHandle: invalid argument" when ranks exchange buffers
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    # the exchange buffers are persistent; without this, ProcessGroupNCCL's
    # recordStream on every collective's tensors leaves events that the
    # caching allocator then polls on each later allocation of the round loop
    "TORCH_NCCL_AVOID_RECORD_STREAMS": "1",
}


def export_comm_env(environ=None) -> list:
    """Set every COMM_ENV variable that is not already set; returns the names
    it had to set (empty when the environment already carried them)."""
    env = os.environ if environ is None else environ
    added = []
    for k, v in COMM_ENV.items():
        if k not in env:
            env[k] = v
            added.append(k)
    return added
