"""Replay of the reference's torch-RNG consumption (compat mode).

The reference's only protocol decision that depends on the torch RNG is the
+-0.01 % tie-break noise on vote scores (``torch.rand(1)`` in
``calculate_mse_score``, `src/Trainer/client_trainer.py:243-245`, SURVEY
Q17).  Its value depends on every earlier draw from the global CPU
generator, which the reference consumes as a side effect of (SURVEY
Appendix C):

* model construction (``nn.Linear`` default init + ``uniform_`` overwrite),
  once per client at setup and once per ``ModelVerifier._evaluate_model``
  call (`src/Trainer/model_verifier.py:88-91`, Q16);
* one ``int64.random_()`` per DataLoader iterator creation (every train and
  valid epoch loop, every evaluator loop);
* ``torch.rand(1)`` per vote/MSE score.

Our kernels replace all of that work, so in ``--compat reference`` mode this
class advances a private copy of the generator by exactly the same draws,
which makes client selection, elections and hence the whole protocol
trajectory reproduce the reference for the same seeds.
"""
from __future__ import annotations

import torch

from ..models.layout import ModelDims, DEFAULT_DIMS


class TorchRngReplay:
    def __init__(self, state: torch.Tensor, dims: ModelDims = DEFAULT_DIMS):
        self.state = state.clone()
        self.dims = dims
        self.draws = 0

    def _run(self, fn):
        from ..models.reference import GLOBAL_RNG_LOCK

        with GLOBAL_RNG_LOCK, torch.random.fork_rng(devices=[]):
            torch.set_rng_state(self.state)
            out = fn()
            self.state = torch.get_rng_state()
        return out

    def iterators(self, n: int) -> None:
        if n <= 0:
            return

        def f():
            for _ in range(int(n)):
                torch.empty((), dtype=torch.int64).random_()
        self._run(f)
        self.draws += int(n)

    def rand_n(self, n: int):
        import numpy as np

        return np.array([self.rand() for _ in range(n)], dtype=np.float64)

    def rand(self) -> float:
        self.draws += 1
        return float(self._run(lambda: torch.rand(1).item()))

    def model_inits(self, n: int) -> None:
        if n <= 0:
            return
        from ..models.reference import ReferenceSAE

        def f():
            for _ in range(int(n)):
                ReferenceSAE(self.dims, shrink_lambda=0.0)
        self._run(f)
        self.draws += int(n)


class HostNoise:
    """Fixed-mode tie-break noise from a seeded numpy generator."""

    def __init__(self, seed: int):
        import numpy as np

        self.rng = np.random.Generator(np.random.PCG64(seed))

    def iterators(self, n: int) -> None:
        pass

    def model_inits(self, n: int) -> None:
        pass

    def rand(self) -> float:
        return float(self.rng.random())

    def get_state(self):
        """PCG64 state as plain ints (resume snapshots load with weights_only)."""
        st = self.rng.bit_generator.state
        return [int(st["state"]["state"]), int(st["state"]["inc"]), int(st["has_uint32"]), int(st["uinteger"])]

    def set_state(self, s) -> None:
        state, inc, has32, uint = (int(x) for x in s)
        self.rng.bit_generator.state = {"bit_generator": "PCG64", "state": {"state": state, "inc": inc},
                                        "has_uint32": has32, "uinteger": uint}

    def rand_n(self, n: int):
        """``n`` draws at once: the same values, in the same order, as ``n``
        calls of :meth:`rand` (one vectorised call: the k(k-1) election draws
        of an 80-client round cost 0.6 ms of host time one by one)."""
        return self.rng.random(n)
