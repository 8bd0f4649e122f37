"""Global (round-level) early stopping (`src/main.py:55-57`, `:357-365`).

``compat="reference"`` reproduces SURVEY Q8: the state is process-global and
never reset between sweep combinations, and the *minimum client AUC* is
compared with ``<`` as if it were a loss, so later combinations typically stop
after one or two rounds (observed in `src/run21.log:2407`).  ``compat="fixed"``
resets per combination and treats the metric as higher-is-better.
"""
from __future__ import annotations

import logging

log = logging.getLogger("fedmx")


class GlobalEarlyStop:
    def __init__(self, patience: int = 1, compat: str = "reference"):
        self.patience = patience
        self.compat = compat
        self.reset_all()

    def reset_all(self):
        self.best = float("inf") if self.compat == "reference" else float("-inf")
        self.worse = 0

    def start_combination(self):
        if self.compat != "reference":
            self.reset_all()

    def update(self, metric: float) -> bool:
        """Returns True if training should stop."""
        improved = metric < self.best if self.compat == "reference" else metric > self.best
        if improved:
            self.best = metric
            self.worse = 0
            return False
        self.worse += 1
        if self.worse > self.patience:
            log.info("Early stopping in global round!")
            return True
        return False
