"""Does the side-stream evaluation slow the training kernel it overlaps?
Runs the headline federation (bench.py's config) for R rounds; with
--no-eval the per-round evaluation launch is replaced by a no-op (training,
votes, elections and verification are unaffected: evaluation only feeds the
reports).  Compare the training kernel's per-call durations of the two runs
under rocprofv3 (same seeds -> same selections and local epochs).
Diagnostic only."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--no-eval", action="store_true")
    a = p.parse_args()
    import torch

    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("WARNING")
    cfg = ExperimentConfig(num_participants=0.5, epoch=5, num_rounds=10 ** 9, lr_rate=1e-3, shrink_lambda=5.0,
                           network_size=10, batch_size=12, model_types=["hybrid"], update_types=["mse_avg"],
                           synthetic="nbaiot", synthetic_iid=True, compat="fixed", backend="auto",
                           global_early_stop=False, save_checkpoints=False,
                           output_root=tempfile.mkdtemp(prefix="fedmx_diag_"), log_level="WARNING")
    fed = Federation(cfg, "hybrid", "mse_avg", run=0, write_reports=False).setup()
    if a.no_eval:
        fed.engine.evaluate_launch = lambda *args, **kw: None
    for _ in range(a.rounds):
        fed.run_round()
    fed.finish()
    torch.cuda.synchronize()
    print("done", a.rounds, "rounds, eval", not a.no_eval)


if __name__ == "__main__":
    main()
