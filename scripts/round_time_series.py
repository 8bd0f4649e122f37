"""Steady-state round time over a long run (mean ms per block of rounds,
asynchronous rounds: the host enqueues ahead, so block means reflect the
pipeline's throughput).  Same federation as bench.py."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, default=64)
    p.add_argument("--rounds", type=int, default=60)
    p.add_argument("--block", type=int, default=5)
    p.add_argument("--data-kind", default="kitsune")
    p.add_argument("--non-iid", action="store_true")
    p.add_argument("--no-artifacts", action="store_true")
    p.add_argument("--profile-rounds", type=int, default=0, help="cProfile the first N rounds (stderr)")
    a = p.parse_args(argv)
    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("WARNING")
    cfg = ExperimentConfig(num_participants=0.5, epoch=5, num_rounds=10 ** 9, lr_rate=1e-3, shrink_lambda=5.0,
                           network_size=a.clients, batch_size=12, model_types=["hybrid"], update_types=["mse_avg"],
                           synthetic=a.data_kind, synthetic_iid=not a.non_iid, compat="fixed", backend="auto",
                           global_early_stop=False, save_checkpoints=not a.no_artifacts,
                           output_root=tempfile.mkdtemp(prefix="fedmx_ts_"), log_level="WARNING")
    fed = Federation(cfg, "hybrid", "mse_avg", run=0, write_reports=not a.no_artifacts).setup()
    prof = None
    if a.profile_rounds:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    ts = [time.perf_counter()]
    for r in range(a.rounds):
        if prof is not None and r == a.profile_rounds:
            prof.disable()
            import pstats

            pstats.Stats(prof, stream=sys.stderr).sort_stats("cumtime").print_stats(25)
            prof = None
        if r and r % 20 == 0:
            fed.reset_aggregation_counts()
        fed.run_round()
        ts.append(time.perf_counter())
    fed.finish()
    fed.writer.flush()
    torch.cuda.synchronize()
    ts.append(time.perf_counter())
    d = np.diff(ts[:-1]) * 1e3
    blocks = [round(float(d[i:i + a.block].mean()), 3) for i in range(0, len(d), a.block)]
    print(json.dumps({"clients": a.clients, "ms_per_round_by_block": blocks, "block": a.block,
                      "total_s": round(ts[-1] - ts[0], 3)}))


if __name__ == "__main__":
    main()
