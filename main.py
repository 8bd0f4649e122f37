"""Experiment entry point — same sweep and artefacts as the reference's
``python main.py`` (`src/main.py:80-400`), re-built on the MI355X engine.

Loops over ``model_types x update_types x num_runs``; each combination is one
decentralised federation (``fedmse_decentralized_amd.federation``) and
appends the reference's per-round results JSONL and verification JSONL;
a ``training_summary.json`` with the best metric per combination is written
at the end.  All reference constants are CLI flags (``--help``).

Single GPU / CPU:   python main.py --synthetic nbaiot
Multi-GPU (RCCL):   python -m torch.distributed.run --nproc-per-node 8 \
                        --master-addr 127.0.0.1 main.py --synthetic nbaiot
Reference data:     python main.py --config-file /root/reference/src/Configuration/scen2-nba-iot-10clients.json
"""
from __future__ import annotations

import argparse
import logging
import sys

from fedmse_decentralized_amd.parallel.env import export_comm_env

# RCCL's transport settings reach HSA only if exported before the HIP runtime
# starts (parallel/env.py); nothing has touched the GPU yet
export_comm_env()

from fedmse_decentralized_amd.io.files import reserve_fd_table  # noqa: E402

# grow the descriptor table while the process is still single-threaded
# (io.files.reserve_fd_table: later growth waits on RCU in threaded processes)
reserve_fd_table()

import torch  # noqa: E402

from fedmse_decentralized_amd.config import ExperimentConfig, add_arguments, from_args  # noqa: E402
from fedmse_decentralized_amd.federation import Federation  # noqa: E402
from fedmse_decentralized_amd.io import reports  # noqa: E402
from fedmse_decentralized_amd.parallel.comm import LoopbackComm  # noqa: E402
from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown  # noqa: E402
from fedmse_decentralized_amd.protocol.early_stop import GlobalEarlyStop  # noqa: E402
from fedmse_decentralized_amd.utils.logging import setup_logging  # noqa: E402


def run_sweep(cfg: ExperimentConfig, comm=None) -> dict:
    log = logging.getLogger("fedmx")
    own_comm = comm is None
    if comm is None:
        dev = cfg.device
        if dev == "auto":
            dev = "cuda" if torch.cuda.is_available() else "cpu"
        comm = init_comm(device=dev, comm_impl=cfg.comm)
    total = len(cfg.update_types) * len(cfg.model_types) * cfg.num_runs
    best = {mt: {ut: float("-inf") for ut in cfg.update_types} for mt in cfg.model_types}
    log.info("\n" + "=" * 50)
    log.info("Training Parameters:")
    log.info("=" * 50)
    log.info(f"Number of runs: {cfg.num_runs}")
    log.info(f"Number of rounds per run: {cfg.num_rounds}")
    log.info(f"Epochs per round: {cfg.epoch}")
    log.info(f"Learning rate: {cfg.lr_rate}")
    log.info(f"Shrink lambda: {cfg.shrink_lambda}")
    log.info(f"Network size: {cfg.network_size}")
    log.info(f"Number of participants ratio: {cfg.num_participants}")
    log.info(f"Batch size: {cfg.batch_size}")
    log.info(f"Data seed: {cfg.data_seed}")
    log.info(f"Experiment name: {cfg.experiment_name}")
    log.info(f"Model types: {cfg.model_types}")
    log.info(f"Update types: {cfg.update_types}")
    log.info(f"Total combinations to run: {total}")
    log.info(f"Backend: {cfg.backend}  compat: {cfg.compat}  world size: {comm.world_size}")
    log.info("=" * 50 + "\n")
    early = GlobalEarlyStop(cfg.global_patience, cfg.compat)   # process-global in compat mode (Q8)
    combos = [(mt, ut, run) for mt in cfg.model_types for ut in cfg.update_types for run in range(cfg.num_runs)]
    parallel = cfg.parallel_combos and comm.world_size > 1
    results = []
    if cfg.concurrent_combos and not parallel:
        if comm.world_size > 1:
            # each concurrent federation issues its collectives from its own
            # HIP stream; the exchange channels (RCCL communicator, IPC
            # seq/parity slots) assume one ordered stream per rank
            raise SystemExit("--concurrent-combos runs every combination in ONE process on one GPU; with "
                             f"{comm.world_size} ranks use --parallel-combos (one combination per rank) instead")
        if cfg.compat != "fixed":
            raise SystemExit("--concurrent-combos needs --compat fixed (the reference's early-stop state is "
                             "shared across combinations run in sequence)")
        results = _run_concurrent(cfg, combos, comm, log)
        combos = []
    for k, (model_type, update_type, run) in enumerate(combos, start=1):
        if parallel and (k - 1) % comm.world_size != comm.rank:
            continue
        log.info(f"\nStarting combination {k}/{total}")
        log.info(f"Model type: {model_type}, Update type: {update_type}, Run: {run + 1}/{cfg.num_runs}")
        early.start_combination()
        # parallel combos: a single-rank federation on this rank's device
        fcomm = LoopbackComm(comm.device) if parallel else comm
        fed = Federation(cfg, model_type, update_type, run, comm=fcomm, early_stop=early).setup()
        m = fed.run_all()
        results.append((model_type, update_type, m))
        del fed
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    if parallel:
        results = [r for part in comm.all_gather_object(results) for r in part]
    for model_type, update_type, m in results:
        best[model_type][update_type] = max(best[model_type][update_type], m)
    log.info("\nTraining Summary:")
    log.info("=" * 50)
    for mt in cfg.model_types:
        for ut in cfg.update_types:
            log.info(f"{mt} + {ut}: Best {cfg.metric} = {best[mt][ut]:.10f}")
    log.info("=" * 50)
    if comm.is_root:
        path = reports.write_summary(cfg, best)
        log.info(f"Saved training summary to {path}")
    if own_comm:
        shutdown(comm)
    return best


def _run_concurrent(cfg: ExperimentConfig, combos, comm, log):
    """Every combination's federation at once on this process's device: each
    gets its own HIP stream and launch rings, and their rounds are issued
    round-robin, so the GPU runs several federations' kernels side by side
    (a 10-client round occupies 5 of 256 CUs) while the host prepares the
    next federation's round.  Per-combination results equal the sequential
    sweep's (independent RNG streams, separate report files)."""
    from fedmse_decentralized_amd.ops import _hip

    cuda = comm.device.type == "cuda"
    feds = []
    for k, (model_type, update_type, run) in enumerate(combos, start=1):
        log.info(f"\nStarting combination {k}/{len(combos)} (concurrent)")
        log.info(f"Model type: {model_type}, Update type: {update_type}, Run: {run + 1}/{cfg.num_runs}")
        rt = _hip.Runtime(comm.device, private=True) if cuda and cfg.backend != "torch" else None
        with _hip.use_runtime(rt):
            fed = Federation(cfg, model_type, update_type, run, comm=comm,
                             early_stop=GlobalEarlyStop(cfg.global_patience, cfg.compat))
            fed.defer_verification = True   # the run's verification file is shared: combination order
            fed.setup()
        feds.append((model_type, update_type, fed, rt))
    for _, _, fed, _ in feds:
        if getattr(fed, "_fast", None) is not None:
            fed._fast.eager_collect = False   # issue every federation's round before reading any
    active = list(range(len(feds)))
    while active:
        issued = []
        for i in active:
            _, _, fed, rt = feds[i]
            with _hip.use_runtime(rt):
                issued.append((i, fed.begin_step()))
        for i, r in issued:
            _, _, fed, rt = feds[i]
            with _hip.use_runtime(rt):
                if fed.end_step(r):
                    active.remove(i)
    results = []
    for model_type, update_type, fed, rt in feds:
        with _hip.use_runtime(rt):
            results.append((model_type, update_type, fed.conclude()))
    return results


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_arguments(p)
    ns = p.parse_args(argv)
    cfg = from_args(ns)
    import os

    setup_logging(cfg.log_level, rank=int(os.environ.get("RANK", "0")))
    run_sweep(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
