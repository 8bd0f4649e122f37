"""Flagship benchmark: federated rounds/sec + detection AUC of the 10-client
SAE-CEN FedMSE scenario on N-BaIoT-shaped data (BASELINE.json), 1..8 MI355X.

One timed *step* = one complete decentralised round, exactly the reference's
round (`src/main.py:267-365`): client selection (50 %), local training of the
selected clients (5 epochs, batch 12, Adam lr 1e-3, shrink lambda 5, patience 1,
validation every epoch), MSE-scored aggregator election, FedMSE aggregation
(dev-set MSE weights), broadcast + verification by every other client,
SAE-CEN evaluation (ROC-AUC) of every client, results/verification JSONL and
per-client model.cpt / training_tracking.pkl artefacts.

Multi-GPU (N > 1, one process per GPU).  ``value`` is ALWAYS the
10-client federation's rounds/s, the BASELINE metric's named configuration:
at N > 1 its 10 clients are sharded over the N ranks (BASELINE config 4's
shape; strong scaling), with vote scores, FedMSE weights and AUCs exchanged
by RCCL all-reduce and the selected models by an RCCL all-gather over xGMI.
No x N factor is applied: five trained clients occupy 5 of one GPU's 256 CUs,
so sharding them can only add exchange latency, and the curve shows that.
Two further measurements ride along in their own fields, never folded into
``value``:
  * ``weak_scaling`` – ONE decentralised federation of 10*N clients (10 per
    GPU; the reference's 10/15/20/50-client network-scale configs
    generalised): its rounds/s and AUC;
  * ``independent_federations`` – N concurrent one-GPU 10-client federations,
    one per rank with its own seed, no collectives (experiment-level
    parallelism: the reference's runs loop, `src/main.py:108-110`): the
    aggregate rounds/s of the job.
``--clients C`` / ``--clients-per-gpu K`` choose another headline federation
(C clients, or K*N clients) — e.g. ``--clients-per-gpu 1`` is BASELINE
config 3 (8 clients, one per GPU).

Data: synthetic N-BaIoT-shaped tabular data (115 features, per-client sizes of
the shipped IID-10 split) with random-init weights of the reference
architecture — there is no network access for the real dataset.  Compute is
fp32 end to end (the reference's dtype).  ``vs_baseline`` divides by the
reference's best measured round rate, 0.30 rounds/s.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

from fedmse_decentralized_amd.parallel.env import export_comm_env

# RCCL's transport settings reach HSA only if exported before the HIP runtime
# starts (parallel/env.py): first statement, before torch is imported
export_comm_env()

from fedmse_decentralized_amd.io.files import reserve_fd_table  # noqa: E402

# grow the descriptor table while the process is still single-threaded
# (io.files.reserve_fd_table: later growth waits on RCU in threaded processes)
reserve_fd_table()

import numpy as np  # noqa: E402
import torch  # noqa: E402

BASELINE_ROUNDS_PER_SEC = 0.30
METRIC = "rounds/sec + detection AUC, 10-client SAE (N-BaIoT shape) at 1/2/4/8 MI355X"
EPISODE = 20   # paper schedule: 20 rounds per run; aggregation caps reset per episode


def _collectives_label(comm) -> str:
    """What carries the per-round exchange: RCCL (torch.distributed "nccl"
    on ROCm), gloo, or nothing (one rank: in-process loopback).  "xGMI" only
    when several ranks sit on distinct GPUs (launch.collective_self_test)."""
    if type(comm).__name__ == "PhantomComm":
        return "collectives stubbed: one-GPU projection of rank 0"
    if getattr(comm, "world_size", 1) <= 1:
        link = "one rank"
    else:
        link = "over xGMI" if getattr(comm, "devices_distinct", False) else "ranks share one GPU"
    if getattr(comm, "active", False):
        return f"peer-memory one-shot all-gather/all-reduce (IPC, {link})"
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            b = dist.get_backend()
            if b == "nccl":
                return f"RCCL all-gather/all-reduce ({link})"
            return f"{b} all-gather/all-reduce"
    except Exception:
        pass
    return "in-process loopback; RCCL all-gather/all-reduce at N > 1"


def _spawn_ranks(n: int, argv) -> int:
    """``python bench.py --gpus N`` without a launcher: start N rank processes
    through torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) and
    return their exit code.  Runs before this process touches the GPU; the
    children inherit stdout, so rank 0's JSON line is this command's output."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)   # carries COMM_ENV (exported at import)
    return subprocess.run(cmd, env=env).returncode


# transport probe outcome of this rank (parallel/probe.py): the record's
# ``transport_fallback`` when the requested transport did not work
_TRANSPORT = {"used": None, "fallback": None}


def _probe_wanted(known) -> bool:
    """A torch.distributed.run rank of a GPU job (FEDMX_BENCH_PROBE=1 forces
    the probe on the CPU too, =0 skips it).  device_count() does not start
    the HIP runtime."""
    flag = os.environ.get("FEDMX_BENCH_PROBE", "auto")
    if flag == "0" or int(os.environ.get("WORLD_SIZE", "1")) <= 1 or known.phantom_ranks > 1:
        return False
    if "TORCHELASTIC_USE_AGENT_STORE" not in os.environ:   # no launcher store to agree through
        return False
    return flag == "1" or torch.cuda.device_count() > 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    from fedmse_decentralized_amd.parallel import probe

    if argv[:1] == [probe.PROBE_FLAG]:   # a probe child (parallel/probe.py)
        return probe.child_main(argv[1])
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    pre.add_argument("--phantom-ranks", type=int, default=0)
    pre.add_argument("--comm", default=None)
    known, _ = pre.parse_known_args(argv)
    if known.gpus > 1 and "WORLD_SIZE" not in os.environ and known.phantom_ranks <= 1:
        return _spawn_ranks(known.gpus, argv)
    if _probe_wanted(known):
        # before this process touches the GPU: the first transport that works
        # on every rank (RCCL, else peer-memory IPC, else gloo)
        requested = probe.requested_transport(known.comm)
        used, fb = probe.choose_transport(os.path.abspath(__file__), requested,
                                          timeout_s=float(os.environ.get("FEDMX_PROBE_TIMEOUT_S", "180")))
        probe.apply_env(os.environ, used)
        _TRANSPORT["used"], _TRANSPORT["fallback"] = used, fb
        if fb is not None and os.environ.get("RANK") == "0":
            print(f"transport fallback: {requested} -> {used}: {fb['failures']}", file=sys.stderr)
    # stdout carries exactly ONE line, the JSON record: native libraries'
    # chatter (RCCL prints a version banner to stdout when a communicator is
    # created) is routed to stderr for the duration of the run
    sys.stdout.flush()
    real_stdout = os.dup(1)
    os.dup2(2, 1)
    try:
        return _main(argv, real_stdout)
    finally:
        sys.stdout.flush()
        os.dup2(real_stdout, 1)
        os.close(real_stdout)


def _measure(fed, comm, device, steps: int, warmup: int, profile):
    """Warm-up rounds, then exactly ``steps`` timed rounds bracketed by a
    barrier + device synchronisation on both sides; every report and artefact
    of the timed rounds is written before the clock stops.  Returns (seconds,
    max over ranks; the last RoundResult; per-rank training-launch ms of the
    timed rounds [ranks, steps] when timed, else None)."""
    def one_round():
        if fed.round_idx and fed.round_idx % EPISODE == 0:
            fed.reset_aggregation_counts()   # new 20-round episode (fresh protocol counters)
        return fed.run_round()

    for _ in range(warmup):
        one_round()
    fed.finish()
    fed.writer.flush()
    comm.barrier()
    if device == "cuda":
        torch.cuda.synchronize()
    prof = None
    if profile and comm.is_root:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    fed.tel.reset_totals()   # phase totals cover the timed rounds only
    fed.writer.mark()
    r0 = fed.round_idx
    t0 = time.perf_counter()
    last = None
    results = []
    for _ in range(steps):
        last = one_round()
        results.append(last)
    fed.finish()         # device-protocol rounds: collect results, hand reports to the writer
    fed.writer.flush()   # artefacts of the timed rounds are on disk before the clock stops
    if prof is not None:
        prof.disable()
        import io
        import pstats

        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
        with open(profile, "w") as f:
            f.write(s.getvalue())
    comm.barrier()
    if device == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the job is as slow as its slowest rank
    allt = comm.all_gather(torch.tensor([dt], dtype=torch.float64))
    dt = float(allt.max())
    train_ms = None
    fr = getattr(fed, "_fast", None)
    if fr is not None and getattr(fr, "train_timing", False):
        mine = torch.tensor([fr.train_ms.get(r, 0.0) for r in range(r0, r0 + steps)], dtype=torch.float64)
        train_ms = comm.all_gather(mine).reshape(comm.world_size, steps).numpy()
    # local epochs the trained clients actually ran in the timed rounds
    # (validation early stopping, patience 1): the work behind ms_per_step
    # (read after the clock: the device-protocol rounds are collected by now)
    ep = [0.0, 0.0]
    for res in results:
        e = getattr(res, "epochs_run", None) or {}
        ep[0] += float(sum(e.values()))
        ep[1] += float(len(e))
    tot = comm.all_gather(torch.tensor(ep, dtype=torch.float64)).reshape(comm.world_size, 2).sum(0)
    epochs_mean = float(tot[0] / tot[1]) if float(tot[1]) > 0 else None
    return dt, last, train_ms, epochs_mean


def _auc(last, fed=None, phantom=False):
    """(mean, min) detection AUC over the federation's clients after the last
    timed round.  A phantom rank only ever evaluates its own clients (the AUC
    all-reduce is stubbed): those, not the zero-filled others."""
    if last is None:
        return float("nan"), float("nan")
    m = np.asarray(last.metrics, dtype=np.float64)
    if phantom and fed is not None and fed.local:
        m = m[fed.local[0]:fed.local[-1] + 1]
    m = m[~np.isnan(m)]   # (a client without abnormal test rows has no AUC)
    return (float(np.mean(m)), float(np.min(m))) if m.size else (float("nan"), float("nan"))


def distinct_devices(comm) -> int:
    """Number of distinct physical GPUs the job's ranks run on (the collective
    self-test's device identities; ranks sharing one GPU count once)."""
    if getattr(comm, "world_size", 1) <= 1:
        return 1
    ids = getattr(comm, "peer_devices", None)
    if ids is None:
        from fedmse_decentralized_amd.parallel.launch import _device_identity

        ids = comm.all_gather_object(_device_identity(comm.device))
    return len({tuple(i) for i in ids})


def _extra_fields(rec, build, fed, comm, device, args, n_gpus, dt, auc, auc_min):
    """N > 1 fields beside the headline (VERDICT r3 Next #1): ``weak_scaling``
    (one federation of 10 clients per GPU) and ``independent_federations``
    (every rank its own one-GPU 10-client federation).  Never multiplied into
    ``value``."""
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm

    # (a) weak scaling: one federation of 10 clients per GPU
    if fed.N != 10 * n_gpus:
        fw = build(10 * n_gpus)
        dtw, lastw, _, _ = _measure(fw, comm, device, args.steps, args.warmup, None)
        aw, aw_min = _auc(lastw)
        fw.finish()
        del fw
    else:
        dtw, aw, aw_min = dt, auc, auc_min
    # (b) experiment-level parallelism: every rank its own one-GPU 10-client
    # federation (run index = rank, i.e. its own seeds), no collectives;
    # the job's clock is the slowest rank's, as for the headline
    fi = build(10, fcomm=LoopbackComm(comm.device), run=comm.rank)
    dti, lasti, _, _ = _measure(fi, comm, device, args.steps, args.warmup, None)
    ai = comm.all_gather(torch.tensor(_auc(lasti), dtype=torch.float64)).reshape(n_gpus, 2).numpy()
    fi.finish()
    if rec is not None:
        rec["weak_scaling"] = {
            "clients": 10 * n_gpus,
            "federation_rounds_per_sec": round(args.steps / dtw, 4),
            "ms_per_step": round(1e3 * dtw / args.steps, 4),
            "detection_auc_mean": round(aw, 6),
            "detection_auc_min": round(aw_min, 6),
            "note": "ONE federation of 10 clients per GPU; rounds/s of that larger federation (not x N)"}
        rec["independent_federations"] = {
            "federations": n_gpus,
            "clients_each": 10,
            "aggregate_rounds_per_sec": round(n_gpus * args.steps / dti, 4),
            "per_federation_rounds_per_sec": round(args.steps / dti, 4),
            "ms_per_step": round(1e3 * dti / args.steps, 4),
            "detection_auc_mean": round(float(ai[:, 0].mean()), 6),
            "detection_auc_min": round(float(ai[:, 1].min()), 6),
            "note": ("N concurrent one-GPU 10-client federations (run r on rank r, as the reference's "
                     "runs loop src/main.py:108-110); aggregate = N x steps / slowest rank's time")}


def _main(argv, real_stdout: int):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--clients", type=int, default=None,
                   help="headline federation size (default 10: BASELINE's 10-client federation at every N)")
    p.add_argument("--clients-per-gpu", type=int, default=None,
                   help="headline = ONE federation of K x N clients (weak scaling; K=1 is BASELINE config 3)")
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--shrink-lambda", type=float, default=5.0)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=12)
    p.add_argument("--model-type", default="hybrid")
    p.add_argument("--update-type", default="mse_avg")
    p.add_argument("--backend", default="auto")
    p.add_argument("--comm", default=None, choices=["rccl", "ipc"],
                   help="N > 1: per-round collectives over RCCL (default) or one-shot peer-memory kernels "
                        "(parallel/ipc.py); default: FEDMX_COMM or rccl")
    p.add_argument("--data-kind", default="nbaiot", choices=["nbaiot", "kitsune"],
                   help="synthetic feature family (BASELINE config 5 uses kitsune, non-IID)")
    p.add_argument("--non-iid", action="store_true", help="Dirichlet non-IID client mixtures")
    p.add_argument("--compat", default="fixed")
    p.add_argument("--init-mode", default="auto", choices=["auto", "shared", "per_client"],
                   help="initial client models (auto: shared under compat fixed, see config.init_mode)")
    p.add_argument("--no-artifacts", action="store_true", help="skip model.cpt/tracking/JSONL writes")
    p.add_argument("--trace", default=None, help="per-phase JSONL trace (adds device syncs)")
    p.add_argument("--out", default=None, help="also write the JSON line to this file")
    p.add_argument("--profile", default=None, help="cProfile the timed rounds (rank 0) into this file")
    p.add_argument("--phantom-ranks", type=int, default=0,
                   help="projection on ONE GPU: run rank 0 of a W-rank weak-scaling job (10 clients per rank) "
                        "with the collectives stubbed out (parallel.comm.PhantomComm); labelled as a projection")
    p.add_argument("--no-extra", action="store_true",
                   help="N > 1: skip the weak_scaling and independent_federations measurements")
    args = p.parse_args(argv)
    if args.clients is not None and args.clients_per_gpu is not None:
        p.error("--clients and --clients-per-gpu are exclusive")

    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown
    from fedmse_decentralized_amd.utils.logging import setup_logging

    device = "cuda" if torch.cuda.is_available() else "cpu"
    phantom = args.phantom_ranks > 1
    if phantom:
        from fedmse_decentralized_amd.parallel.comm import PhantomComm

        comm = PhantomComm(args.phantom_ranks, device)
    else:
        # (a probed job: the transport the probe settled on, exported in FEDMX_COMM)
        comm = init_comm(device=device, comm_impl=None if _TRANSPORT["used"] else args.comm)
    setup_logging("WARNING", rank=comm.rank)
    n_gpus = comm.world_size
    if args.gpus != n_gpus and comm.is_root:
        print(f"note: --gpus {args.gpus} but world size is {n_gpus}; using the world size", file=sys.stderr)
    # GPUs actually used: ranks that share a device (one-box rehearsals) count once
    n_dev = 1 if phantom else distinct_devices(comm)
    out_root = tempfile.mkdtemp(prefix="fedmx_bench_") if comm.is_root else tempfile.mkdtemp(prefix="fedmx_bench_r")

    def build(network_size: int, fcomm=comm, run: int = 0):
        cfg = ExperimentConfig(
            num_participants=0.5, epoch=args.epochs, num_rounds=10 ** 9, lr_rate=args.lr,
            shrink_lambda=args.shrink_lambda, network_size=network_size, batch_size=args.batch_size,
            model_types=[args.model_type], update_types=[args.update_type],
            synthetic=args.data_kind, synthetic_iid=not args.non_iid, compat=args.compat, backend=args.backend,
            global_early_stop=False, save_checkpoints=not args.no_artifacts,
            output_root=os.path.join(out_root, f"fed{network_size}_run{run}"),
            trace_file=args.trace, log_level="WARNING", init_mode=args.init_mode)
        fed = Federation(cfg, args.model_type, args.update_type, run=run, comm=fcomm,
                         write_reports=not args.no_artifacts).setup()
        if phantom and fed._fast is None:
            # the host protocol reads other ranks' vote records, which a phantom job does not have
            raise SystemExit("--phantom-ranks needs the device-resident round protocol (HIP engine, compat fixed)")
        return fed

    # the headline federation: BASELINE's 10 clients unless asked otherwise;
    # a phantom projection is of the weak-scaling job (10 clients per rank)
    if phantom:
        clients, scaling = 10 * args.phantom_ranks, "weak"
    elif args.clients_per_gpu is not None:
        clients, scaling = args.clients_per_gpu * n_gpus, "weak"
    else:
        clients, scaling = (args.clients or 10), "strong"
    fed = build(clients)
    # N > 1: time every rank's training launch (HIP events around it), so the
    # cost of waiting for the slowest rank's largest client is measured
    time_train = n_gpus > 1 and fed._fast is not None
    if time_train:
        fed._fast.train_timing = True
    dt, last, train_ms, epochs_mean = _measure(fed, comm, device, args.steps, args.warmup, args.profile)
    fed_rps = args.steps / dt
    auc, auc_min = _auc(last, fed, phantom)
    rec = None
    if comm.is_root:
        rec = {
            "metric": METRIC,
            "value": None if phantom else round(fed_rps, 4),
            "unit": f"rounds/s of one {fed.N}-client federation (whole job, {n_gpus} rank(s) on {n_dev} GPU(s))",
            "n_gpus": n_dev,
            "world_size": 1 if phantom else n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None if phantom else round(fed_rps / BASELINE_ROUNDS_PER_SEC, 2),
            "dtype": "fp32",
            "data": (f"synthetic ({'N-BaIoT' if args.data_kind == 'nbaiot' else 'Kitsune'}-shaped, 115 features, "
                     f"{'non-IID (Dirichlet)' if args.non_iid else 'IID'} client mixtures, "
                     f"{'IID-10 client sizes' if not args.non_iid else 'Dirichlet client sizes'}); "
                     "random-init weights"),
            "config": {
                "model": f"SAE 115-27-7-27-115 ({args.model_type}, {args.update_type}), {fed.N} clients",
                "global_batch": args.batch_size,
                "seq_len": 115,
                "parallelism": f"client-sharded x{n_gpus} ({_collectives_label(comm)})",
                "clients": fed.N,
                "participation": 0.5,
                "local_epochs": args.epochs,
                "backend": fed.engine.name,
                "compat": args.compat,
                # the shared initial model (compat fixed default since r3) changes
                # AUC and epochs run vs per_client records: compare like with like
                "init_mode": fed.cfg.resolved_init_mode(),
                "device_protocol": fed._fast is not None,
            },
            "federation_rounds_per_sec": round(fed_rps, 4),
            # of config.local_epochs: clients stop early once their validation
            # loss stops improving (patience 1), so the work per round varies
            "local_epochs_run_mean": None if epochs_mean is None else round(epochs_mean, 3),
            "detection_auc_mean": round(auc, 6),
            "detection_auc_min": round(auc_min, 6),
            "phase_ms_total": {k: round(v, 3) for k, v in fed.tel.summary().items()},
            "timed_ms": round(1e3 * dt, 3),
            "writer_busy_ms_per_round": round(1e3 * fed.writer.busy_s_timed / args.steps, 4),
        }
        if _TRANSPORT["used"] is not None:
            rec["config"]["transport"] = _TRANSPORT["used"]
        if _TRANSPORT["fallback"] is not None:
            rec["transport_fallback"] = _TRANSPORT["fallback"]
        if train_ms is not None:
            t = train_ms                       # [ranks, timed rounds], 0 = no local selection
            own = t[t > 0]
            rmax = t.max(axis=0)
            rec["train_launch_ms"] = {
                "rank_mean": round(float(own.mean()), 4) if own.size else None,
                "round_max_mean": round(float(rmax.mean()), 4),
                "per_rank_mean": [round(float(r[r > 0].mean()), 4) if (r > 0).any() else None for r in t],
                "note": "HIP-event time of each rank's fused training launch; a round waits for round_max",
            }
        if phantom:
            # a one-GPU projection, not a multi-GPU measurement: n_gpus stays 1
            # and the whole-job figure goes to projected_value
            rec["projected_ranks"] = args.phantom_ranks
            rec["projected_value"] = round(fed_rps, 4)
            rec["detection_auc_scope"] = "rank-0 clients only"
            rec["projection"] = (f"rank 0 of a {args.phantom_ranks}-rank job on ONE GPU, collectives stubbed "
                                 "(no RCCL time); projected_value assumes every rank is as fast as this one")
    import threading

    emit_lock, emitted = threading.Lock(), []

    def emit(r):
        # once per job: the extras' watchdog and the main thread may both get here
        with emit_lock:
            if emitted:
                return
            line = json.dumps(r)
            emitted.append(line)
        os.write(real_stdout, (line + "\n").encode())
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")

    if n_gpus > 1 and not phantom and not args.no_extra:
        fed.finish()
        # The headline must not depend on the extras: a rank that raises in
        # them leaves the others blocked in a collective.  Every rank arms a
        # watchdog; when it fires, rank 0 prints the headline (marked) and
        # every rank leaves, so the launcher sees the job end.
        # (the 8-rank extras took < 150 s with all ranks sharing ONE GPU: 300 s is
        # ample on a node and keeps a stuck job well inside a driver time limit)
        limit = float(os.environ.get("FEDMX_BENCH_EXTRA_TIMEOUT_S", "300"))

        def _give_up():
            # (the main thread may be adding extra fields to rec meanwhile:
            # emit a copy, and leave whatever happens -- the job must end)
            try:
                if rec is not None:
                    for _ in range(3):
                        try:
                            r = dict(rec)
                            break
                        except RuntimeError:   # (rec changed size while copied)
                            time.sleep(0.01)
                    r["extra_fields_error"] = f"extras did not finish within {limit:.0f} s (a rank failed or hung)"
                    emit(r)
                print(f"rank {comm.rank}: extra measurements timed out; exiting", file=sys.stderr, flush=True)
            finally:
                # status 0: the headline line above is complete and valid on its own
                os._exit(0)

        watchdog = threading.Timer(limit, _give_up)
        watchdog.daemon = True
        watchdog.start()
        try:
            if os.environ.get("FEDMX_BENCH_TEST_STALL_RANK") == str(comm.rank):   # tests: a stuck rank
                time.sleep(3600)
            _extra_fields(rec, build, fed, comm, device, args, n_gpus, dt, auc, auc_min)
        except Exception as e:   # the headline stands on its own: record why the extras are missing
            print(f"rank {comm.rank}: extra measurements failed: {e!r}", file=sys.stderr)
            if rec is not None:
                rec["extra_fields_error"] = repr(e)[:300]
        watchdog.cancel()
    if rec is not None:
        emit(rec)
    fed.writer.report_stats()   # FEDMX_WRITER_STATS=1: per-job writer times on stderr
    shutdown(comm)
    return 0


if __name__ == "__main__":
    sys.exit(main())
