"""Multi-process decentralised federation over torch.distributed (gloo on CPU,
world size 2): every rank reaches the same protocol decisions and metrics as
a single-process run, and the parameter all-gather / score all-reduce give
bit-identical aggregates (SURVEY §4 tier T3)."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from fedmse_decentralized_amd.config import ExperimentConfig


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(out):
    return ExperimentConfig(synthetic="nbaiot", network_size=4, num_rounds=2, epoch=1, batch_size=12,
                            output_root=out, backend="torch", device="cpu", log_level="WARNING",
                            global_early_stop=False, save_checkpoints=False, compat="fixed")


def _shrink():
    from fedmse_decentralized_amd.data import synthetic

    orig = synthetic.SyntheticSpec.resolved

    def resolved(self):
        s = orig(self)
        s.normal_rows, s.abnormal_rows, s.test_normal_rows = (60, 70), (80, 90), 15
        return s
    synthetic.SyntheticSpec.resolved = resolved


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    _shrink()
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cpu")
    fed = Federation(_cfg(out), "hybrid", "mse_avg", 0, comm=comm).setup()
    rs = [fed.run_round() for _ in range(2)]
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"agg": [r.aggregator for r in rs], "sel": [r.selected for r in rs],
                   "metrics": [r.metrics.tolist() for r in rs],
                   "params": fed.engine.store.params.sum(1).tolist(), "local": fed.local}, f)
    shutdown(comm)


@pytest.mark.timeout(300)
def test_gloo_two_ranks_match_single_process(tmp_path):
    out = str(tmp_path)
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    # single-process reference
    _shrink()
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    fed = Federation(_cfg(out), "hybrid", "mse_avg", 0).setup()
    rs = [fed.run_round() for _ in range(2)]
    ref_params = fed.engine.store.params.sum(1).tolist()
    for r in range(2):
        d = json.load(open(os.path.join(out, f"rank{r}.json")))
        assert d["agg"] == [x.aggregator for x in rs]
        assert d["sel"] == [x.selected for x in rs]
        for a, b in zip(d["metrics"], rs):
            np.testing.assert_array_equal(np.array(a), b.metrics)
        loc = d["local"]
        assert d["params"] == ref_params[loc[0]:loc[-1] + 1]


def _combo_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    _shrink()
    import dataclasses

    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    sys_path = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import sys
    sys.path.insert(0, sys_path)
    import main as driver

    comm = init_comm(backend="gloo", device="cpu")
    cfg = dataclasses.replace(_cfg(out), parallel_combos=True, update_types=["avg", "fedprox", "mse_avg"],
                              model_types=["hybrid"], num_rounds=1)
    best = driver.run_sweep(cfg, comm=comm)
    with open(os.path.join(out, f"combo_rank{rank}.json"), "w") as f:
        json.dump(best, f)
    shutdown(comm)


@pytest.mark.timeout(300)
def test_parallel_combos_two_ranks(tmp_path):
    """Experiment-level parallelism: the 3 combinations split over 2 ranks give
    the same summary as running them one after another in one process."""
    out = str(tmp_path)
    mp.start_processes(_combo_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    _shrink()
    import dataclasses
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import main as driver
    from fedmse_decentralized_amd import federation

    federation._PREP_CACHE.clear()
    cfg = dataclasses.replace(_cfg(out + "/seq"), update_types=["avg", "fedprox", "mse_avg"], model_types=["hybrid"],
                              num_rounds=1)
    ref = driver.run_sweep(cfg)
    for r in range(2):
        got = json.load(open(os.path.join(out, f"combo_rank{r}.json")))
        assert got == ref
    assert os.path.exists(os.path.join(out, "Checkpoint", "Results", "Update", "4"))


def test_phantom_comm_semantics():
    """PhantomComm (single-GPU projection of rank 0 of a W-rank job): the
    all-gather repeats the local contribution, all-reduces keep local values."""
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm, PhantomComm

    c = PhantomComm(8)
    assert c.world_size == 8 and c.rank == 0 and c.is_root and c.phantom
    assert not LoopbackComm().phantom
    x = torch.arange(6, dtype=torch.float32).reshape(3, 2)
    g = c.all_gather(x)
    assert g.shape == (8, 3, 2) and g.is_contiguous()
    assert all(torch.equal(g[r], x) for r in range(8))
    v = np.arange(4, dtype=np.float64)
    np.testing.assert_array_equal(c.all_reduce_sum(v), v)
    t = x.clone()
    c.all_reduce_inplace(t)
    assert torch.equal(t, x)
    assert c.all_gather_object("h") == ["h"] * 8


def test_forced_collectives_one_rank_gloo_matches_loopback(tmp_path):
    """FEDMX_FORCE_COLLECTIVES=1 on a one-rank gloo group takes the multi-rank
    host path (pack, all-gather, all-reduce) with results identical to the
    loopback run (the CPU twin of the one-rank RCCL GPU test)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(extra_env, name):
        env = dict(os.environ, **extra_env)
        out = tmp_path / f"{name}.json"
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                            "--backend", "torch", "--epochs", "1", "--no-artifacts", "--out", str(out)],
                           env=env, cwd=root, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(out.read_text())

    base = run({}, "loopback")
    forced = run({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(_free_port()), "FEDMX_FORCE_COLLECTIVES": "1"}, "gloo1")
    assert forced["detection_auc_mean"] == base["detection_auc_mean"]
    assert forced["detection_auc_min"] == base["detection_auc_min"]


def test_comm_impl_selection(monkeypatch):
    """--comm / FEDMX_COMM: rccl or ipc only; the peer-memory path is a GPU
    multi-rank feature (a one-rank job stays on the loopback comm)."""
    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm
    from fedmse_decentralized_amd.parallel.launch import init_comm

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FEDMX_FORCE_COLLECTIVES", raising=False)
    with pytest.raises(ValueError):
        init_comm(device="cpu", comm_impl="nccl2")
    monkeypatch.setenv("FEDMX_COMM", "bogus")
    with pytest.raises(ValueError):
        init_comm(device="cpu")
    monkeypatch.setenv("FEDMX_COMM", "ipc")
    assert isinstance(init_comm(device="cpu"), LoopbackComm)
    assert isinstance(init_comm(device="cpu", comm_impl="rccl"), LoopbackComm)
    assert ExperimentConfig().comm is None


def test_fault_injection_cli_lists_are_ints():
    import argparse

    from fedmse_decentralized_amd.config import add_arguments, from_args

    ns = add_arguments(argparse.ArgumentParser()).parse_args(["--dropped-clients", "1", "3",
                                                              "--malicious-clients", "2"])
    cfg = from_args(ns)
    assert cfg.dropped_clients == [1, 3] and cfg.malicious_clients == [2]


def _edge_worker(rank, world, port, out, n_clients):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    _shrink()
    import dataclasses

    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cpu")
    cfg = dataclasses.replace(_cfg(out), network_size=n_clients, num_rounds=3, debug_replica_check=True)
    fed = Federation(cfg, "hybrid", "mse_avg", 0, comm=comm).setup()
    rs = [fed.run_round() for _ in range(3)]
    with open(os.path.join(out, f"edge{rank}.json"), "w") as f:
        json.dump({"agg": [r.aggregator for r in rs], "sel": [r.selected for r in rs],
                   "ver": [r.verification for r in rs], "metrics": [r.metrics.tolist() for r in rs],
                   "params": fed.engine.store.params.double().sum(1).tolist(), "local": fed.local}, f)
    shutdown(comm)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_clients", [10, 8, 4],
                         ids=["10-clients-over-8-ranks", "one-client-per-rank", "ranks-without-clients"])
def test_eight_ranks_edge_shapes_match_single_process(tmp_path, n_clients):
    """The shapes the first 8-GPU run meets (VERDICT r3 Next #5), as 8 gloo
    ranks on the CPU: the headline 10-client federation over 8 ranks (most
    ranks have no selected client in a round), one client per rank (BASELINE
    config 3), and 4 clients (ranks hosting no client at all).  Every rank
    must reach the single-process federation's selections, aggregators,
    verification results and AUCs, and hold its shard's parameters exactly."""
    out = str(tmp_path)
    mp.start_processes(_edge_worker, args=(8, _free_port(), out, n_clients), nprocs=8, join=True,
                       start_method="spawn")
    _shrink()
    import dataclasses

    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    cfg = dataclasses.replace(_cfg(out + "/single"), network_size=n_clients, num_rounds=3)
    fed = Federation(cfg, "hybrid", "mse_avg", 0).setup()
    rs = [fed.run_round() for _ in range(3)]
    ref_params = fed.engine.store.params.double().sum(1).tolist()
    hosting = 0
    for r in range(8):
        d = json.load(open(os.path.join(out, f"edge{r}.json")))
        assert d["sel"] == [x.selected for x in rs]
        assert d["agg"] == [x.aggregator for x in rs]
        assert d["ver"] == [x.verification for x in rs]
        for a, b in zip(d["metrics"], rs):
            np.testing.assert_array_equal(np.array(a), b.metrics)
        loc = d["local"]
        hosting += bool(loc)
        assert d["params"] == (ref_params[loc[0]:loc[-1] + 1] if loc else [])
    assert hosting == min(8, n_clients)


def test_ipc_wait_grid_fits_the_device():
    """Round 5's intermittent IPC self-test failure (VERDICT r5 Next #4a):
    8 ranks sharing one GPU, 64 chunks per source, put 8 x 8 x 64 = 4,096
    spinning wait workgroups on a device that holds ~2,048, so the peers'
    push kernels could not run.  The chunk cap keeps every co-located rank's
    wait grid together within WAIT_WORKGROUP_BUDGET; a rank alone on its GPU
    keeps the full chunk count."""
    from fedmse_decentralized_amd.parallel.ipc import WAIT_WORKGROUP_BUDGET, wait_chunk_cap

    assert wait_chunk_cap(8, 1, 64) == 64          # 8-GPU node: one rank per device
    for world, share in [(8, 8), (4, 4), (2, 2), (16, 16), (8, 4)]:
        c = wait_chunk_cap(world, share, 64)
        assert c >= 1 and world * c * share <= WAIT_WORKGROUP_BUDGET, (world, share, c)
    assert wait_chunk_cap(8, 8, 64) == 16
    assert wait_chunk_cap(16, 16, 64) == 4
