"""Peer-memory exchange (parallel/ipc.py, ops/csrc/hip/fedmx_ipc.hip) on one
GPU: several processes share the card (gloo for bring-up, FEDMX_DEVICE_INDEX=0),
each opens the others' receive areas through hipIpcOpenMemHandle, and the
one-shot all-gather / all-reduce kernels are checked against the values every
rank contributed; a federation run over them matches the single-process run
bit for bit.  (Cross-GPU xGMI transfers need the multi-GPU node.)"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FEDMX_DEVICE_INDEX="0", HSA_ENABLE_IPC_MODE_LEGACY="0",
                      FEDMX_IPC_TIMEOUT_S="20")


def _contrib(rank, it, n):
    g = np.random.default_rng(1000 * it + rank)
    return g.standard_normal(n).astype(np.float32)


def _exchange_worker(rank, world, port, out):
    _env(rank, world, port)
    from fedmse_decentralized_amd.ops import _hip
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cuda", comm_impl="ipc")
    dev = comm.device
    _hip.runtime(dev)
    P = 9216
    slots = 5
    ok_setup = comm.setup_exchange((slots + 1) * P, 4 * 10 * world)
    res = dict(active=ok_setup, gather=[], reduce=[])
    side = torch.cuda.Stream(device=dev)
    send = torch.zeros((slots + 1) * P, device=dev)
    allg = torch.zeros(world * (slots + 1) * P, device=dev)
    for it in range(7):
        rows = 1 + (it % (slots + 1))          # prefixes of the persistent buffers, as the round does
        n = rows * P
        send[:n].copy_(torch.from_numpy(_contrib(rank, it, n)))
        got = allg[:world * n].view(world, n)
        comm.all_gather_into(got, send[:n])
        exp = np.stack([_contrib(r, it, n) for r in range(world)])
        torch.cuda.synchronize(dev)
        res["gather"].append(bool(np.array_equal(got.cpu().numpy(), exp)))
        # the reduce on a second stream, as the evaluation stream does
        m = 2 * 10 * world
        t = torch.zeros(m, dtype=torch.float64, device=dev)
        blk = m // world
        vals = np.arange(blk, dtype=np.float64) * (it + 1) + 0.25 * rank
        with _hip.on_stream(side):
            t[rank * blk:(rank + 1) * blk].copy_(torch.from_numpy(vals))
            comm.all_reduce_inplace(t)
        side.synchronize()
        exp_r = np.concatenate([np.arange(blk, dtype=np.float64) * (it + 1) + 0.25 * r for r in range(world)])
        res["reduce"].append(bool(np.array_equal(t.cpu().numpy(), exp_r)))
    res["calls"] = comm.ipc_calls
    res["status_ok"] = comm.status_ok()
    with open(os.path.join(out, f"x{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown(comm)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_ipc_exchange_kernels(tmp_path, world):
    mp.start_processes(_exchange_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        d = json.load(open(tmp_path / f"x{r}.json"))
        assert d["active"], d
        assert all(d["gather"]) and all(d["reduce"]), d
        assert d["calls"] == 14 and d["status_ok"]


def _fed_worker(rank, world, port, out, network_size=6):
    _env(rank, world, port)
    from test_device_protocol_gpu import _cfg, _run, _shrink

    _shrink()
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cuda", comm_impl="ipc")
    fed, res = _run(_cfg(os.path.join(out, f"r{rank}"), save_checkpoints=False, debug_replica_check=True,
                         network_size=network_size), "mse_avg", 4, comm=comm)
    res["fast"] = fed._fast is not None
    res["active"] = comm.active
    res["calls"] = comm.ipc_calls
    res["params"] = fed.engine.store.params.double().sum(1).tolist()
    res["local"] = fed.local
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown(comm)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,network_size", [(2, 6), (8, 10)], ids=["2ranks", "8ranks"])
def test_ipc_federation_matches_single_process(tmp_path, world, network_size):
    """Two ranks, and the 8-GPU job's 8 ranks (VERDICT r4 Next #4b: the bench's
    10-client federation sharded 2/1/1/1/1/1/1/2... over them), on one GPU
    with --comm ipc: the device protocol's exchange runs on the peer-memory
    kernels and every selection, aggregator, verification decision, metric
    and parameter equals the single-process federation's."""
    from test_device_protocol_gpu import _cfg, _run, _shrink

    out = str(tmp_path)
    mp.start_processes(_fed_worker, args=(world, _port(), out, network_size), nprocs=world, join=True,
                       start_method="spawn")
    _shrink()
    fed, ref = _run(_cfg(os.path.join(out, "single"), save_checkpoints=False, network_size=network_size),
                    "mse_avg", 4)
    ref_params = fed.engine.store.params.double().sum(1).tolist()
    for r in range(world):
        d = json.load(open(os.path.join(out, f"rank{r}.json")))
        assert d["fast"] and d["active"] and d["calls"] >= 2 * 4, d
        assert d["agg"] == ref["agg"] and d["sel"] == ref["sel"] and d["ver"] == ref["ver"]
        for x, y in zip(d["metrics"], ref["metrics"]):
            np.testing.assert_array_equal(np.array(x), np.array(y))
        loc = d["local"]
        assert d["params"] == ref_params[loc[0]:loc[-1] + 1]
