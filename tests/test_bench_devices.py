"""bench.py reports the GPUs a job actually ran on (VERDICT r5 Next #4b).

A one-GPU rehearsal runs several ranks on one device; its record must not
read as a multi-GPU result: ``n_gpus`` is the number of distinct physical
devices among the ranks (the collective self-test's device identities,
``parallel/launch.collective_self_test``), and the rank count goes to
``world_size``."""
import importlib.util
import os
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_distinct_devices_counts_shared_gpus_once():
    b = _bench()
    one = types.SimpleNamespace(world_size=1)
    assert b.distinct_devices(one) == 1
    shared = types.SimpleNamespace(world_size=8, peer_devices=[("host", "GPU-aaaa")] * 8)
    assert b.distinct_devices(shared) == 1
    node = types.SimpleNamespace(world_size=8, peer_devices=[("host", f"GPU-{i}") for i in range(8)])
    assert b.distinct_devices(node) == 8
    pairs = types.SimpleNamespace(world_size=4, peer_devices=[("host", "GPU-0"), ("host", "GPU-0"),
                                                              ("host", "GPU-1"), ("host", "GPU-1")])
    assert b.distinct_devices(pairs) == 2


def test_distinct_devices_without_self_test_asks_the_ranks():
    b = _bench()
    calls = []

    class FakeComm:
        world_size = 2
        device = types.SimpleNamespace(type="cpu")

        def all_gather_object(self, obj):
            calls.append(obj)
            return [("host", "GPU-7"), ("host", "GPU-7")]

    assert b.distinct_devices(FakeComm()) == 1
    assert len(calls) == 1
