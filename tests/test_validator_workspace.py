"""Host-side bookkeeping of asynchronous validation (CPU, no GPU).

``TrainBuffers.validator_workspace`` decides whether a training launch gets
validator workgroups (fedmx_train_hw.hip: one per client beside its trainer,
grid 2k) and which launch number stamps its flags.  The kernel side is
covered by tests/test_async_validation_gpu.py; this pins the rules it relies
on: the workspace is allocated once and zeroed, a launch with more clients
than slots runs synchronously, and the launch number is never 0 (zeroed
flags must never match a waiting workgroup).
"""
import types

import torch

from fedmse_decentralized_amd.ops import _hip

SLOT = 16   # floats per client slot (the real size comes from fedmx_train_av_slot())


def _bufs(monkeypatch, cus):
    monkeypatch.setattr(torch.cuda, "get_device_properties",
                        lambda dev: types.SimpleNamespace(multi_processor_count=cus))
    monkeypatch.setattr(_hip, "lib", lambda: types.SimpleNamespace(fedmx_train_av_slot=lambda: SLOT))
    b = _hip.TrainBuffers.__new__(_hip.TrainBuffers)   # (no device buffers needed here)
    b.dev = torch.device("cpu")
    b.vws = None
    b.vseq = 0
    return b


def test_slots_bounded_by_half_the_cus(monkeypatch):
    b = _bufs(monkeypatch, cus=8)
    ptr, seq = b.validator_workspace(4, n_rows=10)
    assert b.vslots == 4                       # a validator per client needs 2k <= CUs
    assert ptr == b.vws.data_ptr() and seq == 1
    assert b.vws.numel() == 4 * SLOT and not bool(b.vws.any())
    assert b.validator_workspace(5, n_rows=10) == (None, 0)   # too many clients: synchronous tail
    ptr2, seq2 = b.validator_workspace(3, n_rows=10)
    assert ptr2 == ptr and seq2 == 2           # allocated once, a new number per launch


def test_slots_bounded_by_store_rows(monkeypatch):
    b = _bufs(monkeypatch, cus=256)
    assert b.validator_workspace(2, n_rows=3)[1] == 1
    assert b.vslots == 3
    assert b.validator_workspace(4, n_rows=3) == (None, 0)


def test_launch_number_wraps_past_zero(monkeypatch):
    b = _bufs(monkeypatch, cus=8)
    b.validator_workspace(1, n_rows=4)
    b.vseq = 0xFFFFFFFE
    assert b.validator_workspace(1, n_rows=4)[1] == 0xFFFFFFFF
    assert b.validator_workspace(1, n_rows=4)[1] == 1   # never 0


def test_ranks_sharing_a_device_get_no_validators(monkeypatch):
    """ranks that share one GPU compete for its CUs, so a trainer's
    validator may never be dispatched beside it; such launches keep the
    synchronous epoch tail."""
    assert not _hip.ranks_share_device({}, device_count=1)
    assert not _hip.ranks_share_device({"WORLD_SIZE": "1"}, device_count=1)
    assert _hip.ranks_share_device({"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}, device_count=1)
    assert not _hip.ranks_share_device({"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}, device_count=8)
    assert _hip.ranks_share_device({"WORLD_SIZE": "2", "FEDMX_DEVICE_INDEX": "0"}, device_count=8)
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("FEDMX_DEVICE_INDEX", "0")
    b = _bufs(monkeypatch, cus=256)
    assert b.validator_workspace(2, n_rows=10) == (None, 0)
