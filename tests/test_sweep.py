"""The reference sweep (main.run_sweep) run concurrently in one process
(--concurrent-combos: every combination's federation built up front, rounds
issued round-robin, one HIP stream + launch rings per federation on the GPU)
gives the sequential sweep's summary and report files."""
import dataclasses
import json
import os
import sys

import pytest

from fedmse_decentralized_amd.config import ExperimentConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _files(root):
    out = {}
    for d, _, fs in os.walk(root):
        for f in fs:
            if f.endswith(".json"):
                p = os.path.join(d, f)
                out[os.path.relpath(p, root)] = open(p).read()
    return out


def _sweep(out, concurrent, **kw):
    import main as driver
    from fedmse_decentralized_amd import federation

    federation._PREP_CACHE.clear()
    cfg = ExperimentConfig(synthetic="nbaiot", network_size=4, num_rounds=3, epoch=1, batch_size=12, output_root=out,
                           log_level="WARNING", compat="fixed", save_checkpoints=False,
                           concurrent_combos=concurrent, **kw)
    return driver.run_sweep(cfg)


@pytest.mark.timeout(600)
def test_concurrent_sweep_matches_sequential_cpu(tmp_path):
    from test_distributed import _shrink

    _shrink()
    a = _sweep(str(tmp_path / "seq"), False, backend="torch", device="cpu")
    b = _sweep(str(tmp_path / "conc"), True, backend="torch", device="cpu")
    assert a == b
    fa, fb = _files(str(tmp_path / "seq")), _files(str(tmp_path / "conc"))
    assert fa == fb and any("training_summary.json" in k for k in fa)


def test_concurrent_sweep_needs_fixed_compat(tmp_path):
    import main as driver

    cfg = ExperimentConfig(synthetic="nbaiot", network_size=4, num_rounds=1, epoch=1, output_root=str(tmp_path),
                           backend="torch", device="cpu", compat="reference", concurrent_combos=True,
                           log_level="WARNING")
    with pytest.raises(SystemExit):
        driver.run_sweep(cfg)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_concurrent_sweep_matches_sequential_hip(tmp_path):
    """Six federations on six private HIP streams of one GPU, interleaved:
    same summary and report files as the sequential device-protocol sweep."""
    from test_device_protocol_gpu import _shrink

    _shrink()
    a = _sweep(str(tmp_path / "seq"), False, backend="hip", device="cuda", global_early_stop=True)
    b = _sweep(str(tmp_path / "conc"), True, backend="hip", device="cuda", global_early_stop=True)
    assert a == b
    assert _files(str(tmp_path / "seq")) == _files(str(tmp_path / "conc"))
