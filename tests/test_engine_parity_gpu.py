"""End-to-end parity (SURVEY §4 tier T4): the same federation run through the
HIP engine on the MI355X and through the plain-PyTorch CPU engine (the
numerical oracle), reference-compat mode (host decisions, the reference's
torch RNG stream replayed).  Selections, elections and verification results
must agree exactly; AUCs and parameters to fp32-trajectory tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fedmse_decentralized_amd.config import ExperimentConfig

from test_device_protocol_gpu import _shrink


def _run(out, backend, device, model_type, update_type, rounds=3):
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    cfg = ExperimentConfig(synthetic="nbaiot", network_size=6, num_rounds=rounds, epoch=2, batch_size=12,
                           output_root=out, backend=backend, device=device, log_level="WARNING",
                           compat="reference", global_early_stop=False, save_checkpoints=False,
                           model_types=[model_type], update_types=[update_type])
    federation._PREP_CACHE.clear()
    fed = Federation(cfg, model_type, update_type, 0).setup()
    assert fed._fast is None          # reference compat: host decisions on both engines
    rs = [fed.run_round() for _ in range(rounds)]
    fed.finish()
    fed.writer.flush()
    if device == "cuda":
        torch.cuda.synchronize()
    return fed, rs


@pytest.mark.parametrize("model_type,update_type", [("hybrid", "mse_avg"), ("autoencoder", "avg"),
                                                    ("hybrid", "fedprox")])
def test_hip_engine_matches_torch_engine(tmp_path, model_type, update_type):
    _shrink()
    fh, rh = _run(str(tmp_path / "hip"), "hip", "cuda", model_type, update_type)
    ft, rt = _run(str(tmp_path / "torch"), "torch", "cpu", model_type, update_type)
    assert fh.engine.name == "hip" and ft.engine.name == "torch"
    for a, b in zip(rh, rt):
        assert a.selected == b.selected
        assert a.aggregator == b.aggregator
        assert a.verification == b.verification
        np.testing.assert_allclose(np.array(a.metrics), np.array(b.metrics), atol=2e-3)
    torch.testing.assert_close(fh.engine.store.params.cpu(), ft.engine.store.params, rtol=2e-2, atol=2e-4)
