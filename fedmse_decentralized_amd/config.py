"""Experiment configuration.

Same knobs, names and defaults as the module constants of the reference
driver (`src/main.py:37-71`), plus the protocol constants that the
reference hard-codes in ``ClientTrainer``/``ModelVerifier``
(`src/Trainer/client_trainer.py:47-95`, `src/Trainer/model_verifier.py:14`)
and the new framework's own switches (backend, compat mode, sharding,
synthetic data).  Every field can be overridden from the command line
(``main.py --help``).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional

DEFAULT_EXP_TEMPLATE = (
    "nonIID_Exp21_Rerun_{epoch}epoch_10client_lr0001_lamda{shrink_lambda}_ratio{ratio}"
)


@dataclass
class ExperimentConfig:
    # --- reference constants (src/main.py:37-71) --------------------------
    num_participants: float = 0.5
    epoch: int = 5
    num_rounds: int = 3
    lr_rate: float = 1e-3
    shrink_lambda: float = 5
    network_size: int = 10
    data_seed: int = 1234
    no_exp: Optional[str] = None
    verification_method: str = "val"     # "val" | "dev"
    num_runs: int = 1
    batch_size: int = 12
    new_device: bool = True
    global_patience: int = 1
    metric: str = "AUC"                  # "AUC" | "classification" | "time"
    model_types: List[str] = field(default_factory=lambda: ["hybrid", "autoencoder"])
    update_types: List[str] = field(default_factory=lambda: ["avg", "fedprox", "mse_avg"])
    dim_features: int = 115
    scen_name: str = "FL-IoT"
    config_file: str = "Configuration/kitsune-iot-10clients.json"
    # --- ClientTrainer / ModelVerifier constants --------------------------
    hidden_neus: int = 27
    latent_dim: int = 7
    fedprox_mu: float = 0.001
    verification_threshold: float = 3.0
    performance_threshold: float = 0.002
    # > 0 (fixed-mode option, not the reference): the verifier's drift limit is
    #   RELATIVE, drift <= drift_threshold_rel x sum_tensors ||history||_2,
    #   instead of the absolute verification_threshold.  The absolute 3.0
    #   (model_verifier.py:72-75) was tuned for the reference's 10 clients;
    #   a large federation's early aggregates move further and were rejected
    #   by nearly every receiver (profiles/r4_adoption_ablation.md).
    drift_threshold_rel: float = 0.0
    max_aggregation: int = 3
    max_rejected_updates: int = 3
    vote_batch_size: int = 128
    scaler: str = "standard"
    # --- new-framework switches -------------------------------------------
    compat: str = "reference"            # "reference" (reproduce quirks) | "fixed"
    backend: str = "auto"                # "auto" | "hip" | "torch"
    device: str = "auto"                 # "auto" | "cpu" | "cuda"
    synthetic: Optional[str] = None      # None (CSV via config_file) | "nbaiot" | "kitsune"
    synthetic_iid: bool = True
    synthetic_alpha: Optional[float] = None
    synthetic_seed: int = 2025
    output_root: str = "."
    save_checkpoints: bool = True        # model.cpt / training_tracking.pkl per client
    save_latents: bool = False           # LatentData pickles
    global_early_stop: bool = True
    trace_file: Optional[str] = None     # per-phase JSONL telemetry
    resume: Optional[str] = None         # resume snapshot path
    snapshot_every: int = 0              # write a resume snapshot every k rounds (0 = never)
    log_level: str = "INFO"
    malicious_clients: List[int] = field(default_factory=list)  # fault injection (tests)
    malicious_scale: float = 10.0
    dropped_clients: List[int] = field(default_factory=list)    # fault injection: never vote / aggregate
    # --- protocol variants ---------------------------------------------------
    # "first_voter": the reference's decentralised election (first selected
    #   voter that finds an eligible candidate decides, client_trainer.py:249-285);
    # "majority": the legacy centralised GlobalAggregator.select_aggregator
    #   (every selected client votes, most votes wins).
    election: str = "first_voter"
    # "decentralized": receivers verify the broadcast aggregate (reference);
    # "centralized": server push, every client adopts the aggregate (legacy
    #   GlobalAggregator.update);
    # "local": ablation, no aggregation at all (selected clients train, every
    #   client is evaluated; profiles/r4_adoption_ablation.md).
    aggregation_mode: str = "decentralized"
    # "code": ModelVerifier rule (drift <= 3.0 and dperf >= -0.002);
    # "thesis": the thesis variant (Thesis p.20-26): loss-ratio acceptance
    #   new <= old * (1 + thesis_loss_ratio) with a NaN/inf check, candidates
    #   with vote MSE > thesis_vote_mse_cap are not voted for, and a random
    #   eligible aggregator is used when no valid one exists.
    protocol_variant: str = "code"
    thesis_loss_ratio: float = 0.1
    thesis_vote_mse_cap: float = 3.0
    # initial client models: "per_client" builds one independently initialised
    #   model per client (the reference, src/main.py:228-236); "shared" gives
    #   every client a copy of client 0's initial model (one global init, as
    #   the FedMSE paper's server does).  "auto": per_client under
    #   compat=reference, shared under compat=fixed — averaging k independent
    #   inits cancels the latent layer by ~sqrt(k), which large federations
    #   never recover from (profiles/r3_collapse_diag.md).
    init_mode: str = "auto"
    fusion_max_rows: int = 1024          # dev rows used by the fusion_avg KDE similarity
    fedavg_sample_weighted: bool = False  # FedAvg weights ∝ training-set size (reference: plain mean, Q13)
    # experiment-level parallelism: with N ranks, combination
    # i of the model_type x update_type x run sweep runs on rank i % N (each
    # as a single-rank federation on that rank's GPU) instead of every
    # combination being sharded over all ranks.
    parallel_combos: bool = False
    # one process, one GPU: build every combination's federation up front and
    # run their rounds interleaved, each federation on its own HIP stream and
    # launch rings (ops/_hip.Runtime(private=True)), so their kernels overlap
    # on the GPU's idle CUs and one federation's host work overlaps another's
    # GPU work.  compat=fixed only (the reference's global early-stop state is
    # shared across combinations in sequence); reports and the
    # summary are identical to the sequential sweep.
    concurrent_combos: bool = False
    # fixed compat + HIP engine: run the round's protocol decisions on the
    # device (engine/device_round.py) so rounds need no host synchronisation
    device_protocol: bool = True
    # debug: all-gather a hash of the replicated protocol state every round
    # and fail on divergence between ranks
    debug_replica_check: bool = False
    # multi-rank transport of the device protocol's per-round collectives:
    # "rccl" (torch.distributed: RCCL on the GPU) or "ipc" (one-shot kernels
    # over peer-mapped memory, parallel/ipc.py; SURVEY §5.8's --comm ipc|rccl);
    # None: FEDMX_COMM, else rccl
    comm: Optional[str] = None

    # -----------------------------------------------------------------------
    @property
    def experiment_name(self) -> str:
        if self.no_exp:
            return self.no_exp
        return DEFAULT_EXP_TEMPLATE.format(
            epoch=self.epoch, shrink_lambda=_fmt_num(self.shrink_lambda), ratio=self.num_participants * 100,
            network_size=self.network_size, num_rounds=self.num_rounds, lr_rate=self.lr_rate,
            data_seed=self.data_seed)

    @property
    def checkpoint_dir(self) -> str:
        return os.path.join(self.output_root, f"Checkpoint/Results/Update/{self.network_size}/{self.experiment_name}")

    def client_save_dir(self, run: int, model_type: str, update_type: str, device_name: str) -> str:
        return os.path.join(self.output_root, f"Checkpoint/{self.network_size}/{self.experiment_name}/{run}/ClientModel",
                            self.scen_name, model_type, update_type, device_name)

    def __post_init__(self):
        # fixed-mode-only options (the reference's rules otherwise): the
        # relative drift rule replaces model_verifier.py:72-75's absolute 3.0
        if self.drift_threshold_rel > 0 and self.compat != "fixed":
            raise ValueError("drift_threshold_rel > 0 replaces the reference's absolute drift rule "
                             "(src/Trainer/model_verifier.py:72-75): it needs compat='fixed'")

    def resolved_init_mode(self) -> str:
        if self.init_mode == "auto":
            return "per_client" if self.compat == "reference" else "shared"
        if self.init_mode not in ("per_client", "shared"):
            raise ValueError(f"init_mode must be auto | per_client | shared, got {self.init_mode!r}")
        return self.init_mode

    def resolved_device(self) -> str:
        if self.device == "auto":
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        return self.device

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=2, sort_keys=True)


def _fmt_num(v):
    # the reference formats shrink_lambda as an int literal (5, 10)
    if isinstance(v, float) and v.is_integer():
        return int(v)
    return v


def _str2bool(s):
    if isinstance(s, bool):
        return s
    return s.lower() in ("1", "true", "yes", "y", "on")


def add_arguments(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    d = ExperimentConfig()
    for f in dataclasses.fields(ExperimentConfig):
        name = "--" + f.name.replace("_", "-")
        default = getattr(d, f.name)
        if isinstance(default, bool):
            p.add_argument(name, type=_str2bool, default=None, metavar="BOOL")
        elif isinstance(default, list):
            elem = int if f.name in ("malicious_clients", "dropped_clients") else str
            p.add_argument(name, type=elem, nargs="*", default=None)
        elif isinstance(default, int) and not isinstance(default, bool):
            p.add_argument(name, type=int, default=None)
        elif isinstance(default, float):
            p.add_argument(name, type=float, default=None)
        elif default is None and str(f.type) in ("Optional[float]", "float"):   # e.g. synthetic_alpha
            p.add_argument(name, type=float, default=None)
        elif default is None and str(f.type) in ("Optional[int]", "int"):
            p.add_argument(name, type=int, default=None)
        else:
            p.add_argument(name, type=str, default=None)
    # reference spelling alias
    p.add_argument("--no-Exp", dest="no_exp", type=str, default=None)
    return p


def from_args(ns: argparse.Namespace, base: Optional[ExperimentConfig] = None) -> ExperimentConfig:
    cfg = base or ExperimentConfig()
    kw = {}
    for f in dataclasses.fields(ExperimentConfig):
        v = getattr(ns, f.name, None)
        if v is not None:
            kw[f.name] = v
    return dataclasses.replace(cfg, **kw)


# --- device-list JSON (src/Configuration/*.json) ---------------------------

@dataclass
class DeviceEntry:
    id: int
    name: str
    normal_data_path: str
    abnormal_data_path: str
    test_normal_data_path: Optional[str] = None


@dataclass
class DeviceListConfig:
    data_path: str
    devices_list: List[DeviceEntry]
    base_dir: str = "."

    def resolve(self, rel: str) -> str:
        p = os.path.join(self.data_path, rel)
        if not os.path.isabs(p):
            p = os.path.join(self.base_dir, p)
        return os.path.normpath(p)


def load_device_list(path: str, base_dir: Optional[str] = None) -> DeviceListConfig:
    """Load a reference device-list JSON verbatim.

    ``data_path`` is relative to the directory the reference is run from
    (``src/``); by default it is resolved relative to the JSON's parent's
    parent (``src/Configuration/x.json`` -> ``src/``), which reproduces that.
    """
    with open(path, "r") as f:
        raw = json.load(f)
    if base_dir is None:
        base_dir = os.path.dirname(os.path.dirname(os.path.abspath(path)))
    devs = []
    for d in raw["devices_list"]:
        devs.append(DeviceEntry(
            id=int(d.get("id", len(devs) + 1)), name=d["name"],
            normal_data_path=d["normal_data_path"], abnormal_data_path=d["abnormal_data_path"],
            test_normal_data_path=d.get("test_normal_data_path")))
    return DeviceListConfig(data_path=raw["data_path"], devices_list=devs, base_dir=base_dir)
