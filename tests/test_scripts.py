"""Tooling scripts on CPU: results tables from report files, rocpd profile
summaries (on a synthetic rocpd-shaped database)."""
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


def test_results_table(tmp_path):
    import results_table

    d = tmp_path / "Run_0" / "AUC"
    d.mkdir(parents=True)
    with open(d / "FL-IoT_0.5_hybrid_mse_avg_results.json", "w") as f:
        for r in range(3):
            f.write(json.dumps({"round": r, "client_metrics": [0.9 + 0.01 * r, 0.8], "update_type": "mse_avg",
                                "model_type": "hybrid", "global_loss": 0.8}) + "\n")
    res = results_table.load_results(str(tmp_path))
    t = results_table.table(res, per_round=True)
    assert "| hybrid | mse_avg | 3 | 0.8600 | 0.8000 | 0.9200 |" in t and "99.01" in t


def test_prof_summary_on_synthetic_db(tmp_path):
    import prof_summary

    db = tmp_path / "x.db"
    c = sqlite3.connect(db)
    c.execute("create table kernels (name text, start int, end int, duration int, grid_x int, grid_y int, "
              "workgroup_x int, lds_size int, scratch_size int, vgpr_count int, accum_vgpr_count int, sgpr_count int)")
    t = 0
    for rnd in range(3):
        for name, dur in (("void fedmx::train_kernel<false>(fedmx::TrainArgs)", 1000), ("fedmx::auc_kernel", 60)):
            c.execute("insert into kernels values (?,?,?,?,?,?,?,?,?,?,?,?)",
                      (name, t, t + dur, dur, 1280, 1, 256, 0, 0, 128, 0, 64))
            t += dur + 10
    c.commit()
    s = prof_summary.summarize(str(db), "t")
    assert "fedmx::train_kernel<false>" in s and "one round timeline" in s


def test_bench_stdout_is_one_json_line():
    """The driver contract: `python bench.py ...` prints exactly one JSON line
    on stdout with the BASELINE metric and the required fields (CPU engine,
    one short round)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--backend", "torch", "--steps", "1",
                        "--warmup", "0", "--epochs", "1", "--no-artifacts"], cwd=root, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 1 and rec["warmup"] == 0 and rec["scaling"] == "strong"
    assert rec["config"]["clients"] == 10 and rec["value"] == rec["federation_rounds_per_sec"]
    assert rec["higher_is_better"] is True and rec["value"] > 0
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in rec["config"], k


def test_partition_devices_pipeline(tmp_path):
    """scripts/partition_devices.py: per-device subsample, 40 % test_normal
    holdout, Dirichlet split, reference layout readable by the CSV loader."""
    import numpy as np

    import partition_devices as mod
    rng = np.random.default_rng(0)
    raw = tmp_path / "raw"
    args = []
    for d in range(3):
        (raw / f"dev{d}").mkdir(parents=True)
        hdr = ",".join(f"f{i}" for i in range(115))
        np.savetxt(raw / f"dev{d}" / "benign_traffic.csv", rng.normal(size=(4000, 115)), delimiter=",",
                   header=hdr, comments="")
        np.savetxt(raw / f"dev{d}" / "attack.csv", rng.normal(5, 1, size=(4000, 115)), delimiter=",",
                   header=hdr, comments="")
        args += ["--device", f"dev{d}={raw}/dev{d}/benign_traffic.csv:{raw}/dev{d}/attack*.csv"]
    out = tmp_path / "fed"
    assert mod.main(args + ["--out", str(out), "--clients", "4", "--min-count", "0", "--abnormal-frac", "0.05"]) == 0
    cfg = json.load(open(out / "Configuration" / "federated.json"))
    assert len(cfg["devices_list"]) == 4
    from fedmse_decentralized_amd.data.csv import load_data

    tot = {"normal": 0, "abnormal": 0, "test_normal": 0}
    for dev in cfg["devices_list"]:
        for split in tot:
            arr = load_data(str(out / "Data" / dev[f"{split}_data_path"]))
            assert arr.shape[1] == 115
            tot[split] += arr.shape[0]
    # 5 % of 3 x 4000 benign = 600 (40 % held out), 5 % of 3 x 4000 attack = 600
    assert tot == {"normal": 360, "abnormal": 600, "test_normal": 240}


def test_bench_two_ranks_under_torch_distributed_run():
    """The driver's N > 1 launch (`python -m torch.distributed.run ...
    bench.py --gpus 2`) on CPU with gloo: rank 0 alone prints one JSON line,
    n_gpus = 2, the 10-client federation as the headline, the collectives
    named by backend."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--backend", "torch", "--steps", "1", "--warmup", "0", "--epochs", "1",
                        "--no-artifacts", "--no-extra"], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["clients"] == 10 and rec["value"] > 0
    assert rec["scaling"] == "strong" and "weak_scaling" not in rec
    assert rec["config"]["parallelism"] == "client-sharded x2 (gloo all-gather/all-reduce)"


def _bench_no_launcher(n, *extra):
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--backend", "torch",
                        "--steps", "1", "--warmup", "0", "--epochs", "1", "--no-artifacts", *extra],
                       cwd=root, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus_flag_spawns_ranks_without_a_launcher():
    """`python bench.py --gpus 8` with no torch.distributed.run around it
    starts the 8 rank processes itself (gloo on the CPU here) and prints ONE
    BASELINE-shaped line (VERDICT r3 Next #1): ``value`` is the 10-client
    federation's rounds/s over the 8 ranks (no x N factor), with the
    10N-client weak-scaling federation and N independent one-GPU
    federations as separate fields."""
    rec = _bench_no_launcher(8)
    assert rec["n_gpus"] == 8 and rec["config"]["clients"] == 10 and rec["scaling"] == "strong"
    assert rec["value"] == rec["federation_rounds_per_sec"] > 0
    assert "x2" not in rec["unit"] and "10-client federation" in rec["unit"]
    w = rec["weak_scaling"]
    assert w["clients"] == 80 and w["federation_rounds_per_sec"] > 0 and 0.0 <= w["detection_auc_mean"] <= 1.0
    ind = rec["independent_federations"]
    assert ind["federations"] == 8 and ind["clients_each"] == 10
    assert abs(ind["aggregate_rounds_per_sec"] - 8 * ind["per_federation_rounds_per_sec"]) < 1e-3
    assert 0.0 <= ind["detection_auc_min"] <= ind["detection_auc_mean"] <= 1.0
    # non-overlapping phase telemetry: the phases sum to at most the timed region
    assert sum(rec["phase_ms_total"].values()) <= rec["timed_ms"] * 1.001


def test_bench_clients_per_gpu_headline_is_the_larger_federation():
    """--clients-per-gpu 1 (BASELINE config 3: one client per GPU): the
    headline is that N-client federation's own round rate, labelled weak."""
    rec = _bench_no_launcher(4, "--clients-per-gpu", "1", "--no-extra")
    assert rec["n_gpus"] == 4 and rec["config"]["clients"] == 4 and rec["scaling"] == "weak"
    assert rec["value"] == rec["federation_rounds_per_sec"]


def test_plots_scale_combos_and_tsne(tmp_path):
    """scripts/plots.py (the reference notebooks' figures): AUC-vs-size bars
    from network_scale records, per-combination bars from report files, and
    a latent t-SNE from a --save-latents pickle of a tiny CPU run."""
    import dataclasses

    import plots
    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation

    recs = tmp_path / "s.jsonl"
    with open(recs, "w") as f:
        for n, a in ((10, 0.985), (20, 0.986)):
            f.write(json.dumps({"clients": n, "participation": 0.5, "iid": True, "rounds": 50, "backend": "hip",
                                "init_mode": "shared", "auc_mean_last10": a}) + "\n")
    assert os.path.getsize(plots.plot_sweep([str(recs)], "clients", plots.SCALE_REF, "clients",
                                            str(tmp_path / "scale.png"), "t")) > 1000
    cfg = ExperimentConfig(synthetic="nbaiot", network_size=3, num_rounds=2, epoch=1, output_root=str(tmp_path),
                           backend="torch", device="cpu", compat="fixed", save_checkpoints=False, save_latents=True,
                           global_early_stop=False, log_level="WARNING", model_types=["hybrid"],
                           update_types=["mse_avg"])
    from test_distributed import _shrink

    _shrink()
    fed = Federation(dataclasses.replace(cfg), "hybrid", "mse_avg", 0).setup()
    fed.run_all()
    run_dir = os.path.join(str(tmp_path), "Checkpoint/LatentData/3", cfg.experiment_name, "Run_0")
    out = plots.plot_tsne(run_dir, fed.clients[0].name, str(tmp_path / "tsne.png"))
    assert os.path.getsize(out) > 1000
    out = plots.plot_combos(os.path.join(str(tmp_path), "Checkpoint/Results"), str(tmp_path / "combos.png"))
    assert os.path.getsize(out) > 1000


def test_ab_variant_names_are_unique():
    """A repeated key in scripts/ab_variants.py's table silently replaces the
    earlier variant's flags (round 4: a second "split" entry built a 4-wave
    kernel variant under the helper-wave SPLIT name)."""
    import ast
    import collections

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tree = ast.parse(open(os.path.join(root, "scripts", "ab_variants.py")).read())
    table = next(n.value for n in tree.body if isinstance(n, ast.Assign) and
                 any(getattr(t, "id", None) == "VARIANTS" for t in n.targets))
    keys = [k.value for k in table.keys]
    assert [k for k, c in collections.Counter(keys).items() if c > 1] == []


def test_isa_timeline_on_a_tiny_listing(tmp_path):
    """scripts/isa_timeline.py: a dependent MFMA pair waits 40 cycles, an LDS
    read's consumer waits for lgkmcnt; the loop / barrier plumbing runs."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    import isa_timeline as T

    body = T.parse([
        "\tds_read_b128 v[0:3], v10",
        "\ts_waitcnt lgkmcnt(0)",
        "\tv_mfma_f32_16x16x4_f32 v[4:7], v0, v1, v[4:7]",
        "\tv_mfma_f32_16x16x4_f32 v[4:7], v2, v3, v[4:7]",
        "\tv_add_f32_e32 v8, v4, v5",
    ])
    rows, t = T.simulate(body)
    assert rows[1]["why"] == "lgkmcnt" and rows[1]["stall"] == T.LDS_LAT + T.LDS_B128 - 4
    assert rows[3]["issue"] - rows[2]["issue"] == 40
    assert rows[4]["issue"] - rows[3]["issue"] == 40
    asm = "\n".join(["_Zk:", ".LBB0_1:", "\ts_barrier", "\tv_mfma_f32_16x16x4_f32 v[4:7], v0, v1, v[4:7]",
                     "\ts_barrier", "\tv_add_f32_e32 v8, v4, v5", "\ts_cbranch_scc1 .LBB0_1", ".Lfunc_end0:"])
    lines = asm.split("\n")
    st, en = T.find_kernel(lines, "_Zk")
    lp = T.loops(lines, st, en)
    assert lp and lp[0]["mfma"] == 1 and lp[0]["barriers"] == 2
    ws = T.cosim([T.parse(lines[lp[0]["start"]:lp[0]["end"] + 1])] * 2, ["a", "b"], iters=3)
    assert all(w.iters == 3 for w in ws)
    # no VALU / MFMA co-execution (--mfma-hold 32, profiles/r4_step_isa_timeline.md):
    # the other wave's VALU waits out the whole MFMA
    pair = [T.parse(["\tv_mfma_f32_16x16x4_f32 v[4:7], v0, v1, v[4:7]", "\ts_cbranch_scc1 .LBB0_1"]),
            T.parse(["\tv_add_f32_e32 v9, v10, v11", "\ts_cbranch_scc1 .LBB0_1"])]
    old_hold = T.MFMA_VPORT_HOLD
    try:
        T.MFMA_VPORT_HOLD = 32
        a, b = T.cosim(pair, ["mfma", "valu"], iters=2)
        assert b.stall["vector port (other wave)"] >= 28
    finally:
        T.MFMA_VPORT_HOLD = old_hold


def test_bench_transport_probe_falls_back_when_a_transport_fails():
    """VERDICT r4 Next #4: every rank of a torch.distributed.run job probes the
    requested transport in a child process before touching the GPU, and the
    ranks agree on the first transport that works on all of them.  Here the
    RCCL probe is made to fail (FEDMX_PROBE_FAIL) and the CPU has no
    peer-memory transport, so the job falls back to gloo and says so."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FEDMX_BENCH_PROBE="1", FEDMX_PROBE_FAIL="rccl", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--backend", "torch", "--steps", "1", "--warmup", "0", "--epochs", "1",
                        "--no-artifacts", "--no-extra"], cwd=root, capture_output=True, text=True, timeout=400,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    fb = rec["transport_fallback"]
    assert fb["requested"] == "rccl" and fb["used"] == "gloo" and rec["config"]["transport"] == "gloo"
    assert [f["transport"] for f in fb["failures"]] == ["rccl", "ipc"]
    assert fb["failures"][0]["ranks_failed"] == [0, 1] and fb["failures"][0]["rc"] == 3
    assert "failure injected" in fb["failures"][0]["first_failure_tail"]
    assert rec["n_gpus"] == 2 and rec["value"] > 0


def test_bench_extras_watchdog_prints_the_headline(monkeypatch):
    """a rank stuck in the N > 1 extras must not lose the headline.
    The watchdog fires, rank 0 prints the record marked with
    extra_fields_error, and every rank exits."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # rank 1 sleeps inside the extras (FEDMX_BENCH_TEST_STALL_RANK), rank 0 waits in a collective
    env = dict(os.environ, FEDMX_BENCH_EXTRA_TIMEOUT_S="20", FEDMX_BENCH_TEST_STALL_RANK="1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--backend", "torch", "--steps", "1", "--warmup", "0", "--epochs", "1",
                        "--no-artifacts"], cwd=root, capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert "did not finish" in rec["extra_fields_error"] and rec["value"] > 0


def test_every_script_is_referenced():
    """VERDICT r4 Next #6: every tracked file under scripts/ is named by the
    README, a test, the package, or profiles/INDEX.md (which describes each
    one); anything nothing names is clutter and goes to git history."""
    import glob
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["git", "ls-files", "scripts"], cwd=root, capture_output=True, text=True)
    tracked = [f for f in r.stdout.split() if f] if r.returncode == 0 else \
        [os.path.relpath(p, root) for p in glob.glob(os.path.join(root, "scripts", "**", "*.*"), recursive=True)
         if "__pycache__" not in p]
    texts = []
    for pat in ("README.md", "profiles/INDEX.md", "tests/*.py", "fedmse_decentralized_amd/**/*.py", "bench.py",
                "main.py", "__graft_entry__.py"):
        for p in glob.glob(os.path.join(root, pat), recursive=True):
            texts.append(open(p, errors="replace").read())
    blob = "\n".join(texts)
    unreferenced = [f for f in tracked if f not in blob and os.path.basename(f) not in blob]
    assert unreferenced == [], unreferenced
    # and the index describes every script it lists as present
    index = open(os.path.join(root, "profiles", "INDEX.md")).read()
    assert all(f"`{f}`" in index for f in tracked), [f for f in tracked if f"`{f}`" not in index]
