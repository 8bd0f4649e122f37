"""ArtefactFiles: in-place rewrites / appends leave exactly the bytes a fresh
``open(..., "wb")`` / ``open(..., "a")`` would."""
import os
import pickle

import numpy as np

from fedmse_decentralized_amd.io import checkpoint as ckpt
from fedmse_decentralized_amd.io.files import ArtifactFiles
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS


def test_overwrite_shrink_grow_and_append(tmp_path):
    f = ArtifactFiles(max_open=2)
    p = str(tmp_path / "a" / "x.bin")
    f.overwrite(p, b"0123456789")
    f.overwrite(p, b"abc")                 # shorter: truncated
    assert open(p, "rb").read() == b"abc"
    f.overwrite(p, b"ABCDEFGH")            # longer again
    assert open(p, "rb").read() == b"ABCDEFGH"
    q = str(tmp_path / "r.jsonl")
    for i in range(3):
        f.append(q, f"{i}\n".encode())
    # more paths than max_open: LRU closing keeps the contents right
    for i in range(5):
        f.overwrite(str(tmp_path / f"y{i}"), bytes([i]) * (i + 1))
    f.append(q, b"3\n")
    f.close()
    assert open(q).read() == "0\n1\n2\n3\n"
    for i in range(5):
        assert open(tmp_path / f"y{i}", "rb").read() == bytes([i]) * (i + 1)


def test_cached_artefacts_equal_plain_writes(tmp_path):
    rng = np.random.default_rng(0)
    f = ArtifactFiles()
    a, b = str(tmp_path / "cached"), str(tmp_path / "plain")
    for rnd in range(3):
        canon = rng.normal(size=DEFAULT_DIMS.num_params).astype(np.float32)
        trk = [(float(x), float(x) / 2) for x in rng.normal(size=5 - rnd)]   # shrinking file
        ckpt.save_model_cpt_fast(a, canon, files=f)
        ckpt.save_tracking(a, trk, files=f)
        ckpt.save_model_cpt_fast(b, canon)
        ckpt.save_tracking(b, trk)
        for name in ("model.cpt", "training_tracking.pkl"):
            assert open(os.path.join(a, name), "rb").read() == open(os.path.join(b, name), "rb").read()
    assert pickle.loads(open(os.path.join(a, "training_tracking.pkl"), "rb").read()) == trk
    f.close()


def test_native_pickle_tracking_matches_pickle():
    from fedmse_decentralized_amd.ops import _host

    rng = np.random.default_rng(1)
    for n in (0, 1, 2, 3, 7, 100, 1000):
        trk = [(float(a), float(b)) for a, b in rng.normal(size=(n, 2))]
        if n > 2:
            trk[1] = (float("nan"), float("inf"))
        assert _host.pickle_tracking(trk) == pickle.dumps(trk, protocol=4), n


def test_native_round_writer_matches_python_writers(tmp_path):
    """write_round_artifacts (one native call per round, threads) leaves the
    bytes of save_model_cpt_fast / save_tracking, across rounds in which
    files shrink and grow and some clients do not improve."""
    import torch

    from fedmse_decentralized_amd.models.layout import P_PAD, padded_index

    cidx = padded_index(DEFAULT_DIMS)[0].numpy()
    rng = np.random.default_rng(2)
    f = ArtifactFiles()
    n = 20
    nat = [str(tmp_path / "nat" / f"c{i}") for i in range(n)]
    ref = [str(tmp_path / "ref" / f"c{i}") for i in range(n)]
    for rnd in range(4):
        snap = torch.from_numpy(rng.normal(size=(n + 3, P_PAD)).astype(np.float32))
        rows = rng.permutation(n + 3)[:n]
        improved = [bool(x) for x in rng.integers(0, 2, size=n)] if rnd else [True] * n
        trks = [[(float(a), float(b)) for a, b in rng.normal(size=(int(rng.integers(1, 6)), 2))]
                for _ in range(n)]
        ckpt.write_round_artifacts(f, nat, snap.numpy(), rows, improved, trks, cidx, DEFAULT_DIMS, n_threads=3)
        for j in range(n):
            if improved[j]:
                ckpt.save_model_cpt_fast(ref[j], snap[rows[j]].numpy()[cidx], DEFAULT_DIMS)
            ckpt.save_tracking(ref[j], trks[j])
    f.close()
    for a, b in zip(nat, ref):
        for name in ("model.cpt", "training_tracking.pkl"):
            assert open(os.path.join(a, name), "rb").read() == open(os.path.join(b, name), "rb").read()
    # the reference's own reader gets the state dict back
    import torch as _t

    sd = _t.load(os.path.join(nat[0], "model.cpt"), weights_only=True)
    assert list(sd.keys())[0] == "encoder.encoder_network.0.weight"


def test_native_async_writer_matches_python_writers(tmp_path):
    """NativeCheckpointWriter (C++ thread, tickets) leaves the bytes of
    save_model_cpt_fast / save_tracking; wait(ticket) orders slot reuse."""
    from fedmse_decentralized_amd.io.native_writer import NativeCheckpointWriter
    from fedmse_decentralized_amd.models.layout import P_PAD, padded_index

    cidx = padded_index(DEFAULT_DIMS)[0].numpy()
    rng = np.random.default_rng(5)
    w = NativeCheckpointWriter(DEFAULT_DIMS)
    n = 12
    nat = [str(tmp_path / "nat" / f"c{i}") for i in range(n)]
    ref = [str(tmp_path / "ref" / f"c{i}") for i in range(n)]
    slots = [rng.normal(size=(n + 2, P_PAD)).astype(np.float32) for _ in range(2)]
    tickets = [0, 0]
    for rnd in range(6):
        si = rnd % 2
        if tickets[si]:
            w.wait(tickets[si])
        slots[si][:] = rng.normal(size=slots[si].shape).astype(np.float32)
        rows = rng.permutation(n + 2)[:n]
        improved = [True] * n if rnd == 0 else [bool(x) for x in rng.integers(0, 2, size=n)]
        trks = [[(float(a), float(b)) for a, b in rng.normal(size=(int(rng.integers(1, 6)), 2))] for _ in range(n)]
        for j in range(n):
            if improved[j]:
                ckpt.save_model_cpt_fast(ref[j], slots[si][rows[j]][cidx], DEFAULT_DIMS)
            ckpt.save_tracking(ref[j], trks[j])
        tickets[si] = w.submit(nat, slots[si], rows, improved, trks)
        if rnd == 3:
            # the writer thread releases its descriptors / mappings and
            # reopens the existing files on the next job
            w.flush()
    w.flush()
    for a, b in zip(nat, ref):
        for name in ("model.cpt", "training_tracking.pkl"):
            assert open(os.path.join(a, name), "rb").read() == open(os.path.join(b, name), "rb").read()
    w.close()


def test_fd_table_reserved_by_entry_points_not_by_import():
    """The entry points grow the descriptor table (io.files.reserve_fd_table):
    a descriptor near the top of the reserved range is usable at once.  A
    plain package import changes no process-wide state."""
    import subprocess
    import sys

    code = ("import resource, fedmse_decentralized_amd; "
            "print(resource.getrlimit(resource.RLIMIT_NOFILE)[0])")
    env = dict(os.environ)
    env.pop("FEDMX_RESERVE_FDS", None)
    soft = int(subprocess.run([sys.executable, "-c", "import resource; print(resource.getrlimit(resource.RLIMIT_NOFILE)[0])"],
                              capture_output=True, text=True, env=env).stdout)
    after = int(subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                               cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).stdout)
    assert after == soft
    from fedmse_decentralized_amd.io import files

    top = files.reserve_fd_table()
    assert top >= 256
    fd = os.open(os.devnull, os.O_RDONLY)
    try:
        os.dup2(fd, top - 1)
        os.close(top - 1)
    finally:
        os.close(fd)
