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
