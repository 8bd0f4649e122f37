"""Checkpoint artefacts and resume snapshots.

Reference artefacts (written byte-compatible):

* ``model.cpt`` — legacy (non-zip) torch serialisation of the 8-tensor state
  dict, written by ``torch.save(..., _use_new_zipfile_serialization=False)``
  on every validation improvement (`src/Trainer/client_trainer.py:337-350`,
  SURVEY B.4).  The fused training kernel keeps a device-side best snapshot,
  so the file is written once per client per round with the same content
  the reference's last ``save_model`` call produced.
* ``training_tracking.pkl`` — pickle protocol 4 of ``[(train_loss,
  valid_loss), ...]`` (`:416`, `:419`, B.4b).
* ``latent_hybrid_{update}.pkl`` — ``{round: {device: (latent f32 [n, d],
  labels f32 [n])}}`` consumed by `src/Visualization/latent_visualization.ipynb`
  (B.5; the writer is absent from the reference snapshot).

New: ``save_resume``/``load_resume`` — a per-round snapshot of every hosted
client's device state plus the replicated protocol state and RNG states.
It only holds tensors and plain containers, so it loads with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
import pickle
import time
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from ..models.layout import ModelDims, DEFAULT_DIMS, canonical_to_state_dict, padded_to_canonical


class _CptTemplate:
    """Byte template of a legacy ``torch.save`` of the 8-tensor state dict.

    The legacy format is a few pickles followed by each storage's raw bytes;
    for a fixed tensor structure only those raw bytes change.  The template is
    produced once by ``torch.save`` itself (tensors filled with distinct
    marker values, located afterwards), and every ``model.cpt`` is then the
    template with the parameter bytes patched in — one buffer write, no
    pickling, negligible GIL time in the background writer.  Storage keys are
    fixed, so equal parameters give byte-identical files.
    """

    def __init__(self, dims: ModelDims):
        import io as _io

        from collections import OrderedDict

        self.dims = dims
        shapes = dims.shapes()
        markers = []
        state = OrderedDict()
        for t, (k, s) in enumerate(shapes):
            v = np.float32(1234.5 + 17.25 * t)
            markers.append(v)
            state[k] = torch.full(s, float(v), dtype=torch.float32)
        state._metadata = _state_metadata()
        bio = _io.BytesIO()
        torch.save(state, bio, _use_new_zipfile_serialization=False)
        self.blob = bytearray(bio.getvalue())
        self.regions = []
        off = 0
        for (k, s), v in zip(shapes, markers):
            n = int(np.prod(s))
            pat = np.full(n, v, dtype=np.float32).tobytes()
            pos = self.blob.find(pat)
            if pos < 0 or self.blob.find(pat, pos + 1) >= 0 and n > 1:
                raise RuntimeError("could not locate tensor bytes in the legacy checkpoint template")
            self.regions.append((pos, n, off))
            off += n

    def render(self, canonical: np.ndarray) -> bytes:
        buf = bytearray(self.blob)
        c = np.ascontiguousarray(canonical, dtype=np.float32)
        for pos, n, off in self.regions:
            buf[pos:pos + 4 * n] = c[off:off + n].tobytes()
        return bytes(buf)


_TEMPLATES = {}


def _state_metadata():
    from collections import OrderedDict

    meta = OrderedDict()
    for prefix in ("", "encoder", "encoder.encoder_network", "encoder.encoder_network.0",
                   "encoder.encoder_network.1", "encoder.encoder_network.2", "decoder",
                   "decoder.decoder_network", "decoder.decoder_network.0", "decoder.decoder_network.1",
                   "decoder.decoder_network.2"):
        meta[prefix] = {"version": 1}
    return meta


def save_model_cpt_fast(save_dir: str, canonical: np.ndarray, dims: ModelDims = DEFAULT_DIMS,
                        files=None) -> str:
    """``model.cpt`` from a canonical parameter vector via the byte template
    (``files``: an ``io.files.ArtifactFiles`` cache — rewrite in place)."""
    tpl = _TEMPLATES.get(dims)
    if tpl is None:
        tpl = _TEMPLATES[dims] = _CptTemplate(dims)
    path = os.path.join(save_dir, "model.cpt")
    if files is not None:
        files.overwrite(path, tpl.render(canonical))
        return path
    os.makedirs(save_dir, exist_ok=True)
    with open(path, "wb") as f:
        f.write(tpl.render(canonical))
    return path


def _template(dims: ModelDims) -> "_CptTemplate":
    tpl = _TEMPLATES.get(dims)
    if tpl is None:
        tpl = _TEMPLATES[dims] = _CptTemplate(dims)
    if not hasattr(tpl, "np_blob"):
        tpl.blob_bytes = bytes(tpl.blob)
        tpl.np_blob = np.frombuffer(tpl.blob_bytes, dtype=np.uint8)
        tpl.np_regions = np.ascontiguousarray(np.asarray(tpl.regions, dtype=np.int64).reshape(-1, 3))
    return tpl


_PATHS: Dict[str, Tuple[str, str]] = {}
# FEDMX_WRITER_STATS=1: seconds spent preparing / inside the native writer
WRITE_STATS = {} if os.environ.get("FEDMX_WRITER_STATS") == "1" else None


def _artifact_paths(save_dir: str) -> Tuple[str, str]:
    p = _PATHS.get(save_dir)
    if p is None:
        p = _PATHS[save_dir] = (os.path.join(save_dir, "model.cpt"), os.path.join(save_dir, "training_tracking.pkl"))
    return p


def write_round_artifacts(files, save_dirs: Sequence[str], snap: np.ndarray, rows: Sequence[int],
                          improved: Sequence[bool], tracking: Sequence[Sequence[Tuple[float, float]]],
                          canon_idx: np.ndarray, dims: ModelDims = DEFAULT_DIMS, n_threads: int = 0) -> None:
    """Every trained client's ``model.cpt`` (when its validation improved) and
    ``training_tracking.pkl`` for one round, in ONE native call
    (``ops/csrc/host/fedmx_artifacts.cpp``: template patch + exact protocol-4
    pickle + pwrite into cached descriptors, on a few threads, GIL released).
    The bytes are those of ``save_model_cpt_fast`` / ``save_tracking``; a
    job the native path cannot render (> 1000 tracked epochs) falls back to
    them.  ``snap`` is the padded host snapshot [rows, P_PAD] fp32."""
    from ..ops import _host

    n = len(save_dirs)
    if n == 0:
        return
    t0 = time.perf_counter() if WRITE_STATS is not None else 0.0
    c0 = time.thread_time() if WRITE_STATS is not None else 0.0
    tpl = _template(dims)
    cpt_paths, trk_paths = zip(*[_artifact_paths(d) for d in save_dirs])
    # model.cpt: fixed-size files kept mapped (template bytes written once);
    # tracking pickles: cached descriptors
    cpt_dst = np.asarray([files.mapped(p, tpl.blob_bytes) if improved[j] else 0
                          for j, p in enumerate(cpt_paths)], dtype=np.int64)
    fd_trk = np.asarray([files.open_overwrite(p, 2 * n) for p in trk_paths], dtype=np.int32)
    size_trk = np.asarray([files.size_of(p) for p in trk_paths], dtype=np.int64)
    lens = np.asarray([len(t) for t in tracking], dtype=np.int32)
    trk = np.zeros((n, max(1, int(lens.max(initial=0))), 2), dtype=np.float64)
    for j, t in enumerate(tracking):
        if len(t):
            trk[j, :len(t)] = np.asarray(t, dtype=np.float64).reshape(-1, 2)
    if n_threads <= 0:
        n_threads = 1   # page-cache copies + small pwrites: threads measured no faster
    snap = np.ascontiguousarray(snap, dtype=np.float32)
    t1 = time.perf_counter() if WRITE_STATS is not None else 0.0
    c1 = time.thread_time() if WRITE_STATS is not None else 0.0
    status = _host.write_artifacts(snap, np.ascontiguousarray(canon_idx, dtype=np.int32), tpl.np_blob,
                                   tpl.np_regions, np.asarray(rows, dtype=np.int32),
                                   np.asarray(improved, dtype=np.int32), cpt_dst, fd_trk, size_trk,
                                   trk, lens, n_threads)
    if WRITE_STATS is not None:
        t2 = time.perf_counter()
        WRITE_STATS["prep"] = WRITE_STATS.get("prep", 0.0) + (t1 - t0)
        WRITE_STATS["native"] = WRITE_STATS.get("native", 0.0) + (t2 - t1)
        WRITE_STATS["calls"] = WRITE_STATS.get("calls", 0) + 1
        WRITE_STATS["prep_cpu"] = WRITE_STATS.get("prep_cpu", 0.0) + (c1 - c0)
    for j in range(n):
        files.set_size(trk_paths[j], size_trk[j])
        if status[j] == -1:      # too many epochs for the native pickler
            if improved[j]:
                save_model_cpt_fast(save_dirs[j], snap[rows[j]][canon_idx], dims, files=files)
            save_tracking(save_dirs[j], tracking[j], files=files)
        elif status[j] != 0:
            raise OSError(-int(status[j]), f"writing the artefacts of {save_dirs[j]}")


def save_model_cpt(save_dir: str, padded_params: torch.Tensor, dims: ModelDims = DEFAULT_DIMS) -> str:
    os.makedirs(save_dir, exist_ok=True)
    flat = padded_to_canonical(padded_params.detach().float().cpu(), dims)
    sd = canonical_to_state_dict(flat, dims)
    # the reference saves nn.Module.state_dict(): OrderedDict with per-module _metadata
    from collections import OrderedDict

    state = OrderedDict(sd)
    meta = OrderedDict()
    for prefix in ("", "encoder", "encoder.encoder_network", "encoder.encoder_network.0",
                   "encoder.encoder_network.1", "encoder.encoder_network.2", "decoder",
                   "decoder.decoder_network", "decoder.decoder_network.0", "decoder.decoder_network.1",
                   "decoder.decoder_network.2"):
        meta[prefix] = {"version": 1}
    state._metadata = meta
    path = os.path.join(save_dir, "model.cpt")
    torch.save(state, path, _use_new_zipfile_serialization=False)
    return path


def save_tracking(save_dir: str, tracking: Sequence[Tuple[float, float]], files=None) -> str:
    path = os.path.join(save_dir, "training_tracking.pkl")
    blob = pickle.dumps([(float(a), float(b)) for a, b in tracking], protocol=4)
    if files is not None:
        files.overwrite(path, blob)
        return path
    os.makedirs(save_dir, exist_ok=True)
    with open(path, "wb") as f:
        f.write(blob)
    return path


def save_latents(path: str, data: Dict[int, Dict[str, Tuple[np.ndarray, np.ndarray]]]) -> str:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        pickle.dump(data, f, protocol=4)
    return path


def save_resume(path: str, payload: Dict) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)
    return path


def load_resume(path: str) -> Dict:
    return torch.load(path, map_location="cpu", weights_only=True)
