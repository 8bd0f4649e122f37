"""Cost of the FIRST write of a client's artefact files on this host's
filesystem: new-file mapping (ftruncate + mmap + template copy) vs pwrite."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedmse_decentralized_amd.io import checkpoint as ck  # noqa: E402
from fedmse_decentralized_amd.io.files import ArtifactFiles  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS  # noqa: E402

tpl = ck._template(DEFAULT_DIMS)
out = {}
for mode in ("mapped", "pwrite", "makedirs_only"):
    root = tempfile.mkdtemp(prefix=f"fedmx_fw_{mode}_")
    f = ArtifactFiles(max_open=1 << 20)
    t0 = time.perf_counter()
    for i in range(64):
        d = os.path.join(root, f"Checkpoint/10/exp/0/ClientModel/FL-IoT/hybrid/mse_avg/Client-{i}")
        os.makedirs(d, exist_ok=True)
        if mode == "mapped":
            f.mapped(os.path.join(d, "model.cpt"), tpl.blob_bytes)
        elif mode == "pwrite":
            f.overwrite(os.path.join(d, "model.cpt"), tpl.blob_bytes)
    out[f"{mode}_us_per_client"] = round((time.perf_counter() - t0) / 64 * 1e6, 1)
    t0 = time.perf_counter()
    if mode == "mapped":
        import ctypes
        for (addr, size) in list(f._maps.values()):
            ctypes.memmove(addr + 1000, b"x" * 20000, 20000)
        out["mapped_second_touch_us_per_client"] = round((time.perf_counter() - t0) / 64 * 1e6, 1)
    f.close()
print(json.dumps(out))
