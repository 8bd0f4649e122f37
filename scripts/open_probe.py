"""Time os.open(O_CREAT) of new files on this host's /tmp (the artefact
writer's first-creation cost) under the conditions of a bench process:
descriptors held open (--hold), idle threads (--threads N), a GPU held
(--gpu), directories created just before or long before."""
import json
import os
import sys
import tempfile
import threading
import time

if "--reserve" in sys.argv:
    # the package's fix: grow the descriptor table before any thread exists
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fedmse_decentralized_amd.io.files import reserve_fd_table

    reserve_fd_table()
if "--gpu" in sys.argv:
    # same measurement from a process holding the GPU (like the bench)
    import torch

    _keep = torch.empty(1 << 30, device="cuda")
    torch.cuda.synchronize()
n_thr = int(sys.argv[sys.argv.index("--threads") + 1]) if "--threads" in sys.argv else 0
stop = threading.Event()
ths = [threading.Thread(target=stop.wait) for _ in range(n_thr)]
for t in ths:
    t.start()
hold = "--hold" in sys.argv
root = tempfile.mkdtemp(prefix="fedmx_open_")
us = lambda v: round(1e6 * sum(v) / max(1, len(v)), 1)
held = []


def create(paths):
    t = []
    for p in paths:
        t0 = time.perf_counter()
        fd = os.open(p, os.O_RDWR | os.O_CREAT, 0o644)
        t.append(time.perf_counter() - t0)
        if hold:
            held.append(fd)
        else:
            os.close(fd)
    return t


dirs = [os.path.join(root, f"a/b/c/Client-{i}") for i in range(128)]
for d in dirs:
    os.makedirs(d)
time.sleep(0.2)
t1 = create([os.path.join(d, "model.cpt") for d in dirs])
t2 = create([os.path.join(d, "training_tracking.pkl") for d in dirs])
t3 = []
for i in range(64):
    d = os.path.join(root, f"x/y/Client-{i}")
    os.makedirs(d)
    t3 += create([os.path.join(d, "model.cpt")])
t4 = []   # existing files reopened
for d in dirs[:64]:
    t0 = time.perf_counter()
    fd = os.open(os.path.join(d, "model.cpt"), os.O_RDWR)
    t4.append(time.perf_counter() - t0)
    os.close(fd)
stop.set()
for t in ths:
    t.join()
print(json.dumps({"gpu": "--gpu" in sys.argv, "hold": hold, "reserve": "--reserve" in sys.argv, "threads": n_thr,
                  "new_in_old_dir_us_by_32": [us(t1[i:i + 32]) for i in range(0, len(t1), 32)],
                  "second_file_us_by_32": [us(t2[i:i + 32]) for i in range(0, len(t2), 32)],
                  "new_in_fresh_dir_us": us(t3), "reopen_existing_us": us(t4),
                  "max_us": round(1e6 * max(t1 + t2 + t3), 1)}))
