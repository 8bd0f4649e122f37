"""Time os.open(O_CREAT) of new files in directories created earlier vs just
before, on this host's /tmp (the artefact writer's first-creation cost)."""
import json
import os
import tempfile
import time

root = tempfile.mkdtemp(prefix="fedmx_open_")
dirs = [os.path.join(root, f"a/b/c/Client-{i}") for i in range(64)]
for d in dirs:
    os.makedirs(d)
time.sleep(0.5)
t = []
for d in dirs:
    t0 = time.perf_counter()
    fd = os.open(os.path.join(d, "model.cpt"), os.O_RDWR | os.O_CREAT, 0o644)
    t.append(time.perf_counter() - t0)
    os.close(fd)
t2 = []
for i in range(64):
    d = os.path.join(root, f"x/y/Client-{i}")
    os.makedirs(d)
    t0 = time.perf_counter()
    fd = os.open(os.path.join(d, "model.cpt"), os.O_RDWR | os.O_CREAT, 0o644)
    t2.append(time.perf_counter() - t0)
    os.close(fd)
t3 = []
for d in dirs:
    t0 = time.perf_counter()
    fd = os.open(os.path.join(d, "training_tracking.pkl"), os.O_RDWR | os.O_CREAT, 0o644)
    t3.append(time.perf_counter() - t0)
    os.close(fd)
us = lambda v: round(1e6 * sum(v) / len(v), 1)
print(json.dumps({"open_new_in_old_dir_us": us(t), "open_new_in_fresh_dir_us": us(t2),
                  "second_file_same_dir_us": us(t3), "max_us": round(1e6 * max(t + t2 + t3), 1),
                  "tmp": os.statvfs("/tmp").f_bsize}))
