"""Build A/B variants of the HIP library from patched copies of the kernel
sources (the production sources carry no experiment switches since round 6).

    python scripts/ab_build.py NAME [NAME ...]     # -> ops/lib/libfedmx_hip_NAME.so
    bash scripts/ab_train.sh                        # (GPU box) times them, AB_LIBS="main NAME ..."

Each variant is a list of (file, exact old text, new text) substitutions
applied to a temporary copy of ``ops/csrc/hip``; a substitution whose old
text is missing fails the build (a stale variant never times the production
kernel by accident).
"""
from __future__ import annotations

import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from fedmse_decentralized_amd.ops import build  # noqa: E402

HW = "fedmx_train_hw.hip"


def _mask(name, old, new):
    return (HW, f"constexpr int {name} = {old};", f"constexpr int {name} = {new};")


VARIANTS = {
    # per-instantiation masks (bit 0 plain, 1 FedProx, 2 batch > 12): r6 re-check
    # of the r5 choice on the round-6 code
    "bu7vm7": [_mask("BIAS_UNITS", 6, 7), _mask("VALUE_MASKS", 6, 7)],
    "pp7": [_mask("PINGPONG", 5, 7)],
    "all7": [_mask("BIAS_UNITS", 6, 7), _mask("VALUE_MASKS", 6, 7), _mask("PINGPONG", 5, 7)],
    "w4flag3": [_mask("W4FLAG_ROLES", 2, 3)],
    "av3": [("fedmx_train_hw.hip", "constexpr int ASYNC_VALID = 1;", "constexpr int ASYNC_VALID = 3;")],
    # FedProx with asynchronous validation and without the W4 LDS-flag hand-off
    "av3nf": [("fedmx_train_hw.hip", "constexpr int ASYNC_VALID = 1;", "constexpr int ASYNC_VALID = 3;"),
              _mask("W4FLAG_ROLES", 2, 0)],
    "nf": [_mask("W4FLAG_ROLES", 2, 0)],
    # the decision check two steps earlier (round 5 measured step 4 slower; the
    # round-6 publication is faster: stamps put the decision ~3 steps after it)
    "avc4": [_mask("AV_CHECK", 6, 4)],
    "avc4st": [_mask("AV_CHECK", 6, 4)],   # (stamped, below: the decision timeline at step 4)
    "stamps": [],   # (built with -DFEDMX_STAMPS=1 below)
    # round-6 compiler-scheduler sweep: the production sources, other
    # machine-scheduler settings (no numerics change: bit-identical results)
    "s_ilp": [], "s_iterilp": [], "s_nounclust": [], "s_trackers": [], "s_bias0": [], "s_relaxed": [],
    "s_agpr": [], "s_o2": [], "s_exact": [], "s_nocluster": [], "s_bias100": [],
    "m_pre_td": [], "m_pre_bu": [], "m_post_td": [], "m_post_bu": [], "m_nopost": [], "m_nocyclic": [],
    "m_norp": [],
    # FedProx with asynchronous validation, memory clustering off
    "av3_nocluster": [("fedmx_train_hw.hip", "constexpr int ASYNC_VALID = 1;", "constexpr int ASYNC_VALID = 3;")],
}
FLAGS = {"stamps": ["-DFEDMX_STAMPS=1"], "avc4st": ["-DFEDMX_STAMPS=1"],
         "s_ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
         "s_iterilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
         "s_nounclust": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"],
         "s_trackers": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
         "s_bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
         "s_relaxed": ["-mllvm", "-amdgpu-schedule-relaxed-occupancy"],
         "s_agpr": ["-mllvm", "-amdgpu-mfma-vgpr-form=0"],   # (the last -mllvm setting wins)
         "s_o2": ["-O2"],
         "s_exact": ["-mllvm", "-amdgpu-igrouplp-exact-solver"],
         "s_nocluster": ["-mllvm", "-misched-cluster=false"],
         "s_bias100": ["-mllvm", "-amdgpu-schedule-metric-bias=100"],
         "av3_nocluster": ["-mllvm", "-misched-cluster=false"],
         "m_pre_td": ["-mllvm", "-misched-prera-direction=topdown"],
         "m_pre_bu": ["-mllvm", "-misched-prera-direction=bottomup"],
         "m_post_td": ["-mllvm", "-misched-postra-direction=topdown"],
         "m_post_bu": ["-mllvm", "-misched-postra-direction=bottomup"],
         "m_nopost": ["-mllvm", "-enable-post-misched=false"],
         "m_nocyclic": ["-mllvm", "-misched-cyclicpath=false"],
         "m_norp": ["-mllvm", "-misched-regpressure=false"]}


def build_variant(name: str) -> Path:
    subs = VARIANTS[name]
    src = build.CSRC / "hip"
    with tempfile.TemporaryDirectory() as td:
        dst = Path(td) / "hip"
        shutil.copytree(src, dst)
        for fname, old, new in subs:
            p = dst / fname
            text = p.read_text()
            if text.count(old) != 1:
                raise SystemExit(f"variant {name}: {fname} has {text.count(old)} copies of {old!r}")
            p.write_text(text.replace(old, new))
        target = build.LIBDIR / f"libfedmx_hip_{name}.so"
        base = build._hip_flags(FLAGS.get(name, []))
        flags = [*base[:3], "-fPIC", "-shared", *base[3:]]
        # the library's own per-source flags too (build.SOURCE_FLAGS), so a
        # variant differs from production only by its substitutions / FLAGS
        for cmd in build.hip_link_commands(sorted(dst.glob("*.hip")), flags, dst, target):
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            if r.returncode != 0:
                raise SystemExit(f"variant {name} failed:\n{r.stdout[-3000:]}")
        for o in target.parent.glob(f"{target.name}.*.o"):
            o.unlink()
    return target


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print("built", build_variant(n))
