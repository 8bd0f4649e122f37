#!/bin/bash
# Build the committed (HEAD) kernels as libfedmx_hip_head.so next to the
# working-tree library, for a same-box A/B with scripts/ab_train.sh.
set -eu
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive HEAD fedmse_decentralized_amd/ops/csrc | tar -x -C "$TMP"
python - "$ROOT" "$TMP" <<'PY'
import sys
from pathlib import Path
root, tmp = Path(sys.argv[1]), Path(sys.argv[2])
sys.path.insert(0, str(root))
from fedmse_decentralized_amd.ops import build
build.CSRC = tmp / "fedmse_decentralized_amd/ops/csrc"
build.build_hip(force=True, target=build.LIBDIR / "libfedmx_hip_head.so")
print("built", build.LIBDIR / "libfedmx_hip_head.so")
PY
rm -rf "$TMP"
