"""Host-side runtime checks that need no GPU (ops/_hiprt.py, ops/build.py)."""
import numpy as np

from fedmse_decentralized_amd.ops import _hiprt


def test_cpu_mapping_check_sees_host_buffers_and_rejects_unmapped(tmp_path):
    buf = np.zeros(1 << 16, dtype=np.uint8)
    addr = buf.ctypes.data
    assert _hiprt._cpu_mapped_rw(addr, buf.nbytes)
    assert not _hiprt._cpu_mapped_rw(0x1000, 64)          # page 1 is never mapped
    # spans made of adjacent mappings are accepted, holes are not
    maps = tmp_path / "maps"
    maps.write_text("10000-20000 rw-p 0 0:0 0\n20000-30000 rw-s 0 0:0 0\n40000-50000 rw-p 0 0:0 0\n"
                    "50000-60000 r--p 0 0:0 0\n")
    assert _hiprt._cpu_mapped_rw(0x18000, 0x10000, str(maps))
    assert not _hiprt._cpu_mapped_rw(0x28000, 0x10000, str(maps))   # hole 30000-40000
    assert not _hiprt._cpu_mapped_rw(0x48000, 0x10000, str(maps))   # read-only tail
    assert not _hiprt._cpu_mapped_rw(0x18000, 16, str(tmp_path / "missing"))
