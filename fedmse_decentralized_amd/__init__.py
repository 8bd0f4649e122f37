"""fedmse_decentralized_amd — MI355X-native decentralised federated anomaly
detection (FedMSE, peer-to-peer variant).

Subpackages: ``models`` (SAE/AE layouts + torch reference), ``ops`` (HIP
kernels for gfx950 + C++ host runtime), ``engine`` (device-resident client
stores, torch/HIP engines), ``protocol`` (selection, election, aggregation,
verification, early stop), ``parallel`` (RCCL/gloo/loopback comm, sharding),
``data``, ``eval``, ``io``, ``utils``.
"""
__version__ = "0.1.0"

# The entry points (main.py, bench.py) grow the descriptor table while the
# process is still single-threaded (io.files.reserve_fd_table); a library
# import changes no process-wide state unless FEDMX_RESERVE_FDS=1 asks for it.
import os as _os

if _os.environ.get("FEDMX_RESERVE_FDS") == "1":
    from .io.files import reserve_fd_table as _reserve_fd_table

    _reserve_fd_table()
