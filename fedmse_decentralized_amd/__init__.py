"""fedmse_decentralized_amd — MI355X-native decentralised federated anomaly
detection (FedMSE, peer-to-peer variant).

Subpackages: ``models`` (SAE/AE layouts + torch reference), ``ops`` (HIP
kernels for gfx950 + C++ host runtime), ``engine`` (device-resident client
stores, torch/HIP engines), ``protocol`` (selection, election, aggregation,
verification, early stop), ``parallel`` (RCCL/gloo/loopback comm, sharding),
``data``, ``eval``, ``io``, ``utils``.
"""
__version__ = "0.1.0"

# grow the descriptor table while the process is (usually) still
# single-threaded: see io.files.reserve_fd_table
from .io.files import reserve_fd_table as _reserve_fd_table  # noqa: E402

_reserve_fd_table()
