"""fedmse_decentralized_amd — MI355X-native decentralised federated anomaly
detection (FedMSE, peer-to-peer variant).

Subpackages: ``models`` (SAE/AE layouts + torch reference), ``ops`` (HIP
kernels for gfx950 + C++ host runtime), ``engine`` (device-resident client
stores, torch/HIP engines), ``protocol`` (selection, election, aggregation,
verification, early stop), ``parallel`` (RCCL/gloo/loopback comm, sharding),
``data``, ``eval``, ``io``, ``utils``.
"""
__version__ = "0.1.0"
