from .layout import DP, HP, ZP, P_PAD, ModelDims, DEFAULT_DIMS, canonical_to_padded, padded_to_canonical
from .reference import ReferenceSAE, init_client_params
