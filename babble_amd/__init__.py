"""babble_amd — MI355X-native batch verifier for Babble's event-ingestion
hot path (SHA-256 of canonical bodies + ECDSA/secp256k1 verification).

The product is libbabbleverify.so (include/babbleverify.h); this package is
its Python host side: ctypes binding (native), SoA batches (batch), the
device handle (verifier) and a mirror of the reference's Go interface
(hashgraph).  synth generates benchmark/test workloads.
"""
from .native import ACCEPT, REF_PANIC, REJECT, REJECT_ERR, BvError, ReferencePanic  # noqa: F401

__all__ = ["ACCEPT", "REJECT", "REJECT_ERR", "REF_PANIC", "BvError", "ReferencePanic"]
