"""Build-owned stand-in for the ``tensorpack`` import of the reference driver (train_concap_struc.py:16).
Only ``tensorpack.dataflow``'s serializer NAMES are used by the driver (the ``serializer=`` loader
argument, :330, :347); the loaders here read record directories / TSVs (k3m_amd/loaders.py), not
tensorpack's LMDB container."""
from . import dataflow  # noqa: F401
