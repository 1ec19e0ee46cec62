"""``vilbert_k3m.datasets`` (reference vilbert_k3m/datasets/__init__.py): the pretraining loaders
(concept_cap_dataset_struc.py:297, :419) on the native preprocessing + GPU collation path."""
from k3m_amd.loaders import ConceptCapLoaderTrain_struc, ConceptCapLoaderVal_struc  # noqa: F401
from k3m_amd.data import BertPreprocessBatch, K3MPreprocessBatch  # noqa: F401

__all__ = ["ConceptCapLoaderTrain_struc", "ConceptCapLoaderVal_struc", "BertPreprocessBatch", "K3MPreprocessBatch"]
