"""Import surface of the reference package ``vilbert_k3m`` (sunzeyeah/K3M) on the MI355X build.

``train_concap_struc.py:25-26`` imports::

    from vilbert_k3m.datasets import ConceptCapLoaderTrain_struc, ConceptCapLoaderVal_struc
    from vilbert_k3m.vilbert_k3m import BertConfig, BertForMultiModalPreTraining_tri_stru

With this repository on ``sys.path`` those lines resolve here, unchanged, to the HIP-kernel model
(k3m_amd/vilbert_k3m.py) and the native/GPU loaders (k3m_amd/loaders.py).
"""
