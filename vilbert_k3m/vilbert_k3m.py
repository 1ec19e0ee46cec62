"""``vilbert_k3m.vilbert_k3m`` (reference vilbert_k3m/vilbert_k3m.py): the config ABI
(BertConfig :149-308), the pretraining model (BertForMultiModalPreTraining_tri_stru :2186-2859) and
the item-alignment model (K3MForItemAlignment :2862-3456), backed by the MI355X engine."""
from k3m_amd.config import BertConfig  # noqa: F401
from k3m_amd.finetune import K3MForItemAlignment  # noqa: F401
from k3m_amd.vilbert_k3m import BertForMultiModalPreTraining_tri_stru  # noqa: F401

__all__ = ["BertConfig", "BertForMultiModalPreTraining_tri_stru", "K3MForItemAlignment"]
