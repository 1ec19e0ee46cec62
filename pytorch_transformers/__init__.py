"""Build-owned stand-in for the two ``pytorch_transformers`` (1.1.0) modules the reference driver imports
(train_concap_struc.py:22-23).  pytorch_transformers is not installable offline; these restate the
parts the driver uses so ``train_concap_struc.py`` imports unchanged:

* ``tokenization_bert.BertTokenizer`` — vocab-file WordPiece tokenizer (from a local vocab.txt only:
  names that would need a download raise);
* ``optimization.AdamW`` / ``WarmupLinearSchedule`` — the optimizer and schedule of the fp32 branch
  (:434-448), AdamW stepping through the HIP kernel ``k3m_adamw`` (libk3m_hip.so).
"""
