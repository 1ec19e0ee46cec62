"""BertConfig — the config ABI of the K3M pretraining step.

Behaviour follows the reference ``BertConfig`` (vilbert_k3m/vilbert_k3m.py:149-308):

* ``BertConfig(int)`` fills the documented defaults (:153-196, :234-276);
* ``BertConfig(path)`` / ``from_json_file`` / ``from_dict`` copy every JSON key verbatim onto
  the instance, unknown keys included (:226-233, :283-296), so
  ``config/bert_base_6layer_6conect.json`` loads unchanged;
* ``from_dict`` first builds ``BertConfig(-1)`` so attributes absent from the JSON keep their
  defaults (e.g. ``margin`` 1.0, ``num_negative_pv`` 4, ``use_image`` True: :189-195);
* the driver then mutates attributes (train_concap_struc.py:198-211).
"""
import copy
import json


_DEFAULTS = dict(
    hidden_size=768,
    num_hidden_layers=12,
    num_attention_heads=12,
    intermediate_size=3072,
    hidden_act="gelu",
    hidden_dropout_prob=0.1,
    attention_probs_dropout_prob=0.1,
    max_position_embeddings=512,
    type_vocab_size=2,
    initializer_range=0.02,
    v_feature_size=2048,
    v_target_size=1601,
    v_hidden_size=768,
    v_num_hidden_layers=3,
    v_num_attention_heads=12,
    v_intermediate_size=3072,
    bi_hidden_size=1024,
    bi_num_attention_heads=16,
    v_attention_probs_dropout_prob=0.1,
    v_hidden_act="gelu",
    v_hidden_dropout_prob=0.1,
    v_initializer_range=0.2,
    v_biattention_id=[0, 1],
    t_biattention_id=[10, 11],
    visual_target=0,
    fast_mode=False,
    fixed_v_layer=0,
    fixed_t_layer=0,
    in_batch_pairs=False,
    fusion_method="mul",
    dynamic_attention=False,
    with_coattention=True,
    objective=0,
    num_negative_image=128,
    num_negative_pv=4,
    margin=1.0,
    model="bert",
    task_specific_tokens=False,
    visualization=False,
    use_image=True,
)


class BertConfig(object):
    """Configuration of the tri-modal K3M model (same constructor contract as the reference)."""

    def __init__(self, vocab_size_or_config_json_file, **kwargs):
        if isinstance(vocab_size_or_config_json_file, str):
            with open(vocab_size_or_config_json_file, "r", encoding="utf-8") as reader:
                json_config = json.loads(reader.read())
            for key, value in json_config.items():
                self.__dict__[key] = value
        elif isinstance(vocab_size_or_config_json_file, int):
            self.vocab_size = vocab_size_or_config_json_file
            for key, value in _DEFAULTS.items():
                setattr(self, key, copy.deepcopy(kwargs.pop(key, value)))
            if kwargs:
                raise TypeError("unexpected BertConfig arguments: %s" % sorted(kwargs))
            assert len(self.v_biattention_id) == len(self.t_biattention_id)
            assert max(self.v_biattention_id) < self.v_num_hidden_layers
            assert max(self.t_biattention_id) < self.num_hidden_layers
        else:
            raise ValueError(
                "First argument must be either a vocabulary size (int)"
                "or the path to a pretrained model config file (str)"
            )

    @classmethod
    def from_dict(cls, json_object):
        config = BertConfig(vocab_size_or_config_json_file=-1)
        for key, value in json_object.items():
            config.__dict__[key] = value
        return config

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, "r", encoding="utf-8") as reader:
            text = reader.read()
        return cls.from_dict(json.loads(text))

    def __repr__(self):
        return str(self.to_json_string())

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n"


def pretrain_config(path, with_coattention=True, if_pre_sampling=1, visual_target=0,
                    dynamic_attention=False, num_negative=255):
    """Load a JSON config and apply the pretraining driver's mutations
    (train_concap_struc.py:184, :198-211)."""
    cfg = BertConfig.from_json_file(path)
    cfg.v_target_size = 1601 if visual_target == 0 else 2048
    cfg.visual_target = visual_target
    cfg.with_coattention = with_coattention
    cfg.dynamic_attention = dynamic_attention
    cfg.if_pre_sampling = if_pre_sampling
    cfg.num_negative = num_negative
    return cfg


def finetune_config(path, loss_type="ce", use_image=True, with_coattention=True, if_pre_sampling=1, visual_target=0,
                    dynamic_attention=False, num_negative_image=255):
    """Load a JSON config and apply the fine-tuning driver's mutations (finetune.py:1307-1322):
    model "roberta" (whose embeddings behave as BERT's — BertEmbeddings.forward ignores the
    position ids RobertaEmbeddings passes, vilbert_k3m.py:361-367, :394-408), loss_type, use_image."""
    cfg = BertConfig.from_json_file(path)
    cfg.v_target_size = 1601 if visual_target == 0 else 2048
    cfg.visual_target = visual_target
    cfg.model = "roberta"
    cfg.use_image = use_image
    cfg.with_coattention = with_coattention
    cfg.dynamic_attention = dynamic_attention
    cfg.if_pre_sampling = if_pre_sampling
    cfg.num_negative_image = num_negative_image
    cfg.loss_type = loss_type
    cfg.task = "item_alignment"
    return cfg
