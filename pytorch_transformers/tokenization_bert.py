"""``pytorch_transformers.tokenization_bert.BertTokenizer`` (1.1.0 API) restated for the offline build.

The published algorithm: a basic tokenizer (clean control characters, pad CJK ideographs with spaces,
lower-case and strip accents when ``do_lower_case``, split on punctuation) followed by greedy
longest-match-first WordPiece over the vocabulary (continuation pieces prefixed ``##``; a word longer
than 100 characters or with no match becomes ``[UNK]``).  The reference driver sets
``do_basic_tokenize = False`` after loading (train_concap_struc.py:220), so only WordPiece runs there.

Only local vocabularies load: ``from_pretrained(path)`` takes a directory holding ``vocab.txt`` or the
vocab file itself.  Model NAMES (``bert-base-chinese`` ...) would be downloaded by the real library;
here they raise ``OSError`` with that explanation (there is no network and no bundled vocab).
"""
import collections
import os
import unicodedata

VOCAB_NAME = "vocab.txt"


def load_vocab(vocab_file):
    vocab = collections.OrderedDict()
    with open(vocab_file, "r", encoding="utf-8") as f:
        for i, line in enumerate(f):
            vocab[line.rstrip("\n")] = i
    return vocab


def whitespace_tokenize(text):
    text = text.strip()
    return text.split() if text else []


def _is_whitespace(ch):
    if ch in (" ", "\t", "\n", "\r"):
        return True
    return unicodedata.category(ch) == "Zs"


def _is_control(ch):
    if ch in ("\t", "\n", "\r"):
        return False
    return unicodedata.category(ch).startswith("C")


def _is_punctuation(ch):
    cp = ord(ch)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return unicodedata.category(ch).startswith("P")


def _is_cjk(cp):
    return (0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0x20000 <= cp <= 0x2A6DF or 0x2A700 <= cp <= 0x2B73F
            or 0x2B740 <= cp <= 0x2B81F or 0x2B820 <= cp <= 0x2CEAF or 0xF900 <= cp <= 0xFAFF
            or 0x2F800 <= cp <= 0x2FA1F)


class BasicTokenizer(object):
    def __init__(self, do_lower_case=True, never_split=None, tokenize_chinese_chars=True):
        self.do_lower_case = do_lower_case
        self.never_split = set(never_split or ())
        self.tokenize_chinese_chars = tokenize_chinese_chars

    def tokenize(self, text, never_split=None):
        never = self.never_split | set(never_split or ())
        out = []
        for ch in text:
            cp = ord(ch)
            if cp == 0 or cp == 0xFFFD or _is_control(ch):
                continue
            if _is_whitespace(ch):
                out.append(" ")
            elif self.tokenize_chinese_chars and _is_cjk(cp):
                out.append(" %s " % ch)
            else:
                out.append(ch)
        tokens = []
        for tok in whitespace_tokenize("".join(out)):
            if self.do_lower_case and tok not in never:
                tok = "".join(c for c in unicodedata.normalize("NFD", tok.lower()) if unicodedata.category(c) != "Mn")
            tokens.extend(self._split_punc(tok, never))
        return whitespace_tokenize(" ".join(tokens))

    @staticmethod
    def _split_punc(tok, never):
        if tok in never:
            return [tok]
        pieces, cur = [], []
        for ch in tok:
            if _is_punctuation(ch):
                if cur:
                    pieces.append("".join(cur))
                    cur = []
                pieces.append(ch)
            else:
                cur.append(ch)
        if cur:
            pieces.append("".join(cur))
        return pieces


class WordpieceTokenizer(object):
    def __init__(self, vocab, unk_token="[UNK]", max_input_chars_per_word=100):
        self.vocab, self.unk_token, self.max_chars = vocab, unk_token, max_input_chars_per_word

    def tokenize(self, text):
        out = []
        for word in whitespace_tokenize(text):
            if len(word) > self.max_chars:
                out.append(self.unk_token)
                continue
            start, pieces, bad = 0, [], False
            while start < len(word):
                end, cur = len(word), None
                while start < end:
                    sub = word[start:end] if start == 0 else "##" + word[start:end]
                    if sub in self.vocab:
                        cur = sub
                        break
                    end -= 1
                if cur is None:
                    bad = True
                    break
                pieces.append(cur)
                start = end
            out.extend([self.unk_token] if bad else pieces)
        return out


class BertTokenizer(object):
    def __init__(self, vocab_file, do_lower_case=True, do_basic_tokenize=True, never_split=None, unk_token="[UNK]",
                 sep_token="[SEP]", pad_token="[PAD]", cls_token="[CLS]", mask_token="[MASK]",
                 tokenize_chinese_chars=True, **kwargs):
        if not os.path.isfile(vocab_file):
            raise OSError("BertTokenizer: vocabulary file %r not found" % vocab_file)
        self.vocab = load_vocab(vocab_file)
        self.ids_to_tokens = collections.OrderedDict((i, t) for t, i in self.vocab.items())
        self.unk_token, self.sep_token, self.pad_token = unk_token, sep_token, pad_token
        self.cls_token, self.mask_token = cls_token, mask_token
        self.all_special_tokens = [unk_token, sep_token, pad_token, cls_token, mask_token]
        self.do_basic_tokenize = do_basic_tokenize
        self.basic_tokenizer = BasicTokenizer(do_lower_case, never_split, tokenize_chinese_chars)
        self.wordpiece_tokenizer = WordpieceTokenizer(self.vocab, unk_token)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, *inputs, **kwargs):
        p = pretrained_model_name_or_path
        if p is None:
            raise OSError("BertTokenizer.from_pretrained(None): pass a directory holding %s or the vocab file "
                          "(train_concap_struc.py --pretrained_model_path)" % VOCAB_NAME)
        vocab_file = os.path.join(p, VOCAB_NAME) if os.path.isdir(p) else p
        if not os.path.isfile(vocab_file):
            raise OSError("BertTokenizer.from_pretrained(%r): no %s there.  Model names are downloaded by the real "
                          "pytorch_transformers; this offline build reads local vocabularies only." % (p, VOCAB_NAME))
        return cls(vocab_file, *inputs, **kwargs)

    def __len__(self):
        return len(self.vocab)

    @property
    def vocab_size(self):
        return len(self.vocab)

    def tokenize(self, text):
        if self.do_basic_tokenize:
            out = []
            for tok in self.basic_tokenizer.tokenize(text, never_split=self.all_special_tokens):
                out.extend(self.wordpiece_tokenizer.tokenize(tok))
            return out
        return self.wordpiece_tokenizer.tokenize(text)

    def convert_tokens_to_ids(self, tokens):
        unk = self.vocab.get(self.unk_token)
        if isinstance(tokens, str):
            return self.vocab.get(tokens, unk)
        return [self.vocab.get(t, unk) for t in tokens]

    def convert_ids_to_tokens(self, ids):
        if isinstance(ids, int):
            return self.ids_to_tokens.get(ids, self.unk_token)
        return [self.ids_to_tokens.get(i, self.unk_token) for i in ids]

    def add_special_tokens_single_sentence(self, token_ids):
        return [self.vocab[self.cls_token]] + list(token_ids) + [self.vocab[self.sep_token]]

    def add_special_tokens_sentences_pair(self, token_ids_0, token_ids_1):
        sep, cls = [self.vocab[self.sep_token]], [self.vocab[self.cls_token]]
        return cls + list(token_ids_0) + sep + list(token_ids_1) + sep

    def encode(self, text, text_pair=None, add_special_tokens=False):
        a = self.convert_tokens_to_ids(self.tokenize(text))
        if text_pair is None:
            return self.add_special_tokens_single_sentence(a) if add_special_tokens else a
        b = self.convert_tokens_to_ids(self.tokenize(text_pair))
        return self.add_special_tokens_sentences_pair(a, b) if add_special_tokens else (a, b)
