"""WikiText-2 token ids for evaluate_lstm.py (the reference keeps the PyTorch word-LM
example's Dictionary/Corpus in lstm_models/data.py:1-48; this is a separate implementation of
the same contract: one vocabulary over train, valid and test in that order, every line's
words followed by '<eos>', splits as int64 id tensors).

The reference snapshot lacks train.txt (.MISSING_LARGE_BLOBS), so the 33,278-word vocabulary
-- and therefore the test-split ids -- cannot be rebuilt offline; evaluate_lstm.py
--synthetic draws ids from that vocabulary size instead."""
import os

import torch

SPLITS = ("train", "valid", "test")


def _words(path):
    with open(path, "r", encoding="utf8") as f:
        for line in f:
            yield from line.split()
            yield "<eos>"


class Vocabulary(object):
    """word -> id in first-seen order; ``idx2word`` / ``word2idx`` / ``len`` as the example's
    Dictionary exposes them."""

    def __init__(self):
        self.word2idx = {}

    @property
    def idx2word(self):
        return list(self.word2idx)

    def add_word(self, word):
        return self.word2idx.setdefault(word, len(self.word2idx))

    def __len__(self):
        return len(self.word2idx)


class Corpus(object):
    def __init__(self, path):
        files = {s: os.path.join(path, s + ".txt") for s in SPLITS}
        missing = [f for f in files.values() if not os.path.exists(f)]
        if missing:
            raise FileNotFoundError("WikiText-2 split(s) missing: %s" % ", ".join(missing))
        self.dictionary = Vocabulary()
        for s in SPLITS:  # the vocabulary sees every split before any is encoded
            for w in _words(files[s]):
                self.dictionary.add_word(w)
        ids = self.dictionary.word2idx
        for s in SPLITS:
            setattr(self, s, torch.tensor([ids[w] for w in _words(files[s])], dtype=torch.int64))
