"""WikiText-2 tokenisation -- the reference's lstm_models/data.py (Dictionary, Corpus)."""
import os
from io import open

import torch


class Dictionary(object):
    def __init__(self):
        self.word2idx = {}
        self.idx2word = []

    def add_word(self, word):
        if word not in self.word2idx:
            self.idx2word.append(word)
            self.word2idx[word] = len(self.idx2word) - 1
        return self.word2idx[word]

    def __len__(self):
        return len(self.idx2word)


class Corpus(object):
    """Vocabulary built from train, valid, test in that order (lstm_models/data.py:20-48);
    the reference snapshot lacks train.txt, so the 33,278-word vocabulary -- and the test
    token ids -- cannot be rebuilt offline."""

    def __init__(self, path):
        self.dictionary = Dictionary()
        self.train = self.tokenize(os.path.join(path, 'train.txt'))
        self.valid = self.tokenize(os.path.join(path, 'valid.txt'))
        self.test = self.tokenize(os.path.join(path, 'test.txt'))

    def tokenize(self, path):
        assert os.path.exists(path), path
        with open(path, 'r', encoding="utf8") as f:
            for line in f:
                for word in line.split() + ['<eos>']:
                    self.dictionary.add_word(word)
        with open(path, 'r', encoding="utf8") as f:
            idss = []
            for line in f:
                ids = [self.dictionary.word2idx[w] for w in line.split() + ['<eos>']]
                idss.append(torch.tensor(ids).type(torch.int64))
        return torch.cat(idss)
