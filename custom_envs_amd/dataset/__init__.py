"""Host-side dataset container (custom_envs/dataset/inmemorydataset.py:8-38).

The engine stages ``features``/``targets`` into HBM once at construction;
batching and shuffling then happen on the device (the reset permutation and
the first-B-rows minibatch of optimize.py:64,73).  This class only carries
the arrays and the reference's ``Sequence`` surface for callers that use it
directly.
"""
from collections import namedtuple

import numpy as np

BatchType = namedtuple('BatchType', ['features', 'labels'])


class InMemoryDataSet:
    def __init__(self, features, targets, batch_size=None):
        if len(features) != len(targets):
            raise ValueError('features and targets differ in length')
        self.features = np.asarray(features)
        self.targets = np.asarray(targets)
        self.batch_size = len(self.features) if batch_size is None else int(batch_size)

    def on_epoch_end(self, np_random=np.random):
        index = np.arange(len(self.features))
        np_random.shuffle(index)
        self.features, self.targets = self.features[index], self.targets[index]

    shuffle = on_epoch_end  # optimize.py:64 calls it under this name

    def __len__(self):
        return -(-len(self.features) // self.batch_size)

    def __getitem__(self, idx):
        begin = idx * self.batch_size
        end = begin + self.batch_size if idx < len(self) else None
        return BatchType(self.features[begin:end], self.targets[begin:end])

    @property
    def feature_shape(self):
        return self.features.shape[1:]

    @property
    def target_shape(self):
        return self.targets.shape[1:]

    label_shape = target_shape

    @property
    def labels(self):
        return self.targets


DataSet = InMemoryDataSet
