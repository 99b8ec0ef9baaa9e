"""Loader for the committed golden fixtures (tests/golden/<set>.{json,bin})."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


class Golden:
    def __init__(self, name):
        with open(os.path.join(GOLDEN, name + '.json')) as f:
            self.manifest = json.load(f)
        with open(os.path.join(GOLDEN, name + '.bin'), 'rb') as f:
            self.blob = f.read()
        self.meta = self.manifest['meta']

    def keys(self):
        return self.manifest['arrays'].keys()

    def __contains__(self, k):
        return k in self.manifest['arrays']

    def __getitem__(self, k):
        a = self.manifest['arrays'][k]
        arr = np.frombuffer(self.blob, dtype='<' + a['dtype'], count=a['nbytes'] // np.dtype(a['dtype']).itemsize,
                            offset=a['offset'])
        return arr.reshape(a['shape']).copy()

    def table(self, prefix):
        return {c: self[prefix + c] for c in self.meta[prefix + 'columns']}
