"""Partner (mplc/partner.py:14-35): one data owner of a scenario.

Besides the reference's fields (id, x_train, y_train, batch_size, ...), a partner records train_idx,
its row indices into dataset.x_train, so the engine can keep one copy of the data in HBM and gather
batches by index instead of copying arrays per partner (mplc/scenario.py:636-637).
"""
import numpy as np


class Partner:
    def __init__(self, partner_id, **kwargs):
        self.id = partner_id
        self.batch_size = kwargs.get("batch_size", 0)
        self.x_train = kwargs.get("x_train", None)
        self.x_val = kwargs.get("x_val", None)
        self.x_test = kwargs.get("x_test", None)
        self.y_train = kwargs.get("y_train", None)
        self.y_val = kwargs.get("y_val", None)
        self.y_test = kwargs.get("y_test", None)
        self.train_idx = kwargs.get("train_idx", None)
        self.final_nb_samples = 0
        self.clusters_list = []

    @property
    def num_labels(self):
        return self.y_train.shape[1] if self.y_train is not None and np.ndim(self.y_train) == 2 else 0
