"""Reference ``bigdl.dataset.movielens`` (P/dataset/movielens.py): MovieLens-1M ratings as an int array
(user, item, rating, timestamp) from ``data_dir/ml-1m/ratings.dat`` (an ``ml-1m.zip`` there is extracted)."""
import os
import zipfile

import numpy as np

from .base import maybe_download

SOURCE_URL = "http://files.grouplens.org/datasets/movielens/"


def read_data_sets(data_dir):
    extracted_to = os.path.join(data_dir, "ml-1m")
    if not os.path.isdir(extracted_to):
        path = maybe_download("ml-1m.zip", data_dir, SOURCE_URL + "ml-1m.zip")
        with zipfile.ZipFile(path) as z:
            z.extractall(data_dir)
    with open(os.path.join(extracted_to, "ratings.dat")) as f:
        rows = [line.strip().split("::") for line in f if line.strip()]
    return np.array(rows).astype(int)


def get_id_pairs(data_dir):
    return read_data_sets(data_dir)[:, 0:2]


def get_id_ratings(data_dir):
    return read_data_sets(data_dir)[:, 0:3]


__all__ = ["read_data_sets", "get_id_pairs", "get_id_ratings"]
