"""State / action containers -- the boundary data type of the reference
(utils/fancy_vector.py:7-72).  ``values`` is a float64 ndarray in key order.
The reference also carries CasADi symbols (``syms``); nothing in this build is
symbolic, so ``syms``/``variables`` are the key names."""
from __future__ import annotations

from typing import Union

import numpy as np


class FancyVector:
    _keys: list = []

    def __init__(self, *values, **kw):
        vals = [0.0] * len(self._keys)
        for i, v in enumerate(values):
            vals[i] = v
        for k, v in kw.items():
            vals[self._keys.index(k)] = v
        self._values = np.array(vals, dtype=np.float64)

    @classmethod
    def create(cls, *args, **kwargs):
        return cls(*args, **kwargs)

    @property
    def values(self) -> np.ndarray:
        return self._values

    @property
    def keys(self) -> list:
        return list(self._keys)

    @property
    def syms(self):
        return list(self._keys)

    @property
    def variables(self):
        return list(self._keys)

    @property
    def labels(self):
        return list(self._keys)

    def index(self, key):
        return self._keys.index(key)

    def __getitem__(self, key: Union[int, str]):
        if isinstance(key, str):
            return self.values[self._keys.index(key)]
        return self.values[key]

    def __setitem__(self, key: Union[int, str], value):
        if isinstance(key, str):
            key = self._keys.index(key)
        self.values[key] = value

    def __getattr__(self, k):
        keys = type(self)._keys
        if k in keys:
            return self._values[keys.index(k)]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if k in type(self)._keys:
            self._values[type(self)._keys.index(k)] = v
        else:
            object.__setattr__(self, k, v)

    def __len__(self):
        return len(self._values)

    def __str__(self):
        return str({k: f"{v:.2f}" for k, v in zip(self._keys, self._values)})

    __repr__ = __str__

    def __add__(self, other):
        assert isinstance(other, self.__class__), "You can only sum two same states"
        return self.__class__.create(*(self.values + other.values))
